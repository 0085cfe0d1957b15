"""The C-ABI library loads without a GPU and exports exactly what include/wscodec.h declares."""
import ctypes as C
import os
import re

import pytest

from netman_amd import codec as K

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "wscodec.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(wsc_\w+)\s*\(", src, flags=re.M)))


def test_every_declared_symbol_is_exported(codec_lib):
    decl = declared_functions()
    assert len(decl) >= 20
    for name in decl:
        assert hasattr(codec_lib, name), name
    assert set(decl) == set(K.SIGNATURES), set(decl) ^ set(K.SIGNATURES)


def test_struct_sizes_match_header(codec_lib):
    assert C.sizeof(K.WscConfig) == 56
    assert C.sizeof(K.WscBatch) == 96
    assert C.sizeof(K.WscEvent) == 40
    assert C.sizeof(K.WscConnState) == 40 and K.CONN_STATE_DTYPE.itemsize == 40
    assert K.FRAME_DTYPE.itemsize == 32 and K.SEG_RESULT_DTYPE.itemsize == 32


def test_config_default_and_version(codec_lib):
    assert codec_lib.wsc_abi_version() == K.ABI_VERSION == 5
    cfg = K.default_config()
    assert cfg.max_frame_len == (1 << 40) - 1 and cfg.unmask_window == 4096
    assert cfg.walk_mode == 0 and cfg.u8_inline_max == 256 and cfg.walk_flags == 0


def test_no_silent_cpu_fallback(codec_lib):
    """without a gfx950 device the product path fails loudly"""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(K.WscError) as ei:
        K.Codec(0)
    assert ei.value.rc in (K.WSC_E_NODEVICE, K.WSC_E_DEVICE)


def test_library_is_gfx950_code_object():
    so = open(os.path.join(ROOT, "netman_amd", "libwscodec.so"), "rb").read()
    assert b"gfx950" in so


def test_library_reads_no_environment():
    """round-5 VERDICT: a deployment's environment must never change results -- the shipped library
    imports no getenv and carries no A/B knob names (variants are config fields, session flags, or
    tools/build_variant.sh builds)"""
    so = open(os.path.join(ROOT, "netman_amd", "libwscodec.so"), "rb").read()
    assert b"getenv" not in so
    assert b"WSC_AB_" not in so
