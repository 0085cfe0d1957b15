"""Batched server -> client framing (wsc_encode) against the oracle's restatement of
websocketProtocol.encode (server/websocket_ctrl.go:23-70).

CPU tests pin the oracle: the RFC 6455 §5.7 unmasked example frames held in
tests/golden/rfc6455_kat.json are exactly what encode(firstByte, payload) must produce (the
reference sends unmasked server frames), plus the 7/16/64-bit length boundaries against an
independent struct-based restatement.  GPU tests compare the HIP framer with the oracle
byte-for-byte on seeded batches (edge lengths, unaligned sources, many tiny frames per output
window, frames larger than a window) and check the out_cap contract.
"""
import json
import os
import struct

import numpy as np
import pytest

import oracle_ref as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KAT = {k["name"]: k for k in json.load(open(os.path.join(ROOT, "tests", "golden", "rfc6455_kat.json")))}


def ref_encode_struct(first_byte, payload):
    """independent restatement (struct) of websocket_ctrl.go:23-70, used to cross-check the oracle"""
    n = len(payload)
    if n <= 125:
        h = struct.pack(">BB", first_byte, n)
    elif n <= 65535:
        h = struct.pack(">BBH", first_byte, 126, n)
    else:
        h = struct.pack(">BBQ", first_byte, 127, n)
    return h + payload


# ---- CPU: the oracle is pinned by the RFC fixtures --------------------------------------------
def test_oracle_encode_rfc_unmasked_text():
    k = KAT["rfc_single_unmasked_text"]          # RFC 6455 §5.7: 0x81 0x05 "Hello"
    assert O.encode(0x81, b"Hello").hex() == k["hex"]


def test_oracle_encode_rfc_unmasked_ping():
    k = KAT["rfc_unmasked_ping"]                 # 0x89 0x05 "Hello"
    assert O.encode(0x89, b"Hello").hex() == k["hex"]


@pytest.mark.parametrize("name,size", [("rfc_256B_unmasked_binary_header", 256),
                                       ("rfc_64KiB_unmasked_binary_header", 65536)])
def test_oracle_encode_rfc_binary_headers(name, size):
    k = KAT[name]
    payload = bytes(k.get("pad_zeros", 0))
    assert len(payload) == size
    out = O.encode(0x82, payload)
    assert out.hex() == k["hex"] + "00" * size


@pytest.mark.parametrize("n", [0, 1, 124, 125, 126, 127, 65534, 65535, 65536, 65537, 1 << 20])
def test_oracle_encode_length_boundaries(n):
    payload = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    for fb in (0x81, 0x82, 0x8A, 0x88):
        assert O.encode(fb, payload) == ref_encode_struct(fb, payload)


def test_oracle_encode_batch_is_concatenation():
    rng = np.random.default_rng(5)
    src = rng.integers(0, 256, 300000, dtype=np.uint8)
    lens = np.array([0, 5, 125, 126, 70000, 3, 65535, 65536], np.uint64)
    offs = rng.integers(0, 300000 - 70000, len(lens)).astype(np.uint64)
    fbs = np.array([0x81, 0x82, 0x8A, 0x82, 0x82, 0x88, 0x81, 0x82], np.uint8)
    out, off = O.encode_batch(src, offs, lens, fbs)
    exp = b"".join(ref_encode_struct(int(f), src[int(o):int(o) + int(n)].tobytes()) for f, o, n in zip(fbs, offs, lens))
    assert out.tobytes() == exp
    assert int(off[-1]) == len(exp)


# ---- GPU: the HIP framer vs the oracle --------------------------------------------------------
def _batch(seed, n, len_choices, src_bytes=None, p=None):
    rng = np.random.default_rng(seed)
    lens = rng.choice(np.array(len_choices, np.uint64), size=n, p=p)
    src_bytes = src_bytes or int(lens.max()) * 2 + 4096
    src = rng.integers(0, 256, src_bytes, dtype=np.uint8)
    offs = np.array([rng.integers(0, src_bytes - int(L) + 1) for L in lens], np.uint64)
    fbs = rng.choice(np.array([0x81, 0x82, 0x8A, 0x88], np.uint8), size=n)
    msgs = np.zeros(n, O_MSG())
    msgs["src_off"], msgs["len"], msgs["first_byte"] = offs, lens, fbs
    return msgs, src


def O_MSG():
    from netman_amd import codec as K
    return K.OUT_MSG_DTYPE


def _check(c, msgs, src):
    out, off = c.encode_host(msgs, src)
    exp, eoff = O.encode_batch(src, msgs["src_off"], msgs["len"], msgs["first_byte"])
    assert np.array_equal(off, eoff)
    assert out.tobytes() == exp.tobytes()


@pytest.fixture(scope="module")
def codec(codec_lib):
    from netman_amd import codec as K
    c = K.Codec(0, max_batch_bytes=64 << 20, max_segs=1024, max_frames=1 << 18)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_encode_edge_lengths(codec, seed):
    lens = [0, 1, 2, 3, 15, 16, 17, 124, 125, 126, 127, 1000, 4095, 4096, 4097, 65535, 65536, 65537]
    msgs, src = _batch(100 + seed, 700, lens)
    _check(codec, msgs, src)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_gpu_encode_small_and_large_mix(codec, seed):
    """small and large frames mixed in one batch (windows holding frame edges of every kind),
    then another batch in the same context"""
    lens = [0, 1, 9, 15, 16, 100, 1000, 1024, 3999, 4000, 4001, 4005, 4096, 9000, 70000]
    msgs, src = _batch(200 + seed, 3000, lens)
    _check(codec, msgs, src)
    msgs, src = _batch(300 + seed, 5000, [1, 17, 1000, 4000])
    _check(codec, msgs, src)


@pytest.mark.gpu
def test_gpu_encode_many_tiny_frames_per_window(codec):
    msgs, src = _batch(7, 50000, [0, 1, 5, 17, 60, 125], src_bytes=1 << 16)
    _check(codec, msgs, src)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [65536, 65537, 262144, 262145, 300000])
def test_gpu_encode_scan_widths(codec_lib, n):
    """the scan's messages per thread change with the batch (1 up to 64 Ki messages, 4 up to
    256 Ki, 16 beyond: wsc_api.cpp enc_scan_ipt); each width, at its boundaries, equals the oracle"""
    from netman_amd import codec as K
    c = K.Codec(0, max_batch_bytes=64 << 20, max_segs=1024, max_frames=1 << 19)
    try:
        msgs, src = _batch(11 + n, n, [0, 3, 40, 125, 126, 300], src_bytes=1 << 16)
        _check(c, msgs, src)
    finally:
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("src_bytes", [1, 7, 15, 16, 17, 40, 4096])
def test_gpu_encode_gathers_at_the_ends_of_src(codec, src_bytes):
    """the copy's one-round-trip window (encode_window_direct) reads plain 16-byte pieces only when
    every gather of the window lies inside src, else the window takes the two-pass path: sources
    shorter than 16 bytes, and messages starting at src byte 0 or ending at its last byte (their
    pieces' 16-byte reads cross the ends of src), equal the oracle either way"""
    from netman_amd import codec as K
    rng = np.random.default_rng(5000 + src_bytes)
    src = rng.integers(0, 256, src_bytes, dtype=np.uint8)
    n = 3000
    lens = rng.integers(0, src_bytes + 1, n).astype(np.uint64)
    at = rng.integers(0, 3, n)   # 0: from src byte 0, 1: ending at its last byte, 2: anywhere
    offs = np.where(at == 0, 0, np.where(at == 1, src_bytes - lens,
                                         [rng.integers(0, src_bytes - int(L) + 1) for L in lens])).astype(np.uint64)
    msgs = np.zeros(n, K.OUT_MSG_DTYPE)
    msgs["src_off"], msgs["len"] = offs, lens
    msgs["first_byte"] = rng.choice(np.array([0x81, 0x82], np.uint8), size=n)
    _check(codec, msgs, src)


@pytest.mark.gpu
def test_gpu_encode_large_frames(codec):
    msgs, src = _batch(8, 24, [1 << 20, (1 << 20) + 3, 3 * 65536 + 7, 131], src_bytes=8 << 20)
    _check(codec, msgs, src)


@pytest.mark.gpu
def test_gpu_encode_single_and_empty(codec):
    from netman_amd import codec as K
    msgs = np.zeros(1, K.OUT_MSG_DTYPE)
    msgs["first_byte"] = 0x81
    msgs["len"] = 5
    out, off = codec.encode_host(msgs, np.frombuffer(b"Hello" + bytes(11), np.uint8))
    assert out.tobytes().hex() == KAT["rfc_single_unmasked_text"]["hex"]
    out, off = codec.encode_host(np.zeros(0, K.OUT_MSG_DTYPE), np.zeros(16, np.uint8))
    assert len(out) == 0 and int(off[0]) == 0


@pytest.mark.gpu
def test_gpu_encode_out_cap_too_small(codec):
    from netman_amd import codec as K
    msgs, src = _batch(9, 100, [1000])
    need = int(msgs["len"].sum()) + 4 * 100
    with pytest.raises(K.WscError) as ei:
        codec.encode_host(msgs, src, out_cap=need - 1)
    assert ei.value.rc == K.WSC_E_CAPACITY
    out, off = codec.encode_host(msgs, src, out_cap=need)   # exactly enough
    assert int(off[-1]) == need


@pytest.mark.gpu
def test_gpu_encode_device_resident_never_writes_past_total(codec):
    """device API: bytes between the total and out_cap are left untouched (tail pieces use byte
    stores), and a second encode into the same buffer is identical (look-back state re-armed)"""
    import torch
    msgs, src = _batch(10, 3000, [0, 7, 125, 126, 5000, 65536])
    exp, eoff = O.encode_batch(src, msgs["src_off"], msgs["len"], msgs["first_byte"])
    dev = torch.device("cuda:0")
    d_msgs = torch.from_numpy(msgs.view(np.uint8).copy()).to(dev)
    d_src = torch.from_numpy(src).to(dev)
    cap = len(exp) + 8192
    d_out = torch.full((cap,), 0xEE, dtype=torch.uint8, device=dev)
    d_off = torch.zeros(len(msgs) + 1, dtype=torch.int64, device=dev)
    for _ in range(2):
        codec.encode(d_msgs, len(msgs), d_src, len(src), d_out, cap, d_off)
        torch.cuda.synchronize()
        out = d_out.cpu().numpy()
        assert int(d_off[-1].item()) == len(exp)
        assert out[: len(exp)].tobytes() == exp.tobytes()
        assert (out[len(exp):] == 0xEE).all()
