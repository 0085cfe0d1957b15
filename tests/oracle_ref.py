"""ctypes access to the CPU oracle (oracle/_build/libwsoracle.so) -- test infrastructure.

The oracle restates netman's Go decode path (see oracle/ws_oracle.h).  Only tests/, smoke() and
bench.py's cpu_baseline leg use it, as the checker.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "_build", "libwsoracle.so")
GOPORT = os.path.join(ORACLE_DIR, "_build", "libgoport.so")

EV_MESSAGE, EV_PONG, EV_CLOSE, EV_STALL = 1, 2, 3, 4


class WsoEvent(C.Structure):
    _fields_ = [("type", C.c_uint32), ("msg_id", C.c_uint32), ("opcode", C.c_uint32),
                ("close_code", C.c_uint32), ("err", C.c_uint32), ("pad", C.c_uint32),
                ("data_off", C.c_uint64), ("data_len", C.c_uint64)]


FRAME_DTYPE = np.dtype([("hdr_off", "<u8"), ("payload_off", "<u8"), ("payload_len", "<u8"),
                        ("mask", "<u4"), ("msg_id", "<u4"), ("opcode", "u1"), ("fin", "u1"),
                        ("kind", "u1"), ("mode", "u1"), ("err", "<u4")])


class WsoResult(C.Structure):
    _fields_ = [("consumed", C.c_uint64), ("closed", C.c_uint32), ("stalled", C.c_uint32),
                ("close_code", C.c_uint32), ("err", C.c_uint32), ("msg_id", C.c_uint32),
                ("message_mode", C.c_uint32), ("cont_len", C.c_uint64), ("n_events", C.c_uint32),
                ("n_frames", C.c_uint32), ("arena_used", C.c_uint64), ("overflow", C.c_uint32),
                ("pad", C.c_uint32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
        _lib = C.CDLL(LIB)
        _lib.wso_run.restype = C.c_int
        _lib.wso_run.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_uint64,
                                 C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                 C.c_void_p, C.c_uint64, C.POINTER(WsoResult)]
        _lib.wso_run_ex.restype = C.c_int
        _lib.wso_run_ex.argtypes = _lib.wso_run.argtypes + [C.c_uint32]
        _lib.wso_utf8_valid.restype = C.c_int
        _lib.wso_utf8_valid.argtypes = [C.c_void_p, C.c_uint64]
        _lib.wso_encode.restype = C.c_uint64
        _lib.wso_encode.argtypes = [C.c_uint8, C.c_void_p, C.c_uint64, C.c_void_p]
        _lib.wso_encode_batch.restype = C.c_uint64
        _lib.wso_encode_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                          C.c_void_p, C.c_void_p]
    return _lib


@dataclass
class Ev:
    type: int
    msg_id: int = 0
    opcode: int = 0
    close_code: int = 0
    err: int = 0
    data: bytes = b""

    def key(self):
        return (self.type, self.msg_id, self.opcode, self.close_code, self.err, self.data)


@dataclass
class OracleOut:
    events: list
    frames: np.ndarray
    inplace: bytes
    res: dict = field(default_factory=dict)


MAX_FRAME_LEN = (1 << 40) - 1   # wsc_config_default's max_frame_len (the 40-bit record, Q4)


def run(stream: bytes, chunk_ends=None, max_frame_len=MAX_FRAME_LEN, cap=None, eof=False) -> OracleOut:
    """cap: room for that many events / frame log lines (default: enough for any stream of
    this length -- n / 2; pass a bound for streams of a few large frames).
    eof: the peer closes after the stream (a read returns 0 -> io.EOF -> Close(), epoll.go:108-110)"""
    L = lib()
    s = np.frombuffer(stream, dtype=np.uint8) if stream else np.zeros(1, np.uint8)
    n = len(stream)
    inplace = np.zeros(max(n, 1), np.uint8)
    ev_cap = (n // 2 + 16) if cap is None else int(cap)
    fr_cap = ev_cap
    ev = (WsoEvent * ev_cap)()
    fr = np.zeros(fr_cap, FRAME_DTYPE)
    arena = np.zeros(n + 16, np.uint8)
    res = WsoResult()
    ce = None
    nc = 0
    if chunk_ends is not None:
        ce = np.ascontiguousarray(chunk_ends, dtype=np.uint64)
        nc = len(ce)
    rc = L.wso_run_ex(s.ctypes.data, n, ce.ctypes.data if ce is not None else None, nc, max_frame_len,
                      inplace.ctypes.data, C.cast(ev, C.c_void_p), ev_cap, fr.ctypes.data, fr_cap,
                      arena.ctypes.data, len(arena), C.byref(res), 1 if eof else 0)
    assert rc == 0, "oracle output overflow"
    events = []
    for i in range(res.n_events):
        e = ev[i]
        data = bytes(arena[e.data_off:e.data_off + e.data_len]) if e.type in (EV_MESSAGE, EV_PONG) else b""
        events.append(Ev(e.type, e.msg_id, e.opcode, e.close_code, e.err, data))
    r = {k: getattr(res, k) for k, _ in WsoResult._fields_}
    return OracleOut(events, fr[:res.n_frames].copy(), bytes(inplace[:n]), r)


def utf8_valid(b: bytes) -> bool:
    a = np.frombuffer(b, dtype=np.uint8) if b else np.zeros(1, np.uint8)
    return bool(lib().wso_utf8_valid(a.ctypes.data, len(b)))


_goport = None


def goport():
    global _goport
    if _goport is None:
        if not os.path.exists(GOPORT):
            subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
        _goport = C.CDLL(GOPORT)
        for fn in (_goport.goport_unmask_frames, _goport.goport_unmask_frames_mt):
            fn.restype = C.c_uint64
        _goport.goport_unmask_frames.argtypes = [C.c_void_p] * 4 + [C.c_uint64]
        _goport.goport_unmask_frames_mt.argtypes = [C.c_void_p] * 4 + [C.c_uint64, C.c_int]
    return _goport


def encode(first_byte: int, payload: bytes) -> bytes:
    """websocket_ctrl.go:23-70 encode(firstByte, bs), restated in oracle/ws_oracle.c"""
    out = (C.c_uint8 * (len(payload) + 10))()
    src = (C.c_uint8 * max(1, len(payload))).from_buffer_copy(payload or b"\0")
    n = lib().wso_encode(first_byte, src, len(payload), out)
    return bytes(out[:n])


def encode_batch(src: np.ndarray, src_off: np.ndarray, lens: np.ndarray, first_byte: np.ndarray):
    """encode of every message back to back; returns (frames, out_off[n+1])"""
    src = np.ascontiguousarray(src, dtype=np.uint8)
    so = np.ascontiguousarray(src_off, dtype=np.uint64)
    ln = np.ascontiguousarray(lens, dtype=np.uint64)
    fb = np.ascontiguousarray(first_byte, dtype=np.uint8)
    n = len(ln)
    out = np.zeros(int(ln.sum()) + 10 * n + 16, np.uint8)
    off = np.zeros(n + 1, np.uint64)
    tot = lib().wso_encode_batch(src.ctypes.data, so.ctypes.data, ln.ctypes.data, fb.ctypes.data, n,
                                 out.ctypes.data, off.ctypes.data)
    return out[:tot], off
