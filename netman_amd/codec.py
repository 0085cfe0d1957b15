"""ctypes binding of libwscodec.so (include/wscodec.h) and the Python mirror of netman's
websocket decode surface.

Reference surface mirrored here (ikilobyte/netman, Go):
  util/message.go:4-53      Message{MsgID, DataLen, Data, IsWebSocket, Opcode} + ID/Bytes/String/...
  util/errors.go:9-14       websocket error sentinels (same texts)
  iface/iconnect.go:38-39   IConnectEvent.DecodePacket() (IMessage, error)   -> Session.DecodePacket
  eventloop/epoll.go:106-129 sentinel -> close code                          -> close_code_for()

The product path is the HIP library: if libwscodec.so cannot be loaded, or no gfx950 device is
present, every entry point raises.  There is no CPU fallback in this package.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libwscodec.so")

# ---- constants (include/wscodec.h) -------------------------------------------------------------
WSC_OK = 0
WSC_E_INVAL, WSC_E_DEVICE, WSC_E_NOMEM, WSC_E_CAPACITY, WSC_E_NODEVICE, WSC_E_STATE = -1, -2, -3, -4, -5, -6
WSC_E_INTERNAL = -7

ERR_NONE, ERR_OPCODE_FAIL, ERR_RSV_FAIL, ERR_PING_PAYLOAD_OVERSIZE = 0, 1, 2, 3
ERR_CTRL_FRAGMENTED, ERR_MUST_UTF8, ERR_PROTOCOL_ERROR, ERR_TOO_LARGE = 4, 5, 6, 7
ERR_DEVICE = 8   # session: the connection's batch hit a device error -> CloseCode(1011)
ERR_NO_PROGRESS = 9   # session: a whole batch of a connection's bytes decoded nothing -> CloseCode(1009)
ERR_MSG_TOO_BIG = 10  # session: a message passed wsc_session_set_max_message -> CloseCode(1009)

FK_FRAG, FK_MESSAGE, FK_PING, FK_PONG, FK_CLOSE, FK_PONG_EMPTY, FK_ERROR, FK_STALL, FK_PIECE = range(9)
FF_UNMASKED, FF_CONT_MSG, FF_CTRL_ARENA, FF_HEAD_PREV = 0x01, 0x02, 0x40, 0x80

SEG_OPEN, SEG_CLOSED, SEG_ERROR, SEG_STALLED = 0, 1, 2, 3
F_COMPACT = 0x1
SESSION_BLOCKING_WAIT = 0x100   # wsc_session_create: complete() sleeps on a blocking-sync event
SESSION_TIMING = 0x200          # ... seconds per phase printed to stderr at destroy
SESSION_COPY_ENGINE = 0x400     # ... every staging copy by hipMemcpyAsync
SESSION_KCOPY_ALL = 0x800       # ... every staging copy by wsc_kcopy kernels
# wsc_config.walk_flags (header-walk variants with the same results; tests pin them)
WALK_NO_QUAD_PRE, WALK_NO_HDR_CACHE, WALK_HDR_NT, WALK_DEBUG_STAMPS = 0x1, 0x2, 0x4, 0x8

EV_NONE, EV_MESSAGE, EV_PONG, EV_CLOSE, EV_STALL = 0, 1, 2, 3, 4

# ---- numpy views of the ABI records ------------------------------------------------------------
CONN_STATE_DTYPE = np.dtype([("cont_len", "<u8"), ("msg_id", "<u4"), ("message_mode", "u1"),
                             ("cont_utf8", "u1"), ("status", "u1"), ("frame_hdr", "u1"),
                             ("frame_rem", "<u8"), ("frame_len", "<u8"), ("frame_mask", "<u4"),
                             ("frame_utf8", "u1"), ("pad", "u1", (3,))])
FRAME_DTYPE = np.dtype([("hdr_off", "<u8"), ("payload_len", "<u4"), ("mask", "<u4"), ("seg", "<u4"),
                        ("msg_id", "<u4"), ("opcode", "u1"), ("fin", "u1"), ("kind", "u1"),
                        ("mode", "u1"), ("err", "u1"), ("hdr_len", "u1"), ("flags", "u1"),
                        ("payload_len_hi", "u1")])
SEG_RESULT_DTYPE = np.dtype([("consumed", "<u8"), ("frame_begin", "<u4"), ("frame_count", "<u4"),
                             ("status", "<u4"), ("close_code", "<u4"), ("err", "<u4"), ("pad", "<u4")])
SUMMARY_DTYPE = np.dtype([("data_bytes", "<u8"), ("ctrl_bytes", "<u8"), ("n_frames", "<u4"),
                          ("n_spans", "<u4"), ("overflow", "<u4"), ("pad", "<u4")])
STATE_BYTES = 40   # sizeof(wsc_conn_state)
assert CONN_STATE_DTYPE.itemsize == STATE_BYTES and FRAME_DTYPE.itemsize == 32


def frame_len(rec) -> int:
    """a wsc_frame record's payload length (40 bits: payload_len | payload_len_hi << 32)"""
    return int(rec["payload_len"]) | int(rec["payload_len_hi"]) << 32
assert SEG_RESULT_DTYPE.itemsize == 32 and SUMMARY_DTYPE.itemsize == 32
# wsc_out_msg: one outbound frame for wsc_encode (websocket_ctrl.go:23-70 encode(firstByte, bs))
OUT_MSG_DTYPE = np.dtype([("src_off", "<u8"), ("len", "<u8"), ("first_byte", "u1"), ("pad", "u1", (7,))])
assert OUT_MSG_DTYPE.itemsize == 24


class WscConfig(C.Structure):
    _fields_ = [("max_batch_bytes", C.c_uint64), ("max_segs", C.c_uint32), ("max_frames", C.c_uint32),
                ("max_frame_len", C.c_uint64), ("unmask_window", C.c_uint32),
                ("unmask_waves_per_cu", C.c_uint32), ("unmask_nt", C.c_uint32), ("unmask_minw", C.c_uint32),
                ("walk_mode", C.c_uint32), ("u8_inline_max", C.c_uint32), ("walk_flags", C.c_uint32),
                ("pad", C.c_uint32)]


class WscBatch(C.Structure):
    _fields_ = [("wire", C.c_void_p), ("n_bytes", C.c_uint64), ("seg_off", C.c_void_p),
                ("n_segs", C.c_uint32), ("flags", C.c_uint32), ("state_in", C.c_void_p),
                ("state_out", C.c_void_p), ("seg_out", C.c_void_p), ("frames", C.c_void_p),
                ("frames_cap", C.c_uint32), ("pad", C.c_uint32), ("arena", C.c_void_p),
                ("frame_dst", C.c_void_p), ("summary", C.c_void_p)]


class WscEvent(C.Structure):
    _fields_ = [("type", C.c_uint32), ("msg_id", C.c_uint32), ("opcode", C.c_uint32),
                ("close_code", C.c_uint32), ("err", C.c_uint32), ("pad", C.c_uint32),
                ("data", C.POINTER(C.c_uint8)), ("len", C.c_uint64)]


class WscConnState(C.Structure):
    _fields_ = [("cont_len", C.c_uint64), ("msg_id", C.c_uint32), ("message_mode", C.c_uint8),
                ("cont_utf8", C.c_uint8), ("status", C.c_uint8), ("frame_hdr", C.c_uint8),
                ("frame_rem", C.c_uint64), ("frame_len", C.c_uint64), ("frame_mask", C.c_uint32),
                ("frame_utf8", C.c_uint8), ("pad", C.c_uint8 * 3)]


# every function include/wscodec.h declares, with its ctypes signature
_P, _U32, _U64, _I = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
SIGNATURES = {
    "wsc_abi_version": (_I, []),
    "wsc_last_error": (C.c_char_p, []),
    "wsc_config_default": (_I, [C.POINTER(WscConfig)]),
    "wsc_create": (_I, [_I, C.POINTER(WscConfig), C.POINTER(_P)]),
    "wsc_destroy": (_I, [_P]),
    "wsc_dev_alloc": (_I, [_P, _U64, C.POINTER(_P)]),
    "wsc_dev_free": (_I, [_P, _P]),
    "wsc_host_alloc": (_I, [_U64, C.POINTER(_P)]),
    "wsc_host_free": (_I, [_P]),
    "wsc_kcopy": (_I, [_P, _P, _P, _U64, _P]),
    "wsc_decode": (_I, [_P, C.POINTER(WscBatch), _P]),
    "wsc_sync": (_I, [_P, _P]),
    "wsc_summary_status": (_I, [_P]),
    "wsc_error_flags": (_I, [_P, C.POINTER(_U32), _I]),
    "wsc_decode_split": (_I, [_P, C.POINTER(WscBatch), _P, _P]),
    "wsc_decode_walk": (_I, [_P, C.POINTER(WscBatch), _P]),
    "wsc_decode_finish": (_I, [_P, C.POINTER(WscBatch), _P]),
    "wsc_walk_wait": (_I, [_P]),
    "wsc_stream_create": (_I, [_P, _P, _U32, C.POINTER(_P)]),
    "wsc_stream_create_ex": (_I, [_P, _P, _U32, _I, C.POINTER(_P)]),
    "wsc_stream_destroy": (_I, [_P, _P]),
    "wsc_decode_host": (_I, [_P, _P, _U64, _P, _U32, _U32, _P, _P, _P, _P, _U32, _P, _P, _P]),
    "wsc_encode": (_I, [_P, _P, _U32, _P, _U64, _P, _U64, _P, _P]),
    "wsc_encode_host": (_I, [_P, _P, _U32, _P, _U64, _P, _U64, _P]),
    "wsc_profile": (_I, [_P, C.POINTER(WscBatch), _I, C.POINTER(C.c_double)]),
    "wsc_debug_stamps": (_I, [_P, _P, _U32]),
    "wsc_walk_info": (_I, [_P, C.POINTER(_U32), C.POINTER(_U32)]),
    "wsc_session_create": (_I, [_I, C.POINTER(WscConfig), _U32, C.POINTER(_P)]),
    "wsc_session_destroy": (_I, [_P]),
    "wsc_session_open": (_I, [_P, C.POINTER(_U32)]),
    "wsc_session_remove": (_I, [_P, _U32]),
    "wsc_session_reserve": (_I, [_P, _U32, _U64, C.POINTER(_P), C.POINTER(_U64)]),
    "wsc_session_commit": (_I, [_P, _U32, _U64]),
    "wsc_session_feed": (_I, [_P, _U32, _P, _U64]),
    "wsc_session_submit": (_I, [_P]),
    "wsc_session_complete": (_I, [_P]),
    "wsc_session_decode": (_I, [_P]),
    "wsc_session_pending": (_I, [_P, C.POINTER(_U64)]),
    "wsc_session_ready": (_I, [_P, C.POINTER(_I)]),
    "wsc_session_next": (_I, [_P, _U32, C.POINTER(WscEvent)]),
    "wsc_session_eof": (_I, [_P, _U32]),
    "wsc_session_set_max_message": (_I, [_P, _U64]),
    "wsc_session_state": (_I, [_P, _U32, C.POINTER(WscConnState), C.POINTER(_U64)]),
    "wsc_session_stats": (_I, [_P, C.POINTER(_U64), _U32]),
    "wsc_session_inject_fault": (_I, [_P, _U64]),
}

_lib = None
ABI_VERSION = 5   # include/wscodec.h WSC_ABI_VERSION: the record layouts above


def load_library(path: str = LIB_PATH):
    """Load libwscodec.so (raises OSError if it is missing: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"libwscodec.so not built ({path}); run __graft_entry__.build()")
    # One HIP runtime per process: torch wheels bundle their own libamdhip64.so (SONAME
    # libamdhip64.so.7, the same as /opt/rocm's).  Loading torch first lets our DT_NEEDED resolve
    # to that already-loaded runtime, so torch tensors and our kernels share one HIP/ROCr
    # instance; without torch (C/Go hosts) the library uses /opt/rocm's runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.wsc_abi_version() != ABI_VERSION:
        raise OSError(f"{path}: ABI version {lib.wsc_abi_version()}, this module speaks {ABI_VERSION}: rebuild")
    _lib = lib
    return lib


class WscError(RuntimeError):
    def __init__(self, rc: int, where: str):
        lib = load_library()
        super().__init__(f"{where} failed: rc={rc} ({lib.wsc_last_error().decode(errors='replace')})")
        self.rc = rc


def _check(rc: int, where: str):
    if rc != WSC_OK:
        raise WscError(rc, where)


# Process-wide overrides of wsc_config fields applied by default_config() under its own keyword
# arguments: lets a test pin a walk variant (walk_mode, u8_inline_max, walk_flags) for every context
# it creates, helpers included.  An explicit Python API -- nothing reads the environment.
CFG_DEFAULTS: dict = {}


def default_config(**over) -> WscConfig:
    lib = load_library()
    cfg = WscConfig()
    _check(lib.wsc_config_default(C.byref(cfg)), "wsc_config_default")
    for k, v in {**CFG_DEFAULTS, **over}.items():
        setattr(cfg, k, v)
    return cfg


def _ptr(a) -> int:
    """device/host address of a numpy array or torch tensor (None -> NULL)"""
    if a is None:
        return 0
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()


@dataclass
class DecodeResult:
    seg: np.ndarray          # SEG_RESULT_DTYPE [n_segs]
    state: np.ndarray        # CONN_STATE_DTYPE [n_segs]
    frames: np.ndarray       # FRAME_DTYPE [n_frames]
    summary: np.ndarray      # SUMMARY_DTYPE scalar
    frame_dst: np.ndarray | None = None
    arena: np.ndarray | None = None


def cu_mask(cus, n_cu: int) -> list:
    """u32 words of a hipExtStreamCreateWithCUMask mask with the bits of `cus` set"""
    w = [0] * ((n_cu + 31) // 32)
    for i in cus:
        if not 0 <= i < n_cu:
            raise ValueError(f"CU {i} out of range 0..{n_cu - 1}")
        w[i // 32] |= 1 << (i % 32)
    return w


class Codec:
    """One device context (wsc_ctx)."""

    def __init__(self, device: int = 0, **cfg_over):
        self.lib = load_library()
        self.cfg = default_config(**cfg_over)
        h = C.c_void_p()
        _check(self.lib.wsc_create(device, C.byref(self.cfg), C.byref(h)), "wsc_create")
        self.h = h

    def close(self):
        if self.h:
            self.lib.wsc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # device-resident batch: all arguments are torch CUDA tensors (or None)
    def make_batch(self, wire, seg_off, state_in, state_out, seg_out, frames, summary,
                   compact=False, arena=None, frame_dst=None, n_bytes=None) -> WscBatch:
        b = WscBatch()
        b.wire = _ptr(wire)
        b.n_bytes = int(wire.numel() if n_bytes is None else n_bytes)
        b.seg_off = _ptr(seg_off)
        b.n_segs = int(seg_off.numel() - 1)
        b.flags = F_COMPACT if compact else 0
        b.state_in = _ptr(state_in)
        b.state_out = _ptr(state_out)
        b.seg_out = _ptr(seg_out)
        b.frames = _ptr(frames)
        b.frames_cap = int(frames.numel() // FRAME_DTYPE.itemsize)
        b.arena = _ptr(arena)
        b.frame_dst = _ptr(frame_dst)
        b.summary = _ptr(summary)
        return b

    @staticmethod
    def _stream(stream):
        """default to torch's current stream (0 = the null stream), so launches are ordered after
        the torch ops that produced the batch tensors (fills, copies)"""
        if stream is not None:
            return stream
        import sys
        torch = sys.modules.get("torch")
        if torch is not None and torch.cuda.is_initialized():
            return torch.cuda.current_stream().cuda_stream or None
        return None

    def decode(self, batch: WscBatch, stream=None):
        _check(self.lib.wsc_decode(self.h, C.byref(batch), self._stream(stream)), "wsc_decode")

    def decode_split(self, batch: WscBatch, walk_stream: int, unmask_stream: int):
        """walk on walk_stream, UTF-8 check + unmask on unmask_stream (wsc_decode_split)"""
        _check(self.lib.wsc_decode_split(self.h, C.byref(batch), walk_stream, unmask_stream), "wsc_decode_split")

    def walk_info(self) -> tuple[int, int]:
        """(geometry, blocks) of the last decode's header walk (wsc_walk_info)"""
        m, b = C.c_uint32(), C.c_uint32()
        _check(self.lib.wsc_walk_info(self.h, C.byref(m), C.byref(b)), "wsc_walk_info")
        return m.value, b.value

    def error_flags(self, clear: bool = False) -> int:
        """sticky error bits of every decode/encode on this context (wsc_error_flags): bit0 frame
        capacity exceeded, bit1 decode look-back timeout, bit2 encode look-back timeout"""
        v = C.c_uint32()
        _check(self.lib.wsc_error_flags(self.h, C.byref(v), 1 if clear else 0), "wsc_error_flags")
        return v.value

    @staticmethod
    def summary_status(summary) -> int:
        """wsc_summary_status of a host copy of wsc_summary (SUMMARY_DTYPE record or 32 bytes)"""
        a = np.asarray(summary)
        if a.dtype == SUMMARY_DTYPE:
            a = a.reshape(1)          # a record scalar (e.g. summary[0]) -> 1-element array
        a = np.ascontiguousarray(np.ascontiguousarray(a).view(np.uint8).reshape(-1)[:32])
        return load_library().wsc_summary_status(a.ctypes.data)

    def decode_walk(self, batch: WscBatch, walk_stream: int):
        """staged split decode, part 1: the walk (waits on the host for this context's last staged unmask)"""
        _check(self.lib.wsc_decode_walk(self.h, C.byref(batch), walk_stream), "wsc_decode_walk")

    def decode_finish(self, batch: WscBatch, unmask_stream: int):
        _check(self.lib.wsc_decode_finish(self.h, C.byref(batch), unmask_stream), "wsc_decode_finish")

    def walk_wait(self):
        _check(self.lib.wsc_walk_wait(self.h), "wsc_walk_wait")

    def stream_create(self, cu_mask=None, priority: int = 0) -> int:
        """a raw hipStream_t (int), restricted to the CUs set in cu_mask (list of u32 words);
        priority > 0: the device's greatest queue priority over all CUs (wsc_stream_create_ex)"""
        out = C.c_void_p()
        if priority:
            _check(self.lib.wsc_stream_create_ex(self.h, None, 0, int(priority), C.byref(out)), "wsc_stream_create_ex")
        elif cu_mask is None:
            _check(self.lib.wsc_stream_create(self.h, None, 0, C.byref(out)), "wsc_stream_create")
        else:
            arr = (C.c_uint32 * len(cu_mask))(*cu_mask)
            _check(self.lib.wsc_stream_create(self.h, arr, len(cu_mask), C.byref(out)), "wsc_stream_create")
        return out.value

    def kcopy(self, dst, src, nbytes: int, stream=None):
        """wsc_kcopy: nbytes between device and pinned host memory (tensors, arrays or int
        addresses; host side from wsc_host_alloc) by a kernel on `stream`; returns once queued"""
        a = lambda x: x if isinstance(x, int) else _ptr(x)
        _check(self.lib.wsc_kcopy(self.h, a(dst), a(src), nbytes, self._stream(stream)), "wsc_kcopy")

    def stream_destroy(self, stream: int):
        _check(self.lib.wsc_stream_destroy(self.h, stream), "wsc_stream_destroy")

    def sync(self, stream=None):
        _check(self.lib.wsc_sync(self.h, self._stream(stream)), "wsc_sync")

    def profile(self, batch: WscBatch, iters: int):
        import sys
        torch = sys.modules.get("torch")
        if torch is not None and torch.cuda.is_initialized():
            torch.cuda.synchronize()     # the profile runs on the context's own stream
        out = (C.c_double * 6)()
        _check(self.lib.wsc_profile(self.h, C.byref(batch), iters, out), "wsc_profile")
        v = list(out)
        return {"walk": v[0], "unmask": v[1], "u8": v[2], "total": v[5]}

    # ---- encode (server -> client framing, websocket_ctrl.go:23-70) ----
    def encode(self, msgs, n_msgs: int, src, src_bytes: int, out, out_cap: int, out_off, stream=None):
        """Device-resident batched encode: msgs (OUT_MSG_DTYPE records), src, out, out_off are
        torch CUDA tensors; out_off[n_msgs] receives the total frame bytes."""
        _check(self.lib.wsc_encode(self.h, _ptr(msgs), int(n_msgs), _ptr(src), int(src_bytes), _ptr(out),
                                   int(out_cap), _ptr(out_off), self._stream(stream)), "wsc_encode")

    def encode_host(self, msgs: np.ndarray, src: np.ndarray, out_cap: int | None = None):
        """Host-buffer encode: returns (frames bytes as np.uint8 array, out_off)."""
        msgs = np.ascontiguousarray(msgs, dtype=OUT_MSG_DTYPE)
        src = np.ascontiguousarray(src, dtype=np.uint8)
        n = len(msgs)
        if out_cap is None:
            out_cap = int(msgs["len"].astype(np.uint64).sum()) + 10 * n
        out = np.zeros(max(out_cap, 16), np.uint8)
        off = np.zeros(n + 1, np.uint64)
        _check(self.lib.wsc_encode_host(self.h, _ptr(msgs), n, _ptr(src), len(src), _ptr(out), int(out_cap),
                                        _ptr(off)), "wsc_encode_host")
        return out[: int(off[n])], off

    def decode_host(self, wire: np.ndarray, seg_off: np.ndarray, state_in: np.ndarray | None = None,
                    compact: bool = False, frames_cap: int | None = None) -> DecodeResult:
        """Host-buffer path (H2D, decode, D2H).  In-place mode rewrites `wire`."""
        assert wire.dtype == np.uint8 and wire.flags.c_contiguous
        seg_off = np.ascontiguousarray(seg_off, dtype=np.uint64)
        n = len(seg_off) - 1
        cap = int(frames_cap or self.cfg.max_frames)
        state_out = np.zeros(n, CONN_STATE_DTYPE)
        seg = np.zeros(n, SEG_RESULT_DTYPE)
        frames = np.zeros(cap, FRAME_DTYPE)
        summary = np.zeros(1, SUMMARY_DTYPE)
        arena = np.zeros(len(wire) + 64, np.uint8) if compact else None
        frame_dst = np.zeros(cap, np.uint64) if compact else None
        if state_in is not None:
            state_in = np.ascontiguousarray(state_in, dtype=CONN_STATE_DTYPE)
        rc = self.lib.wsc_decode_host(self.h, _ptr(wire), len(wire), _ptr(seg_off), n,
                                      F_COMPACT if compact else 0, _ptr(state_in), _ptr(state_out),
                                      _ptr(seg), _ptr(frames), cap, _ptr(arena), _ptr(frame_dst),
                                      _ptr(summary))
        _check(rc, "wsc_decode_host")
        nf = int(summary[0]["n_frames"])
        return DecodeResult(seg=seg, state=state_out, frames=frames[:nf].copy(), summary=summary[0],
                            frame_dst=None if frame_dst is None else frame_dst[:nf].copy(),
                            arena=arena)


# ---- netman's message / error surface ----------------------------------------------------------
class Message:
    """util.Message (util/message.go:4-53)."""
    __slots__ = ("MsgID", "DataLen", "Data", "IsWebSocket", "Opcode")

    def __init__(self, MsgID: int, Data: bytes, Opcode: int, IsWebSocket: bool = True):
        self.MsgID = MsgID
        self.Data = Data
        self.DataLen = len(Data)
        self.IsWebSocket = IsWebSocket
        self.Opcode = Opcode

    def ID(self): return self.MsgID
    def String(self): return self.Data.decode("utf-8", errors="replace")
    def Bytes(self): return self.Data
    def Len(self): return self.DataLen
    def SetData(self, b: bytes): self.Data, self.DataLen = b, len(b)
    def GetOpcode(self): return self.Opcode
    def IsWebsocket(self): return self.IsWebSocket
    def IsText(self): return self.Opcode == 1
    def IsBinary(self): return self.Opcode == 2

    def __repr__(self):
        return f"Message(MsgID={self.MsgID}, Opcode={self.Opcode}, DataLen={self.DataLen})"


class NetmanError(Exception):
    pass


# util/errors.go:9-14 (texts verbatim) + syscall.EAGAIN + io.EOF
WebsocketOpcodeFail = NetmanError("websocket opcode fail")
WebsocketRsvFail = NetmanError("websocket RSV must be 0")
WebsocketPingPayloadOversize = NetmanError("websocket ping payload oversize")
WebsocketCtrlMessageMustNotFragmented = NetmanError("websocket control message MUST NOT be fragmented")
WebsocketMustUtf8 = NetmanError("websocket text message must utf-8")
WebsocketProtocolError = NetmanError("websocket protocol error")
WebsocketFrameTooLarge = NetmanError("websocket frame exceeds max_frame_len")  # Q4 divergence
DeviceFailure = NetmanError("websocket decode device failure")                  # session policy -> 1011
NoProgress = NetmanError("websocket frame header larger than the decode batch")  # session guard -> 1009
MessageTooBig = NetmanError("websocket message exceeds the session cap")         # optional cap -> 1009
EAGAIN = NetmanError("resource temporarily unavailable")

SENTINELS = {
    ERR_OPCODE_FAIL: WebsocketOpcodeFail,
    ERR_RSV_FAIL: WebsocketRsvFail,
    ERR_PING_PAYLOAD_OVERSIZE: WebsocketPingPayloadOversize,
    ERR_CTRL_FRAGMENTED: WebsocketCtrlMessageMustNotFragmented,
    ERR_MUST_UTF8: WebsocketMustUtf8,
    ERR_PROTOCOL_ERROR: WebsocketProtocolError,
    ERR_TOO_LARGE: WebsocketFrameTooLarge,
    ERR_DEVICE: DeviceFailure,
    ERR_NO_PROGRESS: NoProgress,
    ERR_MSG_TOO_BIG: MessageTooBig,
}


def close_code_for(err) -> int | None:
    """eventloop/epoll.go:106-129: which CloseCode the poller sends for a DecodePacket error."""
    if err in (WebsocketOpcodeFail, WebsocketRsvFail, WebsocketCtrlMessageMustNotFragmented,
               WebsocketProtocolError, WebsocketPingPayloadOversize, WebsocketFrameTooLarge):
        return 1002
    if err is WebsocketMustUtf8:
        return 1007
    if err is DeviceFailure:
        return 1011
    if err is NoProgress or err is MessageTooBig:
        return 1009
    return None


@dataclass
class Event:
    type: int
    msg_id: int = 0
    opcode: int = 0
    close_code: int = 0
    err: int = 0
    data: bytes = b""


class Session:
    """Many connections decoded in batches on one device (wsc_session_*)."""

    def __init__(self, device: int = 0, compact: bool = False, flags: int = 0, **cfg_over):
        self.lib = load_library()
        self.cfg = default_config(**cfg_over)
        h = C.c_void_p()
        _check(self.lib.wsc_session_create(device, C.byref(self.cfg), (F_COMPACT if compact else 0) | flags,
                                           C.byref(h)), "wsc_session_create")
        self.h = h

    def close(self):
        if self.h:
            self.lib.wsc_session_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def open(self) -> int:
        cid = C.c_uint32()
        _check(self.lib.wsc_session_open(self.h, C.byref(cid)), "wsc_session_open")
        return cid.value

    def remove(self, conn: int):
        _check(self.lib.wsc_session_remove(self.h, conn), "wsc_session_remove")

    def feed(self, conn: int, data: bytes):
        buf = (C.c_uint8 * len(data)).from_buffer_copy(data) if data else None
        _check(self.lib.wsc_session_feed(self.h, conn, buf, len(data)), "wsc_session_feed")

    def reserve_commit(self, conn: int, data: bytes) -> int:
        """one socket read the zero-copy way: reserve room in the pinned staging, write into it
        (here: from `data`, standing in for recv()), commit what was written; returns bytes taken"""
        p, avail = C.c_void_p(), C.c_uint64()
        _check(self.lib.wsc_session_reserve(self.h, conn, len(data), C.byref(p), C.byref(avail)), "wsc_session_reserve")
        if not p.value:
            return 0
        k = min(len(data), avail.value)
        C.memmove(p.value, data, k)
        _check(self.lib.wsc_session_commit(self.h, conn, k), "wsc_session_commit")
        return k

    def read_tls(self, conn: int, layer, max_bytes: int):
        """INTEGRATION.md's Session.ReadTLS: with TLS on, readData reads through the tls.Conn
        (server/baseconnect.go:347-353), which returns at most one record's plaintext per Read and
        keeps later records in its own buffers, out of epoll's sight.  So read into the reserved
        room until the layer reports EAGAIN (layer.read raises BlockingIOError) or the room is
        full.  layer.read(n) returns up to n plaintext bytes, b"" for io.EOF.
        Returns (bytes read, more, eof): more = the room filled, read again next round."""
        p, avail = C.c_void_p(), C.c_uint64()
        _check(self.lib.wsc_session_reserve(self.h, conn, max_bytes, C.byref(p), C.byref(avail)), "wsc_session_reserve")
        if not p.value:
            return 0, False, False
        n, eof = 0, False
        while n < avail.value:
            try:
                b = layer.read(avail.value - n)
            except BlockingIOError:
                break
            if not b:
                eof = True
                break
            C.memmove(p.value + n, b, len(b))
            n += len(b)
        _check(self.lib.wsc_session_commit(self.h, conn, n), "wsc_session_commit")
        return n, (n == avail.value and not eof), eof

    def submit(self):
        _check(self.lib.wsc_session_submit(self.h), "wsc_session_submit")

    def complete(self):
        _check(self.lib.wsc_session_complete(self.h), "wsc_session_complete")

    def decode(self):
        _check(self.lib.wsc_session_decode(self.h), "wsc_session_decode")

    def eof(self, conn: int):
        """the peer closed (a read returned 0): wsc_session_eof -- queued events first, then Close()"""
        _check(self.lib.wsc_session_eof(self.h, conn), "wsc_session_eof")

    def inject_fault(self, k: int):
        """test hook: the k-th device submission from now fails as a device error would"""
        _check(self.lib.wsc_session_inject_fault(self.h, int(k)), "wsc_session_inject_fault")

    def set_max_message(self, nbytes: int):
        _check(self.lib.wsc_session_set_max_message(self.h, int(nbytes)), "wsc_session_set_max_message")

    def ready(self) -> bool:
        """complete() would not wait for the device (wsc_session_ready)"""
        r = C.c_int()
        _check(self.lib.wsc_session_ready(self.h, C.byref(r)), "wsc_session_ready")
        return bool(r.value)

    def pending(self) -> int:
        """bytes fed but not yet submitted (submit again while non-zero)"""
        n = C.c_uint64()
        _check(self.lib.wsc_session_pending(self.h, C.byref(n)), "wsc_session_pending")
        return n.value

    def next_event(self, conn: int) -> Event:
        ev = WscEvent()
        _check(self.lib.wsc_session_next(self.h, conn, C.byref(ev)), "wsc_session_next")
        data = C.string_at(ev.data, ev.len) if ev.len else b""
        return Event(ev.type, ev.msg_id, ev.opcode, ev.close_code, ev.err, data)

    def events(self, conn: int) -> list[Event]:
        out = []
        while True:
            e = self.next_event(conn)
            if e.type == EV_NONE:
                return out
            out.append(e)

    def DecodePacket(self, conn: int):
        """IConnectEvent.DecodePacket() for an already-fed-and-decoded connection:
        (Message, None) | (None, None) after a PONG reply / close | (None, sentinel) | (None, EAGAIN)."""
        e = self.next_event(conn)
        if e.type == EV_MESSAGE:
            return Message(e.msg_id, e.data, e.opcode), None
        if e.type == EV_CLOSE:
            return None, (SENTINELS.get(e.err) if e.err else None)
        if e.type == EV_PONG:
            return None, None
        return None, EAGAIN

    def stats(self) -> dict:
        """wsc_session_stats: bytes read, sent to the device, sent again (carried), batches,
        streamed payload bytes collected into messages"""
        v = (C.c_uint64 * 5)()
        _check(self.lib.wsc_session_stats(self.h, v, 5), "wsc_session_stats")
        return dict(zip(("read", "h2d", "resent", "batches", "pieces"), list(v)))

    def state(self, conn: int):
        st = WscConnState()
        carry = C.c_uint64()
        _check(self.lib.wsc_session_state(self.h, conn, C.byref(st), C.byref(carry)), "wsc_session_state")
        return st, carry.value
