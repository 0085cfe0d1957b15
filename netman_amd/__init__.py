"""netman_amd -- MI355X (gfx950) WebSocket frame decoder for netman's websocket decode path.

The product is libwscodec.so (include/wscodec.h): hand-written HIP kernels behind a C ABI.
This package holds its sources (csrc/), the build recipe, the ctypes binding + Python mirror of
netman's Message/error surface (codec.py) and the synthetic traffic generator (synth.py).
"""
from .codec import (Codec, Session, Message, load_library, default_config,  # noqa: F401
                    CONN_STATE_DTYPE, FRAME_DTYPE, SEG_RESULT_DTYPE, SUMMARY_DTYPE)

__all__ = ["Codec", "Session", "Message", "load_library", "default_config"]
