"""Seeded random client->server streams for parity tests (test infrastructure).

Each stream is one connection's post-handshake bytes: mostly well-formed traffic (single-frame
text/binary, fragmented chains incl. 0-length fragments and multi-byte characters split across
fragments, PING/PONG interleaved) with a small per-frame chance of the things the reference
rejects or mishandles (RSV bits, reserved opcodes, CONT without a start, TEXT inside a chain,
oversize/fragmented control frames, bad close codes / reasons, invalid UTF-8, unmasked frames,
non-minimal length encodings, empty PONG).
"""
from __future__ import annotations

import numpy as np

from netman_amd.synth import frame, OP_CONT, OP_TEXT, OP_BIN, OP_CLOSE, OP_PING, OP_PONG

_SAMPLE_TEXT = ["hello", "netman", "Grüße", "日本語テキスト", "emoji 😀🎉", "ασδφ", "a" * 40,
                "mixed ✓ ✗ ← → ß", ""]


def _rand_text(rng, n_max=200):
    parts = []
    while sum(len(p.encode()) for p in parts) < rng.integers(0, n_max + 1):
        parts.append(_SAMPLE_TEXT[rng.integers(len(_SAMPLE_TEXT))])
        if len(parts) > 50:
            break
    return "".join(parts).encode("utf-8")


def _bad_utf8(rng):
    bads = [b"\xff", b"\xc0\x80", b"\xed\xa0\x80", b"\xe2\x82", b"\xf4\x90\x80\x80", b"\x80", b"\xf8\x88\x80\x80\x80"]
    good = _rand_text(rng, 40)
    cut = int(rng.integers(0, len(good) + 1))
    # keep the cut on a character boundary so the only error is the injected one
    while cut < len(good) and (good[cut] & 0xC0) == 0x80:
        cut += 1
    return good[:cut] + bads[rng.integers(len(bads))] + good[cut:]


def _payload(rng, big_p=0.02):
    r = rng.random()
    if r < big_p:
        n = int(rng.choice([65535, 65536, 70000]))
    elif r < 0.1:
        n = int(rng.choice([0, 1, 2, 3, 4, 5, 125, 126, 127, 255, 256]))
    else:
        n = int(rng.integers(0, 300))
    return rng.bytes(n)


def _ctrl_payload(rng, hi):
    """control payloads: mostly ASCII (valid utf8, so Q6 rarely fires), sometimes random bytes"""
    n = int(rng.integers(0, hi))
    if rng.random() < 0.85:
        return bytes(rng.integers(0x20, 0x7F, n, dtype=np.uint8))
    return rng.bytes(n)


def _ext_for(rng, n):
    """mostly minimal; sometimes a non-minimal (but legal to the reference) length encoding"""
    if rng.random() < 0.05:
        return 8 if n > 125 or rng.random() < 0.5 else 2
    return None


def _big_pong(rng):
    """a PONG payload of any size (the reference has no limit, websocket.go:191-205): ASCII (valid
    UTF-8 under a TEXT message, Q6) or random bytes (almost surely invalid there -> 1007)"""
    n = int(rng.choice([126, 300, 4095, 4096, 9000, 70000]))
    if rng.random() < 0.7:
        return bytes(rng.integers(0x20, 0x7F, n, dtype=np.uint8))
    return rng.bytes(n)


def random_stream(seed: int, n_units: int = 20, err_p: float = 0.03, big_p: float = 0.02,
                  text_p: float = 0.3, pong_big_p: float = 0.0) -> bytes:
    """pong_big_p: chance per unit of a large PONG (and between fragments of a message) -- 0 keeps
    the streams of earlier rounds byte for byte (no extra draws)"""
    rng = np.random.default_rng(seed)
    out = bytearray()

    def F(op, payload=b"", fin=True, masked=True, rsv=0, ext=None):
        if ext is None:
            ext = _ext_for(rng, len(payload))
            if ext == 2 and len(payload) > 65535:
                ext = 8
        out.extend(frame(op, payload, fin=fin, mask=int(rng.integers(0, 2**32)), masked=masked,
                         rsv=rsv, ext=ext))

    for _ in range(n_units):
        r = rng.random()
        if r < err_p:  # something the reference rejects / mishandles
            kind = int(rng.integers(0, 12))
            if kind == 0: F(OP_BIN, b"x", rsv=int(rng.integers(1, 8)))
            elif kind == 1: F(int(rng.choice([3, 4, 5, 6, 7, 11, 12, 13, 14, 15])), b"zz")
            elif kind == 2: F(OP_CONT, b"orphan")
            elif kind == 3: F(OP_PING, rng.bytes(126))
            elif kind == 4: F(OP_PING, b"p", fin=False)
            elif kind == 5: F(OP_CLOSE, b"\x03")
            elif kind == 6: F(OP_CLOSE, (int(rng.choice([999, 1004, 1005, 1006, 1015, 1016, 2999, 5000]))).to_bytes(2, "big") + b"bye")
            elif kind == 7: F(OP_CLOSE, (1000).to_bytes(2, "big") + _bad_utf8(rng))
            elif kind == 8: F(OP_TEXT, _bad_utf8(rng))
            elif kind == 9: F(OP_BIN, b"unmasked", masked=False)
            elif kind == 10: F(OP_PONG, b"")
            else: F(OP_PONG, b"x", fin=False)
            continue
        if pong_big_p and rng.random() < pong_big_p:
            F(OP_PONG, _big_pong(rng))
            continue
        if r < 0.10:
            F(OP_PING, _ctrl_payload(rng, 126))
        elif r < 0.15:
            F(OP_PONG, _ctrl_payload(rng, 200) or b"x")
        elif r < 0.45:  # fragmented message
            text = rng.random() < text_p
            if text:
                body = _rand_text(rng, 300)
                if rng.random() < 0.02:
                    body = _bad_utf8(rng)
            else:
                body = _payload(rng, big_p)
            nfr = int(rng.integers(2, 6))
            cuts = sorted(int(x) for x in rng.integers(0, len(body) + 1, nfr - 1))
            pieces = [body[a:b] for a, b in zip([0] + cuts, cuts + [len(body)])]
            for i, pc in enumerate(pieces):
                F(OP_TEXT if (i == 0 and text) else (OP_BIN if i == 0 else OP_CONT), pc,
                  fin=(i == len(pieces) - 1))
                if i < len(pieces) - 1 and rng.random() < 0.15:
                    F(OP_PING, _ctrl_payload(rng, 20))
                if pong_big_p and i < len(pieces) - 1 and rng.random() < pong_big_p:
                    F(OP_PONG, _big_pong(rng))       # Q6: checked alone under a TEXT message
                if i < len(pieces) - 1 and rng.random() < 0.01:
                    F(OP_CLOSE, (1000).to_bytes(2, "big") + b"frag", fin=False)   # Q7 quirk
        else:
            if rng.random() < text_p:
                F(OP_TEXT, _rand_text(rng, 200))
            else:
                F(OP_BIN, _payload(rng, big_p))
        if rng.random() < 0.005:
            F(OP_CLOSE, b"" if rng.random() < 0.5 else (1000).to_bytes(2, "big") + b"done")
    return bytes(out)


# CLOSE payloads whose verdict depends on messageMode (websocket.go:153-181 with
# websocket_frame.go:49,71-73): (code, reason) byte strings covering every combination of
# whole-payload validity x reason validity x code validity
CLOSE_PAYLOADS = [
    b"\x03\xe8",                      # 1000, no reason; whole invalid (lone E8)
    b"\x03\xe8ok",                    # 1000; whole invalid (E8 6F), reason valid
    b"\x03\xe8\xff",                  # 1000; whole invalid, reason invalid  (VERDICT r1 case)
    b"\x03\xe8ok\xff",                # 1000; whole invalid, reason invalid
    b"\x03\xe8\x80\x80",              # 1000; whole VALID (E8 80 80 = U+8000), reason invalid (80 80)
    b"\x0c\x41ok",                    # 3137; whole valid, reason valid
    b"\x0c\x41o\xff",                 # 3137; whole invalid, reason invalid
    b"\x03\xe7\xff",                  # 999 (bad code); whole invalid, reason invalid
    b"\x03\xe7ok",                    # 999; whole invalid, reason valid
    b"\x0b\xb8\xe2\x82",              # 3000; whole invalid (lone B8), reason truncated
    b"\x0f\xa0\x80\xbf",              # 4000; whole invalid, reason invalid
    b"\x03\xedok",                    # 1005 (reserved); whole invalid, reason valid
    b"\x03\xe9",                      # 1001, no reason
    b"\x03\xe8" + "Grüße".encode(),   # 1000; whole invalid (E8 47), reason valid
]


def close_in_chain_stream(seed: int) -> bytes:
    """A connection that is inside a fragmented TEXT or BIN message (or not in one) when a FIN=1
    CLOSE arrives: a few ordinary frames, a chain start (+ optional fragments, PINGs, FIN=0 CLOSEs
    that join the message, Q7), then a FIN=1 CLOSE with one of CLOSE_PAYLOADS, then trailing
    frames the reference never reads.  Pins the TEXT-mode CLOSE rule."""
    rng = np.random.default_rng(seed)
    out = bytearray()

    def F(op, payload=b"", fin=True):
        out.extend(frame(op, payload, fin=fin, mask=int(rng.integers(0, 2**32))))

    for _ in range(int(rng.integers(0, 3))):
        F(OP_TEXT, _rand_text(rng, 60)) if rng.random() < 0.5 else F(OP_BIN, rng.bytes(int(rng.integers(0, 90))))
    mode = int(rng.integers(0, 3))    # 0: no message in progress, 1: TEXT chain, 2: BIN chain
    if mode:
        F(OP_TEXT if mode == 1 else OP_BIN, _rand_text(rng, 30) if mode == 1 else rng.bytes(int(rng.integers(0, 30))), fin=False)
        for _ in range(int(rng.integers(0, 3))):
            r = rng.random()
            if r < 0.3:
                F(OP_PING, bytes(rng.integers(0x20, 0x7F, int(rng.integers(0, 10)), dtype=np.uint8)))
            elif r < 0.45:
                F(OP_CLOSE, b"\x03\xe8" + _rand_text(rng, 10), fin=False)   # joins the message (Q7)
            else:
                F(OP_CONT, _rand_text(rng, 20) if mode == 1 else rng.bytes(int(rng.integers(0, 20))), fin=False)
    F(OP_CLOSE, CLOSE_PAYLOADS[int(rng.integers(len(CLOSE_PAYLOADS)))])
    F(OP_BIN, b"never read")
    return bytes(out)


def random_splits(rng, n: int, k: int):
    """k random cut points in (0, n) -> increasing chunk ends ending at n"""
    if n == 0:
        return [0]
    cuts = sorted(set(int(x) for x in rng.integers(1, max(n, 2), k))) if k else []
    return [c for c in cuts if 0 < c < n] + [n]
