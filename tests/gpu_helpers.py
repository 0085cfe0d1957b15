"""Shared checks for the GPU parity tests: device records vs the oracle's frame log."""
from __future__ import annotations

import numpy as np

import oracle_ref as O
from netman_amd import codec as K


def pack_streams(streams):
    """concatenate streams as segments (16 B-aligned buffer start)"""
    lens = [len(s) for s in streams]
    off = np.zeros(len(streams) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    wire = np.frombuffer(b"".join(streams), dtype=np.uint8).copy() if sum(lens) else np.zeros(0, np.uint8)
    return wire, off


def header_len(stream, off):
    """(header bytes, payload length) of the masked frame header at stream[off:]"""
    b1 = stream[off + 1] & 0x7F
    if b1 == 126:
        return 8, int.from_bytes(stream[off + 2:off + 4], "big")
    if b1 == 127:
        return 14, int.from_bytes(stream[off + 2:off + 10], "big")
    return 6, b1


def xor_phased(buf, lo, hi, mask):
    """XOR buf[lo:hi] with the 4 mask bytes phased to lo (byte i takes mask byte i & 3)"""
    if hi <= lo:
        return buf
    k = np.frombuffer(int(mask).to_bytes(4, "little"), dtype=np.uint8)
    buf[lo:hi] ^= np.resize(k, hi - lo)
    return buf


def compare_segment(si, stream, seg_start, res: K.DecodeResult, ora: O.OracleOut, wire_after=None,
                    compact=False, check_state=True):
    sr = res.seg[si]
    fb, fc = int(sr["frame_begin"]), int(sr["frame_count"])
    fr = res.frames[fb:fb + fc]
    of = ora.frames
    # A data frame whose payload is still arriving at the segment's end is streamed (ABI 3): its
    # record is a WSC_FK_PIECE holding the bytes that are here, unmasked; the oracle logs a frame
    # only once nextFrame completes it (websocket_frame.go:31), so the piece is checked on its own
    piece = None
    if fc and int(fr[fc - 1]["kind"]) == K.FK_PIECE:
        piece = fr[fc - 1]
        fr, fc = fr[:fc - 1], fc - 1
        p_off = int(piece["hdr_off"]) - seg_start
        hl, plen = header_len(stream, p_off)
        assert int(piece["hdr_len"]) == hl and int(piece["flags"]) & K.FF_UNMASKED, f"seg {si} piece {piece}"
        assert p_off + hl + K.frame_len(piece) == len(stream), f"seg {si}: the piece must end the segment"
        assert int(piece["mask"]) == int.from_bytes(stream[p_off + hl - 4:p_off + hl], "little")
        assert int(sr["consumed"]) == len(stream) and int(sr["status"]) == K.SEG_OPEN
        st = res.state[si]
        assert int(st["frame_rem"]) == plen - K.frame_len(piece) and int(st["frame_len"]) == plen, f"seg {si} {st}"
        assert int(st["frame_hdr"]) == (stream[p_off] & 0x8F), f"seg {si} {st}"
    assert fc == len(of), f"seg {si}: {fc} device frames vs {len(of)} oracle frames\n{fr}\n{of}"
    for i in range(fc):
        d, o = fr[i], of[i]
        ctx = f"seg {si} frame {i}: dev={d} ora={o}"
        assert int(d["hdr_off"]) - seg_start == int(o["hdr_off"]), ctx
        for f in ("kind", "opcode", "fin", "mode", "msg_id"):
            assert int(d[f]) == int(o[f]), f + " " + ctx
        assert int(d["err"]) == int(o["err"]), "err " + ctx
        if int(d["kind"]) != K.FK_STALL and int(d["err"]) != K.ERR_RSV_FAIL:
            assert K.frame_len(d) == min(int(o["payload_len"]), (1 << 40) - 1), ctx   # 40-bit record, saturated
            assert int(d["mask"]) == int(o["mask"]), ctx
            assert int(d["hdr_off"]) + int(d["hdr_len"]) - seg_start == int(o["payload_off"]), ctx
    # terminal status
    r = ora.res
    if r["closed"]:
        assert int(sr["status"]) in (K.SEG_CLOSED, K.SEG_ERROR), f"seg {si} status {sr}"
        assert int(sr["close_code"]) == r["close_code"], f"seg {si} {sr} vs {r}"
        assert int(sr["err"]) == r["err"], f"seg {si} {sr} vs {r}"
    elif r["stalled"]:
        assert int(sr["status"]) == K.SEG_STALLED, f"seg {si} {sr}"
    else:
        assert int(sr["status"]) == K.SEG_OPEN, f"seg {si} {sr} vs {r}"
        if check_state and int(sr["consumed"]) == len(stream):   # no partial frame pending
            st = res.state[si]
            assert int(st["msg_id"]) == r["msg_id"], f"seg {si} {st} vs {r}"
            assert int(st["message_mode"]) == r["message_mode"], f"seg {si} {st} vs {r}"
            assert int(st["cont_len"]) == r["cont_len"], f"seg {si} {st} vs {r}"
    # payload bytes
    ref = np.frombuffer(ora.inplace, dtype=np.uint8)
    if piece is not None:   # the streamed piece is unmasked with the frame's mask from its payload start
        lo = int(piece["hdr_off"]) + int(piece["hdr_len"]) - seg_start
        ref = xor_phased(ref.copy(), lo, lo + K.frame_len(piece), int(piece["mask"]))
        if compact:
            fr = res.frames[fb:fb + fc + 1]
            fc += 1
    if not compact:
        got = wire_after[seg_start:seg_start + len(stream)]
        if not np.array_equal(got, ref):
            bad = np.nonzero(got != ref)[0]
            raise AssertionError(f"seg {si}: in-place bytes differ at {bad[:10]} (n={len(bad)})")
    else:
        for i in range(fc):
            d = fr[i]
            if int(d["flags"]) & K.FF_UNMASKED and K.frame_len(d):
                p = int(d["hdr_off"]) + int(d["hdr_len"]) - seg_start
                L = K.frame_len(d)
                dst = int(res.frame_dst[fb + i])
                assert np.array_equal(res.arena[dst:dst + L], ref[p:p + L]), f"seg {si} frame {i} arena"


def events_of_session(sess, conn):
    return [(e.type, e.msg_id, e.opcode, e.close_code, e.err, e.data) for e in sess.events(conn)]
