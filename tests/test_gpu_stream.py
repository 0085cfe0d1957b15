"""Payloads streamed across batches (ABI 3; VERDICT r2 "next" #1, row A5).

The reference accumulates a frame's payload over any number of reads: nextFrame reads what is
there into rBuffer and completes the frame when its last byte has arrived
(server/websocket_frame.go:16-31, the XOR at :35-39 once complete).  The codec consumes a data
frame as its bytes arrive: each batch unmasks the payload bytes it holds (WSC_FK_PIECE records),
and the connection carries only {frame_rem, frame_mask, frame_hdr, frame_len, UTF-8 state} to its
next segment -- never the bytes.  Parity here: a connection's stream cut into 3 device batches at
every 4 KiB boundary (and at header bytes) gives, after merging each frame's pieces, exactly the
oracle's frame log on the whole stream, the same unmasked bytes, terminal status and carried state;
through wsc_session, frames far larger than a batch are delivered as the oracle delivers them and
every wire byte crosses H2D once.
"""
import numpy as np
import pytest

import oracle_ref as O
from fuzz_streams import random_stream
from gpu_helpers import events_of_session, header_len, xor_phased
from netman_amd import codec as K
from netman_amd import synth

pytestmark = pytest.mark.gpu


def _text(rng, n):
    """n bytes of valid UTF-8 (1-4 byte characters, ASCII tail)"""
    u = synth.utf8_units(rng, n // 4)
    return bytes(u) + b"a" * (n - len(u))


def decode_in_parts(codec, streams, cuts, compact=False):
    """Decode every connection's stream in len(cuts[i]) + 1 device batches, as the session would:
    segment k of a connection = the bytes batch k-1 left unconsumed (an incomplete header or control
    frame) + the next part; its state chained through state_in / state_out.  Returns per connection
    (merged records with stream offsets -- a streamed frame's pieces merged into one record --,
    the stream as the device left it (payload bytes unmasked), bytes consumed, final status
    (status, close_code, err), final state, the open frame if the stream ended inside one)."""
    n = len(streams)
    parts = [np.split(np.frombuffer(s, np.uint8), c) for s, c in zip(streams, cuts)]
    n_batches = max(len(p) for p in parts)
    carry = [b""] * n
    base = [0] * n                      # stream offset of the connection's next segment
    state = None
    out = [bytearray(s) for s in streams]
    merged = [[] for _ in range(n)]
    open_ = [None] * n
    final = [None] * n
    for k in range(n_batches):
        segs = [carry[i] + (parts[i][k].tobytes() if k < len(parts[i]) else b"") for i in range(n)]
        off = np.zeros(n + 1, np.uint64)
        np.cumsum([len(x) for x in segs], out=off[1:])
        wire = np.frombuffer(b"".join(segs), np.uint8).copy() if off[-1] else np.zeros(16, np.uint8)
        res = codec.decode_host(wire, off, state_in=state, compact=compact)
        assert K.Codec.summary_status(res.summary) == K.WSC_OK
        for i in range(n):
            sr = res.seg[i]
            a = int(off[i])
            cons = int(sr["consumed"])
            fb, fc = int(sr["frame_begin"]), int(sr["frame_count"])
            for j in range(fb, fb + fc):
                r = res.frames[j]
                L = K.frame_len(r)
                so = base[i] + int(r["hdr_off"]) - a          # stream offset of the record
                p = so + int(r["hdr_len"])                    # ... of its payload
                if int(r["flags"]) & K.FF_UNMASKED and L:
                    src = (res.arena[int(res.frame_dst[j]):int(res.frame_dst[j]) + L] if compact
                           else wire[a + (p - base[i]):a + (p - base[i]) + L])
                    out[i][p:p + L] = src.tobytes()
                d = {f: int(r[f]) for f in ("kind", "opcode", "fin", "mode", "msg_id", "err", "hdr_len", "mask", "flags")}
                d["hdr_off"], d["len"] = so, L
                if d["flags"] & K.FF_HEAD_PREV:
                    o = open_[i]
                    assert o is not None and d["hdr_len"] == 0, (i, k, d, o)
                    assert d["mask"] == o["next_mask"], (i, k, d, o)
                    o["len"] += L
                    o["next_mask"] = ((o["next_mask"] >> (8 * (L & 3))) | (o["next_mask"] << (32 - 8 * (L & 3)))) & 0xFFFFFFFF
                    if d["kind"] != K.FK_PIECE:
                        for f in ("opcode", "fin", "mode", "msg_id"):
                            assert d[f] == o[f], (i, k, f, d, o)
                        o.update(kind=d["kind"], err=d["err"])
                        merged[i].append(o)
                        open_[i] = None
                elif d["kind"] == K.FK_PIECE:
                    assert open_[i] is None and j == fb + fc - 1, (i, k, d)
                    d["next_mask"] = ((d["mask"] >> (8 * (L & 3))) | (d["mask"] << (32 - 8 * (L & 3)))) & 0xFFFFFFFF
                    open_[i] = d
                else:
                    merged[i].append(d)
            if not compact:   # in place: the segment's consumed bytes as the device left them
                out[i][base[i]:base[i] + cons] = wire[a:a + cons].tobytes()
            carry[i] = segs[i][cons:]
            base[i] += cons
            if final[i] is None and int(sr["status"]) != K.SEG_OPEN:
                final[i] = (int(sr["status"]), int(sr["close_code"]), int(sr["err"]))
        state = res.state.copy()
    return [dict(frames=merged[i], out=bytes(out[i]), consumed=base[i], final=final[i], state=state[i],
                 open=open_[i]) for i in range(n)]


def check_against_oracle(stream, got, ora):
    of = ora.frames
    fr = got["frames"]
    assert len(fr) == len(of), f"{len(fr)} device frames vs {len(of)} oracle frames\n{fr[-3:]}\n{of[-3:]}"
    for d, o in zip(fr, of):
        ctx = f"dev={d} ora={o}"
        assert d["hdr_off"] == int(o["hdr_off"]), ctx
        for f in ("kind", "opcode", "fin", "mode", "msg_id", "err"):
            assert d[f] == int(o[f]), f + " " + ctx
        if d["kind"] != K.FK_STALL and d["err"] != K.ERR_RSV_FAIL:
            assert d["len"] == int(o["payload_len"]) and d["mask"] == int(o["mask"]), ctx
            assert d["hdr_off"] + d["hdr_len"] == int(o["payload_off"]), ctx
    r = ora.res
    if r["closed"]:
        assert got["final"] is not None and got["final"][1:] == (r["close_code"], r["err"]), (got["final"], r)
    elif r["stalled"]:
        assert got["final"] is not None and got["final"][0] == K.SEG_STALLED
    else:
        assert got["final"] is None, got["final"]
        st = got["state"]
        assert int(st["msg_id"]) == r["msg_id"] and int(st["message_mode"]) == r["message_mode"], (st, r)
        assert int(st["cont_len"]) == r["cont_len"], (st, r)
    # bytes: what the oracle unmasked, plus -- for a frame still arriving -- its arrived payload
    ref = np.frombuffer(ora.inplace, np.uint8).copy()
    o = got["open"]
    if o is not None and got["final"] is None:
        lo = o["hdr_off"] + o["hdr_len"]
        xor_phased(ref, lo, lo + o["len"], o["mask"])
        hl, plen = header_len(stream, o["hdr_off"])
        st = got["state"]
        assert int(st["frame_rem"]) == plen - o["len"] and int(st["frame_len"]) == plen, (st, o)
        assert int(st["frame_hdr"]) == stream[o["hdr_off"]] & 0x8F
    c = got["consumed"]
    dev = np.frombuffer(got["out"], np.uint8)
    if not np.array_equal(dev[:c], ref[:c]):
        bad = np.nonzero(dev[:c] != ref[:c])[0]
        raise AssertionError(f"unmasked bytes differ at {bad[:10]} (n={len(bad)}) of {c}")


def _streams(seed):
    rng = np.random.default_rng(seed)
    big_text = synth.frame(1, _text(rng, 200_000), mask=0x1A2B3C4D)
    bad = bytearray(_text(rng, 150_000))
    bad[-1000] = 0xFF                                          # invalid near the end: 1007 at completion
    frag = (synth.frame(2, rng.bytes(70_000), fin=False, mask=0x01020304) + synth.frame(9, b"ping", mask=7)
            + synth.frame(0, rng.bytes(50_001), fin=False, mask=0x05060708)
            + synth.frame(0, rng.bytes(33_333), fin=True, mask=0x090A0B0C) + synth.frame(1, "ok ✓".encode()))
    tfrag = (synth.frame(1, _text(rng, 40_000), fin=False, mask=0x11111111) + synth.frame(0, b"", fin=False)
             + synth.frame(0, _text(rng, 60_002), fin=False, mask=0x22222222)
             + synth.frame(0, _text(rng, 9_001), fin=True, mask=0x33333333))
    small = b"".join(synth.frame(2, rng.bytes(1024), mask=int(rng.integers(0, 2**32))) for _ in range(64))
    fuzz = random_stream(seed + 1, n_units=20, big_p=0.2, text_p=0.5, err_p=0.0)
    return [big_text + synth.frame(2, b"after", mask=9), synth.frame(1, bytes(bad), mask=0x77777777) + b"\x82",
            frag, tfrag, small, fuzz]


@pytest.mark.parametrize("compact,inline_max", [(False, 256), (True, 256), (False, 0), (True, 0)])
def test_cut_at_every_4k_boundary_across_3_batches(codec_lib, monkeypatch, compact, inline_max):
    """every base stream as many connections, connection j cut at 4096 * (j + 1) and 36 KiB later
    (so every 4 KiB boundary is a cut of some connection), 3 device batches; inline_max 0 sends
    every text piece to the chip-wide UTF-8 path"""
    monkeypatch.setitem(K.CFG_DEFAULTS, "u8_inline_max", inline_max)
    c = K.Codec(0, max_batch_bytes=64 << 20, max_segs=1 << 12, max_frames=1 << 17)
    try:
        streams, cuts, refs = [], [], []
        for si, s in enumerate(_streams(31)):
            ora = O.run(s, cap=1 << 14)
            for j in range(len(s) // 4096):
                c1 = 4096 * (j + 1)
                streams.append(s)
                cuts.append([c1, min(len(s), c1 + 36 * 1024)])
                refs.append((si, ora))
        got = decode_in_parts(c, streams, cuts, compact=compact)
        for i, (g, (si, ora)) in enumerate(zip(got, refs)):
            try:
                check_against_oracle(streams[i], g, ora)
            except AssertionError as e:
                raise AssertionError(f"stream {si}, cuts {cuts[i]}: {e}") from None
    finally:
        c.close()


@pytest.mark.parametrize("compact", [False, True])
def test_cut_inside_headers_and_pieces(codec_lib, compact):
    """cuts at every byte of the first 20 bytes of a 14-byte-header frame and at odd offsets inside
    its payload (the mask phase of a piece that starts at 1, 2, 3 mod 4), 3 batches"""
    rng = np.random.default_rng(3)
    s = (synth.frame(2, rng.bytes(3), mask=0x0F0E0D0C) + synth.frame(1, _text(rng, 70_001), mask=0xA1B2C3D4)
         + synth.frame(2, rng.bytes(10), mask=0x55AA55AA))
    ora = O.run(s)
    streams, cuts = [], []
    for a in range(1, 30):
        for b in (a + 1, a + 2, a + 3, a + 4097, len(s) - 17, len(s) - 1):
            if a < b < len(s):
                streams.append(s)
                cuts.append([a, b])
    c = K.Codec(0, max_batch_bytes=64 << 20, max_segs=1 << 12, max_frames=1 << 14)
    try:
        for i, g in enumerate(decode_in_parts(c, streams, cuts, compact=compact)):
            try:
                check_against_oracle(s, g, ora)
            except AssertionError as e:
                raise AssertionError(f"cuts {cuts[i]}: {e}") from None
    finally:
        c.close()


def test_frame_larger_than_any_batch_is_streamed(codec_lib):
    """a 3 MiB BIN frame, a 5 MiB TEXT frame and a fragmented 2 MiB TEXT message through 1 MiB
    batches (the 1 MiB segments each hold one piece): same records and bytes as the oracle"""
    rng = np.random.default_rng(8)
    s = (synth.frame(2, rng.bytes(3 << 20), mask=0x01020304) + synth.frame(1, _text(rng, 5 << 20), mask=0x0A0B0C0D)
         + synth.frame(1, _text(rng, 1 << 20), fin=False, mask=0x13572468)
         + synth.frame(0, _text(rng, (1 << 20) + 3), fin=True, mask=0x24681357) + synth.frame(2, b"end"))
    ora = O.run(s, cap=64)
    step = 1 << 20
    cuts = [list(range(step, len(s), step))]
    c = K.Codec(0, max_batch_bytes=step + 4096, max_segs=16, max_frames=1024)
    try:
        got = decode_in_parts(c, [s], cuts)
        check_against_oracle(s, got[0], ora)
    finally:
        c.close()


# ---- through the session (the DecodePacket mirror) --------------------------------------------
def _feed_chunks(sess, conns, streams, chunk):
    got = {c: [] for c in conns}
    pos = [0] * len(streams)
    while any(p < len(s) for p, s in zip(pos, streams)):
        for i, (c, s) in enumerate(zip(conns, streams)):
            if pos[i] < len(s):
                sess.feed(c, s[pos[i]:pos[i] + chunk])
                pos[i] += chunk
        sess.decode()
        for c in conns:
            got[c].extend(events_of_session(sess, c))
    return got


@pytest.mark.parametrize("compact", [False, True])
def test_session_streams_frames_larger_than_a_batch(codec_lib, compact):
    """a 3 MiB frame and a 100 MiB TEXT frame fed in 64 KiB chunks through a 1 MiB-batch
    session give exactly the oracle's events (O.run on the whole stream); ordinary connections
    decode beside them; each wire byte crosses H2D once (only incomplete headers are re-sent)"""
    rng = np.random.default_rng(11)
    huge = synth.frame(2, rng.bytes(3 << 20), mask=0x01020304) + synth.frame(2, b"after", mask=5)
    text100 = synth.frame(1, _text(rng, 1 << 20) * 100, mask=0x0A0B0C0D) + synth.frame(1, "done ✓".encode(), mask=6)
    bad = bytearray(_text(rng, 2 << 20))
    bad[(1 << 20) + 5] = 0xC0                                 # invalid in the middle: 1007 at completion
    badtext = synth.frame(1, bytes(bad), mask=0x0BADF00D) + synth.frame(2, b"never")
    normal = [random_stream(22000 + i, n_units=20) for i in range(8)]
    streams = [huge, text100, badtext] + normal
    sess = K.Session(0, compact=compact, max_batch_bytes=1 << 20, max_segs=64, max_frames=1 << 14)
    conns = [sess.open() for _ in streams]
    got = _feed_chunks(sess, conns, streams, 64 << 10)
    for i, (c, s) in enumerate(zip(conns, streams)):
        ref = [e.key() for e in O.run(s, cap=1 << 12).events]
        assert len(got[c]) == len(ref) and all(a == b for a, b in zip(got[c], ref)), \
            f"stream {i}: {[(e[0], e[1], len(e[5])) for e in got[c][:4]]} vs {[(e[0], e[1], len(e[5])) for e in ref[:4]]}"
    assert len(got[conns[1]][0][5]) == 100 << 20 and got[conns[2]][-1][3] == 1007
    st = sess.stats()
    # every byte read went to the device once, plus the carried incomplete headers / control frames
    # (bytes fed to a connection after its close are not read)
    assert st["h2d"] == st["read"] + st["resent"], st
    assert st["resent"] <= 139 * len(streams) * st["batches"], st
    assert st["pieces"] >= (100 << 20), st
    sess.close()


def test_session_h2d_once_for_streamed_payloads(codec_lib):
    """byte accounting alone: one 20 MiB BIN frame in 4 KiB reads through 64 KiB batches -- no byte
    of it is sent twice (before streaming, a partial frame's bytes were re-sent every batch)"""
    rng = np.random.default_rng(12)
    s = synth.frame(2, rng.bytes(20 << 20), mask=0x31415926)
    sess = K.Session(0, max_batch_bytes=64 << 10, max_segs=8, max_frames=256)
    c = sess.open()
    got = _feed_chunks(sess, [c], [s], 4096)
    assert len(got[c]) == 1 and got[c][0][5] == bytes(synth.unmask_reference(
        np.frombuffer(s, np.uint8), np.array([14], np.uint64), np.array([20 << 20], np.uint64),
        np.array([0x31415926], np.uint32))[14:])
    st = sess.stats()
    assert st["read"] == len(s) and st["h2d"] == len(s) and st["resent"] == 0, st
    sess.close()


@pytest.mark.parametrize("compact", [False, True])
def test_tiled_walk_simple_segment_tiles(codec_lib, monkeypatch, compact):
    """The tiled walk's simple-segment path (a segment that is exactly one complete plain BIN frame
    of an idle connection: no second walk, outputs straight from the cached header).  2,000
    connections over 4 device batches, cut at frame edges: connections 0..767 send one BIN frame per
    batch (whole tiles of simple segments, carried msgIDs > 0 from the second batch on; payloads of
    1..125 B, 126..65535 B and > 64 KiB: 6, 8 and 14-byte headers), the others mix in empty BIN
    frames, two frames per segment, TEXT and fragmented messages, and cuts inside a frame -- so tiles
    of the same batch take both paths.  Every connection equals the oracle on its whole stream."""
    monkeypatch.setitem(K.CFG_DEFAULTS, "walk_mode", 3)
    rng = np.random.default_rng(606)
    sizes = [1, 5, 125, 126, 1000, 4093, 65535, 65536, 70001]
    streams, cuts = [], []
    for i in range(2000):
        frames = []
        for k in range(4):
            if i < 768:
                frames.append([synth.frame(2, bytes(rng.integers(0, 256, int(rng.choice(sizes)), dtype=np.uint8)), rng=rng)])
                continue
            r = rng.random()
            if r < 0.2:
                frames.append([synth.frame(2, b"", rng=rng)])
            elif r < 0.4:
                frames.append([synth.frame(2, b"ab", rng=rng), synth.frame(2, b"cde", rng=rng)])
            elif r < 0.6:
                frames.append([synth.frame(1, "ü".encode() * int(rng.integers(1, 200)), rng=rng)])
            elif r < 0.8:
                frames.append([synth.frame(2, b"x" * 300, fin=False, rng=rng), synth.frame(0, b"y" * 20, rng=rng)])
            else:
                frames.append([synth.frame(2, bytes(int(rng.integers(1, 3000))), rng=rng)])
        parts = [b"".join(f) for f in frames]
        s = b"".join(parts)
        c = list(np.cumsum([len(p) for p in parts])[:-1])
        if i >= 768 and rng.random() < 0.2:   # a cut inside a frame: that segment streams a piece
            c[1] = c[1] - int(rng.integers(1, 5))
        streams.append(s)
        cuts.append(c)
    c = K.Codec(0, max_batch_bytes=64 << 20, max_segs=1 << 12, max_frames=1 << 16)
    try:
        got = decode_in_parts(c, streams, cuts, compact=compact)
        assert c.walk_info()[0] == 3
        for i, (g, s) in enumerate(zip(got, streams)):
            try:
                check_against_oracle(s, g, O.run(s))
            except AssertionError as e:
                raise AssertionError(f"stream {i}: {e}") from None
    finally:
        c.close()
