"""PONG payloads streamed across batches, the session's no-progress guard, and EOF ordering
(VERDICT r3 items 1 and 2).

PONG (row A8): the reference puts no size limit on a PONG (server/websocket.go:191-205) and
nextFrame accumulates its payload over any number of reads (websocket_frame.go:16-31); under an
open TEXT message the PONG payload alone is UTF-8 checked when complete (websocket_frame.go:71,
Q6) and the PONG counts in msgID (Q5).  Until ABI 4 the codec waited for a control frame whole,
so a PONG longer than a batch re-sent the same prefix forever.  Here every PONG streams like a
data frame and the result equals O.run on the whole stream.

EOF (row A10): BaseConnect.Read maps a 0-byte read to io.EOF (baseconnect.go:100-103), which the
poller turns into Close() (epoll.go:108-110) -- after every frame read before it was delivered.
wsc_session_eof keeps that order; O.run(..., eof=True) is the reference's sequence.
"""
import numpy as np
import pytest

import oracle_ref as O
from fuzz_streams import random_stream
from gpu_helpers import events_of_session
from netman_amd import codec as K
from netman_amd import synth
from test_gpu_stream import check_against_oracle, decode_in_parts

pytestmark = pytest.mark.gpu


def _text(rng, n):
    """n bytes of valid UTF-8 (1-4 byte characters, ASCII tail)"""
    u = synth.utf8_units(rng, n // 4)
    return bytes(u) + b"a" * (n - len(u))


def _pong_streams(seed):
    rng = np.random.default_rng(seed)
    big = synth.frame(2, b"first", mask=1) + synth.frame(10, rng.bytes(2 << 20), mask=0x0A0B0C0D) \
        + synth.frame(2, b"after", mask=2)
    p300 = synth.frame(10, bytes(rng.integers(0x20, 0x7F, 300, dtype=np.uint8)), mask=0x01020304) \
        + synth.frame(1, "ok ✓".encode(), mask=3)
    # inside an open TEXT message (Q6): a valid text PONG, then the message completes
    tv = (synth.frame(1, _text(rng, 1000), fin=False, mask=0x11111111)
          + synth.frame(10, _text(rng, 300_000), mask=0x22222222)
          + synth.frame(0, _text(rng, 500), fin=True, mask=0x33333333) + synth.frame(2, b"tail", mask=4))
    # ... and one with an invalid byte in its middle: 1007 when the PONG completes
    bad = bytearray(_text(rng, 300_000))
    bad[150_007] = 0xFF
    ti = (synth.frame(1, _text(rng, 100), fin=False, mask=0x44444444) + synth.frame(10, bytes(bad), mask=0x55555555)
          + synth.frame(0, b"never", fin=True, mask=6))
    # a PONG outside any message may hold anything (binary payload, no check)
    free = synth.frame(10, rng.bytes(70_000), mask=0x66666666) + synth.frame(2, rng.bytes(10), mask=7)
    # a 4-byte character of the PONG split across a batch boundary under TEXT mode
    pre = _text(rng, 4093)
    split = (synth.frame(1, b"x", fin=False, mask=8) + synth.frame(10, pre + "😀".encode() + b"z" * 10, mask=0x77777777)
             + synth.frame(0, b"y", fin=True, mask=9))
    fuzz = random_stream(seed + 1, n_units=30, text_p=0.5, err_p=0.0, pong_big_p=0.2)
    return [big, p300, tv, ti, free, split, fuzz]


@pytest.mark.parametrize("compact,inline_max", [(False, 256), (True, 256), (False, 0), (True, 0)])
def test_pong_streams_across_batches(codec_lib, monkeypatch, compact, inline_max):
    """every stream cut into 3 device batches at many offsets (inside PONG headers and payloads,
    at odd mask phases, one byte into a 4-byte character); inline_max 0 sends every text piece --
    the PONG's too -- to the chip-wide UTF-8 path"""
    monkeypatch.setitem(K.CFG_DEFAULTS, "u8_inline_max", inline_max)
    c = K.Codec(0, max_batch_bytes=64 << 20, max_segs=1 << 12, max_frames=1 << 16)
    try:
        streams, cuts, refs = [], [], []
        for si, s in enumerate(_pong_streams(41)):
            ora = O.run(s, cap=1 << 14)
            n = len(s)
            pts = sorted(set([1, 5, 7, 13, 14, 15, 16, 300, 301, 4099, 4100, 4101, 4102, 65537]
                             + [int(x) for x in np.linspace(17, n - 2, 24)]))
            for a in pts:
                if 0 < a < n - 1:
                    b = min(n - 1, a + 1 + (a * 7919) % 200_000)
                    streams.append(s)
                    cuts.append([a, b] if b > a else [a])
                    refs.append((si, ora))
        got = decode_in_parts(c, streams, cuts, compact=compact)
        for i, (g, (si, ora)) in enumerate(zip(got, refs)):
            try:
                check_against_oracle(streams[i], g, ora)
            except AssertionError as e:
                raise AssertionError(f"stream {si}, cuts {cuts[i]}: {e}") from None
    finally:
        c.close()


def test_pong_piece_carries_its_utf8_state(codec_lib, monkeypatch):
    """the PONG's own DFA state (frame_utf8) is carried between batches while the message's
    (cont_utf8) is kept apart: cut one byte into a 4-byte character of the PONG"""
    monkeypatch.setitem(K.CFG_DEFAULTS, "u8_inline_max", 256)
    s = _pong_streams(41)[5]
    pong_at = len(synth.frame(1, b"x", fin=False, mask=8))
    cut = pong_at + 8 + 4093 + 1                         # 1 byte into the 4-byte character
    c = K.Codec(0, max_batch_bytes=1 << 20, max_segs=16, max_frames=1024)
    try:
        wire = np.frombuffer(s[:cut], np.uint8).copy()
        res = c.decode_host(wire, np.array([0, cut], np.uint64))
        st = res.state[0]
        assert int(st["frame_hdr"]) == 0x8A and int(st["frame_rem"]) == 3 + 10   # 3 bytes of the character + "z" * 10
        assert int(st["frame_utf8"]) != 0                 # inside a character
        assert int(st["message_mode"]) == 1 and int(st["cont_utf8"]) == 0
        got = decode_in_parts(c, [s], [[cut]])[0]
        check_against_oracle(s, got, O.run(s))
    finally:
        c.close()


# ---- through the session ------------------------------------------------------------------------
def _feed_chunks(sess, conns, streams, chunk, eof=False, pipelined=False, max_rounds=10_000):
    got = {c: [] for c in conns}
    pos = [0] * len(streams)
    for _ in range(max_rounds):
        fed = False
        for i, (c, s) in enumerate(zip(conns, streams)):
            if pos[i] < len(s):
                sess.feed(c, s[pos[i]:pos[i] + chunk])
                pos[i] += chunk
                fed = True
                if eof and pos[i] >= len(s):
                    sess.eof(c)                  # the last read is followed by read() == 0
        if pipelined:
            sess.submit()
            for c in conns:
                got[c].extend(events_of_session(sess, c))
            sess.complete()
        else:
            sess.decode()
        for c in conns:
            got[c].extend(events_of_session(sess, c))
        if not fed and sess.pending() == 0:
            if pipelined:
                sess.submit()
                sess.complete()
                for c in conns:
                    got[c].extend(events_of_session(sess, c))
            return got
    raise AssertionError("the session did not drain (livelock)")


@pytest.mark.parametrize("compact,pipelined", [(False, False), (True, False), (False, True)])
def test_session_streams_pongs_larger_than_a_batch(codec_lib, compact, pipelined):
    """a 2 MiB PONG, a 2 MiB PONG with an invalid byte inside an open TEXT message
    (1007), and a 300 B PONG cut across two batches, through a 1 MiB-batch session in 64 KiB reads
    (the pipelined poller's submit / complete cycle too): exactly the oracle's events, and every
    wire byte crosses H2D once (re-sent: only incomplete headers and PING / CLOSE frames)"""
    rng = np.random.default_rng(12)
    pong2 = synth.frame(10, rng.bytes(2 << 20), mask=0x01020304) + synth.frame(2, b"after", mask=5)
    bad = bytearray(_text(rng, 2 << 20))
    bad[(1 << 20) + 3] = 0xC0
    pong_bad = (synth.frame(1, _text(rng, 5000), fin=False, mask=0x0A0B0C0D) + synth.frame(10, bytes(bad), mask=0x0BADF00D)
                + synth.frame(0, b"never", fin=True))
    good = bytes(_text(rng, 2 << 20))
    pong_good = (synth.frame(1, _text(rng, 5000), fin=False, mask=0x13572468) + synth.frame(10, good, mask=0x24681357)
                 + synth.frame(0, _text(rng, 70_000), fin=True, mask=0x11223344) + synth.frame(2, b"end", mask=9))
    pad = 64 * 1024 - 200
    p300 = (synth.frame(2, rng.bytes(pad - 6 - 4), mask=1)         # the PONG straddles the first 64 KiB read
            + synth.frame(10, bytes(rng.integers(0x20, 0x7F, 300, dtype=np.uint8)), mask=0x0F0E0D0C)
            + synth.frame(1, "done ✓".encode(), mask=6))
    mixed = [random_stream(31000 + i, n_units=30, pong_big_p=0.25, text_p=0.5) for i in range(8)]
    streams = [pong2, pong_bad, pong_good, p300] + mixed
    sess = K.Session(0, compact=compact, max_batch_bytes=1 << 20, max_segs=64, max_frames=1 << 14)
    conns = [sess.open() for _ in streams]
    got = _feed_chunks(sess, conns, streams, 64 << 10, pipelined=pipelined)
    for i, (c, s) in enumerate(zip(conns, streams)):
        ref = [e.key() for e in O.run(s, cap=1 << 12).events]
        assert got[c] == ref, f"stream {i}: {[(e[0], e[3], len(e[5])) for e in got[c][:6]]} vs " \
                              f"{[(e[0], e[3], len(e[5])) for e in ref[:6]]}"
    assert [e[0] for e in got[conns[0]]] == [K.EV_MESSAGE] and got[conns[0]][0][5] == b"after"
    assert got[conns[1]][-1][:5] == (K.EV_CLOSE, 0, 0, 1007, K.ERR_MUST_UTF8)
    st = sess.stats()
    assert st["h2d"] == st["read"] + st["resent"], st
    assert st["resent"] <= 139 * len(streams) * st["batches"], st
    sess.close()


def test_no_progress_guard_closes_instead_of_livelock(codec_lib):
    """max_batch_bytes 64 (the smallest allowed): a PING of 100 B can never fit a batch -- the
    connection is closed with 1009 / WSC_ERR_NO_PROGRESS at once (before ABI 4 wsc_session_decode
    re-sent the prefix 2^20 times); a 1000 B PONG on another connection streams through the 64 B
    batches and the message after it is delivered"""
    sess = K.Session(0, max_batch_bytes=64, max_segs=8, max_frames=64)
    a, b = sess.open(), sess.open()
    sess.feed(a, synth.frame(9, b"p" * 100, mask=3) + synth.frame(2, b"unreached", mask=4))
    pong = synth.frame(10, bytes(range(256)) * 4, mask=0x01020304) + synth.frame(2, b"after the pong", mask=5)
    sess.feed(b, pong)
    sess.decode()
    ea = events_of_session(sess, a)
    assert [e[:5] for e in ea] == [(K.EV_CLOSE, 0, 0, 1009, K.ERR_NO_PROGRESS)]
    eb = events_of_session(sess, b)
    assert eb == [e.key() for e in O.run(pong).events] and eb[0][5] == b"after the pong"
    assert sess.pending() == 0
    st, _ = sess.state(a)
    assert st.status == K.SEG_ERROR
    sess.close()


def test_max_message_cap(codec_lib):
    """wsc_session_set_max_message (off by default, like the reference): a message, or the
    fragments / streamed pieces of one, past the cap closes with 1009 / WSC_ERR_MSG_TOO_BIG;
    messages up to the cap and other connections are untouched"""
    rng = np.random.default_rng(3)
    sess = K.Session(0, max_batch_bytes=1 << 20, max_segs=16, max_frames=1024)
    sess.set_max_message(100_000)
    a, b, c = sess.open(), sess.open(), sess.open()
    ok = synth.frame(2, rng.bytes(100_000), mask=1)
    sess.feed(a, ok + synth.frame(2, rng.bytes(100_001), mask=2) + synth.frame(2, b"x"))
    sess.feed(b, synth.frame(2, rng.bytes(60_000), fin=False, mask=3) + synth.frame(0, rng.bytes(60_000), mask=4))
    sess.feed(c, synth.frame(2, rng.bytes(3 << 20), mask=5))       # streamed: its pieces pass the cap
    sess.decode()
    ea = events_of_session(sess, a)
    assert [e[0] for e in ea] == [K.EV_MESSAGE, K.EV_CLOSE] and len(ea[0][5]) == 100_000
    assert ea[1][3:5] == (1009, K.ERR_MSG_TOO_BIG)
    assert [e[3:5] for e in events_of_session(sess, b)] == [(1009, K.ERR_MSG_TOO_BIG)]
    for _ in range(4):
        sess.decode()
    assert [e[3:5] for e in events_of_session(sess, c)] == [(1009, K.ERR_MSG_TOO_BIG)]
    sess.close()


# ---- EOF ----------------------------------------------------------------------------------------
@pytest.mark.parametrize("pipelined", [False, True])
def test_eof_delivers_queued_messages_first(codec_lib, pipelined):
    """a client sends its frames then closes.  The session delivers every message
    read before the EOF -- including those of the last read, decoded after eof() was called, and
    frames streamed over several batches -- and only then Close() (1000, err 0), exactly as
    O.run(stream, eof=True); an incomplete frame at the EOF is dropped (the reference's read of
    it returns io.EOF)"""
    rng = np.random.default_rng(77)
    streams = [random_stream(32000 + i, n_units=25, pong_big_p=0.1) for i in range(24)]
    streams += [synth.frame(2, rng.bytes(3 << 20), mask=7) + synth.frame(1, b"last", mask=8),        # streamed
                synth.frame(2, b"a", mask=1) + synth.frame(2, rng.bytes(5000), mask=2)[:3000],       # torn frame
                synth.frame(2, b"b", mask=1) + b"\x82",                                             # torn header
                b"",                                                                                # nothing
                synth.frame(2, b"c", mask=1) + synth.frame(8, b"\x03\xe8", mask=3) + synth.frame(2, b"d")]  # CLOSE first
    sess = K.Session(0, max_batch_bytes=1 << 20, max_segs=64, max_frames=1 << 14)
    conns = [sess.open() for _ in streams]
    empty = conns[len(streams) - 2]
    sess.eof(empty)                                           # EOF with nothing read: Close() at once
    got = _feed_chunks(sess, conns, streams, 48 << 10, eof=True, pipelined=pipelined)
    for i, (c, s) in enumerate(zip(conns, streams)):
        ref = [e.key() for e in O.run(s, cap=1 << 12, eof=True).events]
        assert got[c] == ref, f"stream {i}: {[(e[0], e[3]) for e in got[c][-3:]]} vs {[(e[0], e[3]) for e in ref[-3:]]}"
        assert got[c][-1][0] in (K.EV_CLOSE, K.EV_STALL)   # (Q3: an unmasked frame stalls first)
    # after its Close() a connection delivers nothing more and reads nothing
    sess.feed(conns[0], synth.frame(2, b"late"))
    sess.decode()
    assert events_of_session(sess, conns[0]) == []
    sess.close()


@pytest.mark.parametrize("in_flight", [False, True])
def test_eof_between_reserve_and_commit(codec_lib, in_flight):
    """round-4 ADVICE: reserve -> read() == 0 -> wsc_session_eof -> commit(0).  With the
    connection's earlier bytes in flight the reservation is a spill region; Close() must still
    come, after the messages (O.run(stream, eof=True))"""
    import ctypes as C
    sess = K.Session(0, max_batch_bytes=1 << 20, max_segs=16, max_frames=1024)
    a = sess.open()
    s = synth.frame(2, b"one", mask=1) + synth.frame(1, b"two", mask=2)
    sess.feed(a, s)
    got = []
    if in_flight:
        sess.submit()
    p, avail = C.c_void_p(), C.c_uint64()
    assert sess.lib.wsc_session_reserve(sess.h, a, 4096, C.byref(p), C.byref(avail)) == 0 and p.value
    sess.eof(a)
    assert sess.lib.wsc_session_commit(sess.h, a, 0) == 0
    if in_flight:
        sess.complete()
        got += events_of_session(sess, a)
    for _ in range(4):
        sess.decode()
        got += events_of_session(sess, a)
    assert got == [e.key() for e in O.run(s, cap=1 << 12, eof=True).events]
    assert got[-1][0] == K.EV_CLOSE
    sess.close()
