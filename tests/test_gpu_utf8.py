"""Chip-wide UTF-8 validation (k_u8_check) for text the walk defers: bit-exact against the oracle.

By default text payloads above 256 B are deferred; wsc_config.u8_inline_max = 0 sends EVERY text check through k_u8_check, so the fuzz corpus (fragmented text chains, multi-byte
characters split across fragments, PINGs inside text messages (Q6), close reasons, invalid
sequences) exercises the deferred path end to end, including chains that span batches.
Full-size: 64 KiB TEXT frames of 1-4 byte characters, valid and with injected errors."""
import os

import numpy as np
import pytest

import oracle_ref as O
from fuzz_streams import random_stream, random_splits
from gpu_helpers import pack_streams, compare_segment, events_of_session
from netman_amd import codec as K
from netman_amd import synth

pytestmark = pytest.mark.gpu


def _with_inline_max(v, make):
    old = K.CFG_DEFAULTS.get("u8_inline_max")
    K.CFG_DEFAULTS["u8_inline_max"] = v
    try:
        return make()
    finally:
        if old is None:
            del K.CFG_DEFAULTS["u8_inline_max"]
        else:
            K.CFG_DEFAULTS["u8_inline_max"] = old


@pytest.fixture(scope="module")
def codec_all_deferred(codec_lib):
    c = _with_inline_max(0, lambda: K.Codec(0, max_batch_bytes=64 << 20, max_segs=1 << 14, max_frames=1 << 18))
    yield c
    c.close()


def _check(codec, streams, compact=False):
    wire, off = pack_streams(streams)
    res = codec.decode_host(wire, off, compact=compact)
    assert int(res.summary["overflow"]) == 0
    for i, s in enumerate(streams):
        compare_segment(i, s, int(off[i]), res, O.run(s), wire_after=wire, compact=compact)
    return res


@pytest.mark.parametrize("compact", [False, True])
def test_text_heavy_fuzz_all_deferred(codec_all_deferred, compact):
    streams = [random_stream(7000 + i, n_units=30, text_p=0.9, err_p=0.03) for i in range(300)]
    _check(codec_all_deferred, streams, compact=compact)


def test_general_fuzz_all_deferred(codec_all_deferred):
    streams = [random_stream(8000 + i, n_units=int(5 + i % 40)) for i in range(400)]
    _check(codec_all_deferred, streams)


def test_golden_streams_all_deferred(codec_all_deferred):
    import golden_io
    streams = [b for _, b, _ in golden_io.aiohttp_cases()] + [b for _, b, _ in golden_io.kat_cases()]
    _check(codec_all_deferred, streams)


@pytest.mark.parametrize("inline_max", [0, 40])
def test_session_chains_across_batches_deferred(codec_lib, inline_max):
    """text chains whose parts arrive in different decodes: the deferred DFA state is carried"""
    rng = np.random.default_rng(11)
    sess = _with_inline_max(inline_max, lambda: K.Session(0, max_batch_bytes=16 << 20, max_segs=1024,
                                                          max_frames=1 << 16))
    streams = [random_stream(9500 + i, n_units=25, text_p=0.9, err_p=0.02) for i in range(150)]
    conns = [sess.open() for _ in streams]
    splits = [random_splits(rng, len(s), int(rng.integers(1, 6))) for s in streams]
    got = {c: [] for c in conns}
    prev = [0] * len(streams)
    for r in range(max(len(sp) for sp in splits)):
        for i, (c, s, sp) in enumerate(zip(conns, streams, splits)):
            if r < len(sp):
                sess.feed(c, s[prev[i]:sp[r]])
                prev[i] = sp[r]
        sess.decode()
        for c in conns:
            got[c].extend(events_of_session(sess, c))
    for i, (c, s) in enumerate(zip(conns, streams)):
        ref = [e.key() for e in O.run(s).events]
        assert got[c] == ref, f"stream {i}: {got[c][:4]} vs {ref[:4]}"
    sess.close()


def _unmask(cfg, i):
    p, L, m = int(cfg["payload_off"][i]), int(cfg["plen"][i]), int(cfg["mask"][i])
    mb = np.array([(m >> (8 * k)) & 0xFF for k in range(4)], np.uint8)
    return p, L, mb


@pytest.mark.parametrize("compact", [False, True])
def test_text_64k_frames_valid_and_invalid(codec_lib, compact):
    """1,024 connections x 4 x 64 KiB TEXT frames (chip-wide path by default: most bytes are folded
    by the unmask, the rest by k_u8_check); a 0xFF byte is injected into ~6 % of the frames: each
    connection must stop at its first bad frame with 1007, leave later frames masked (re-masked
    after the unmask, in place and in the COMPACT arena), and match the oracle record for record,
    byte for byte."""
    cfg = synth.text_batch(4096, 65536, 4, seed=synth.SEED_BASE + 31)
    rng = np.random.default_rng(5)
    bad = set(int(x) for x in rng.choice(4096, 256, replace=False))
    for i in bad:   # write 0xFF (never valid UTF-8) at a random payload position, masked
        p, L, mb = _unmask(cfg, i)
        q = int(rng.integers(0, L))
        cfg["wire"][p + q] = 0xFF ^ mb[q & 3]
    c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=2048, max_frames=8192)
    wire = cfg["wire"].copy()
    res = c.decode_host(wire, cfg["seg_off"], compact=compact)
    assert int(res.summary["overflow"]) == 0
    n_seg = len(cfg["seg_off"]) - 1
    for s in range(n_seg):
        a, b = int(cfg["seg_off"][s]), int(cfg["seg_off"][s + 1])
        compare_segment(s, bytes(cfg["wire"][a:b]), a, res, O.run(bytes(cfg["wire"][a:b])), wire_after=wire,
                        compact=compact)
    n_err = int((res.seg["status"] == K.SEG_ERROR).sum())
    assert n_err == len({i // 4 for i in bad}) and n_err > 0
    assert int(res.summary["n_frames"]) >= int(res.seg["frame_count"].sum())
    c.close()


def test_text_large_frames_cross_piece_characters(codec_lib):
    """frames larger than several unmask windows with multi-byte characters across window edges
    (folded by the unmask, partial windows by k_u8_check), plus a TEXT chain of big fragments where
    a 4-byte character straddles two fragments"""
    e = "😀".encode()                                        # 4 bytes
    body = ("ab" + "é" * 40000 + "x").encode()               # 80003 bytes, 2-byte chars across 65536
    body2 = b"a" * 65535 + e + b"z" * 100                    # emoji straddles a piece edge (65536)
    body3 = ("abc" + "é" * 30000).encode()                   # 2-byte chars straddle every 16 KiB edge
    frag = e * 30000                                         # 120000 B, cut inside a character
    s1 = synth.frame(1, body) + synth.frame(1, body2) + synth.frame(1, body3)
    s2 = synth.frame(1, frag[:70001], fin=False) + synth.frame(0, frag[70001:], fin=True)
    s3 = synth.frame(1, frag[:70001], fin=False) + synth.frame(0, frag[70001:-1], fin=True)   # truncated char
    s4 = synth.frame(8, (1000).to_bytes(2, "big") + ("ü" * 61).encode())   # close reason, 124 B
    c = _with_inline_max(0, lambda: K.Codec(0, max_batch_bytes=8 << 20, max_segs=64, max_frames=4096))
    streams = [s1, s2, s3, s4]
    wire, off = pack_streams(streams)
    res = c.decode_host(wire, off)
    for i, s in enumerate(streams):
        compare_segment(i, s, int(off[i]), res, O.run(s), wire_after=wire)
    assert [int(x) for x in res.seg["status"]] == [K.SEG_OPEN, K.SEG_OPEN, K.SEG_ERROR, K.SEG_CLOSED]
    c.close()


@pytest.mark.parametrize("compact", [False, True])
def test_text_1k_several_failures_per_connection(codec_lib, compact):
    """1 KiB TEXT frames (deferred single-piece messages, checked 4 per wave step in any order):
    connections with 1-3 bad frames each, and connections whose text chain (fragments of 300 B)
    fails after a bad single-piece frame or before one.  Failures of one connection are applied in
    whatever order the waves finish: each takes part only if it lowers the connection's first
    failure, re-masking just the spans between its frame and the previous minimum's -- the
    records, consumed bytes and bytes must equal the oracle's (first failure wins)."""
    rng = np.random.default_rng(17)
    good = ("ab" + "é" * 300 + "xyz" + "€" * 40).encode()[:1024]
    good = good + b"a" * (1024 - len(good))
    bad = bytearray(good)
    streams = []
    for i in range(2048):
        n = 16
        bad_at = set(int(x) for x in rng.choice(n, int(rng.integers(0, 4)), replace=False))
        parts = []
        for k in range(n):
            if k in bad_at:
                b = bytearray(good)
                b[int(rng.integers(0, 1024))] = 0xFF
                parts.append(synth.frame(1, bytes(b)))
            elif i % 5 == 0 and k == 8:   # a fragmented text message, maybe bad in its second piece
                frag = ("é" * 450).encode()
                f2 = bytearray(frag[300:])
                if i % 10 == 0:
                    f2[7] = 0xC0
                parts.append(synth.frame(1, frag[:300], fin=False) + synth.frame(0, bytes(f2), fin=True))
            else:
                parts.append(synth.frame(1, good))
        streams.append(b"".join(parts))
    c = K.Codec(0, max_batch_bytes=64 << 20, max_segs=4096, max_frames=1 << 16)
    try:
        res = _check(c, streams, compact=compact)
        assert int((res.seg["status"] == K.SEG_ERROR).sum()) > 0
    finally:
        c.close()


def test_rejected_geometry_leaves_utf8_counters_consistent(codec_lib, monkeypatch):
    """round-3 ADVICE (medium): a decode refused by the walk-geometry guard (walk_mode 16 with
    more segments than the look-back state holds) must not flip the UTF-8 item-counter parity nor
    commit its geometry -- the next decodes' chip-wide 1007 verdicts must stay exact"""
    monkeypatch.setitem(K.CFG_DEFAULTS, "walk_mode", 16)
    monkeypatch.setitem(K.CFG_DEFAULTS, "u8_inline_max", 0)
    c = K.Codec(0, max_batch_bytes=8 << 20, max_segs=1 << 15, max_frames=1 << 17)
    try:
        many = [synth.frame(2, b"x", mask=i) for i in range(1 << 15)]
        wire, off = pack_streams(many)
        with pytest.raises(K.WscError) as ei:
            c.decode_host(wire, off)
        assert ei.value.rc == K.WSC_E_INTERNAL
        rng = np.random.default_rng(5)
        for rnd in range(3):
            streams = [random_stream(9100 + 37 * rnd + i, n_units=20, text_p=0.9, err_p=0.05) for i in range(64)]
            bad = bytearray(synth.utf8_units(rng, 300)) + b"\xff"
            streams += [synth.frame(1, bytes(bad), mask=3) + synth.frame(2, b"after")] * 4
            _check(c, streams)
            if rnd == 0:   # a second refusal between good decodes
                with pytest.raises(K.WscError):
                    c.decode_host(wire, off)
    finally:
        c.close()


def _edge_batch(rng, bad, brng=None):
    """TEXT frames of 300..3000 B (multi-byte characters; deferred, no whole window: every byte is
    in an edge window) from 16 connections, so frames start and end at every offset of the 4 KiB
    unmask windows; `bad`: one 0xC0 byte per connection at a random place (often by an edge)"""
    streams = []
    for i in range(16):
        parts = []
        for _ in range(int(rng.integers(8, 20))):
            n = int(rng.integers(300, 3000))
            t = bytearray(("é€😀a" * (n // 10 + 1)).encode()[:n])
            while True:   # cut at a character boundary (valid text)
                try:
                    bytes(t).decode()
                    break
                except UnicodeDecodeError:
                    t = t[:-1]
            parts.append(t)
        if bad:
            br = brng if brng is not None else rng
            k = int(br.integers(0, len(parts)))
            parts[k][int(br.integers(0, len(parts[k])))] = 0xC0
        streams.append(b"".join(synth.frame(1, bytes(p)) for p in parts))
    return streams


def test_text_window_edges_alternating_layouts(codec_lib):
    """Deferred TEXT frames of 300..3000 B starting and ending at every offset of the 4 KiB unmask
    windows (every byte in a partial window: the check's head/tail path), the same window layout
    decoded valid then invalid, in place then COMPACT then in place on one context: every decode
    equals the oracle -- state a decode leaves in the context (window flags and maps) never lets a
    later decode's invalid text pass."""
    rng = np.random.default_rng(23)
    good = _edge_batch(np.random.default_rng(1), bad=False)
    c = K.Codec(0, max_batch_bytes=16 << 20, max_segs=256, max_frames=1 << 14)
    try:
        for compact in (False, True, False, False):
            for streams in (good, _edge_batch(np.random.default_rng(1), bad=True, brng=rng)):
                # the bad batch: same frames as `good` (same seed), one invalid byte per connection
                _check(c, streams, compact=compact)
        res = _check(c, _edge_batch(rng, bad=True))
        assert int((res.seg["status"] == K.SEG_ERROR).sum()) == 16
    finally:
        c.close()


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("inline_max", [256, 0])
def test_failed_single_piece_with_open_composite_zeroes_carried_state(codec_lib, compact, inline_max):
    """round-5 ADVICE: a segment whose single-piece TEXT message fails (1007, decided by k_u8_check's
    fast verdict) while composite items of the same segment are still open -- a TEXT fragment that
    ends inside a 4-byte character (cont_utf8 would be 3) or a PONG under TEXT cut inside a
    character (frame_utf8) -- must leave NO carried DFA state: status ERROR, cont_utf8 = frame_utf8 = 0.
    Many such segments in one batch, the failing frame placed before, between and after the open
    items, so the two verdict paths (per-item fail, per-segment compose) interleave every way."""
    emoji = "\U0001F600".encode()
    ok = ("ab" + "ü" * 300).encode()                      # > 256 B: deferred by default
    bad = bytearray(("x" * 600).encode())
    bad[333] = 0xFF
    frag_open = synth.frame(1, ok + emoji[:1], fin=False, mask=0x01020304)   # ends 1 byte into U+1F600
    pong_open = synth.frame(10, ok + emoji[:2], mask=0x0A0B0C0D)
    streams = []
    for k in range(96):
        failing = synth.frame(1, bytes(bad), mask=0x11223344 + k)
        if k % 3 == 0:
            s = failing + frag_open
        elif k % 3 == 1:
            s = synth.frame(1, ok, fin=False, mask=5) + synth.frame(0, bytes(bad), mask=6 + k) + frag_open
        else:
            # a TEXT message open (fragment), a PONG inside it cut in a character, the failing frame first
            s = failing + synth.frame(1, ok, fin=False, mask=7) + pong_open[:len(pong_open) - 3]
        streams.append(s)
    c = _with_inline_max(inline_max, lambda: K.Codec(0, max_batch_bytes=8 << 20, max_segs=256, max_frames=1 << 14))
    try:
        res = _check(c, streams, compact=compact)
        for i in range(len(streams)):
            st = res.state[i]
            if int(res.seg[i]["status"]) == K.SEG_ERROR:
                assert int(st["cont_utf8"]) == 0 and int(st["frame_utf8"]) == 0, (i, st)
                assert int(st["frame_rem"]) == 0, (i, st)
        assert int((res.seg["status"] == K.SEG_ERROR).sum()) == len(streams)
    finally:
        c.close()
