"""GPU parity: libwscodec (HIP, gfx950) against the CPU oracle on the same inputs.

Bit-exact for everything (integer/byte work): frame records, unmasked payload bytes, statuses,
carried state, delivered events.
"""
import numpy as np
import pytest

import oracle_ref as O
from fuzz_streams import random_stream, random_splits
from gpu_helpers import pack_streams, compare_segment, events_of_session
from netman_amd import codec as K
from netman_amd import synth

pytestmark = pytest.mark.gpu

HELLO = bytes.fromhex("818537fa213d7f9f4d5158")        # RFC 6455 §5.7 masked "Hello"
PONG_HELLO = bytes.fromhex("8a8537fa213d7f9f4d5158")   # RFC 6455 §5.7 masked Pong "Hello"


@pytest.fixture(scope="module")
def codec(codec_lib):
    c = K.Codec(0, max_batch_bytes=64 << 20, max_segs=1 << 14, max_frames=1 << 18)
    yield c
    c.close()


def _check_batch(codec, streams, compact=False, max_frame_len=O.MAX_FRAME_LEN):
    wire, off = pack_streams(streams)
    orig = wire.copy()
    res = codec.decode_host(wire, off, compact=compact)
    assert int(res.summary["overflow"]) == 0
    for i, s in enumerate(streams):
        ora = O.run(s, max_frame_len=max_frame_len)
        compare_segment(i, s, int(off[i]), res, ora, wire_after=wire, compact=compact)
    if compact:
        assert np.array_equal(wire, orig), "COMPACT mode must not modify the wire"
    return res


def test_rfc6455_known_answers(codec):
    streams = [HELLO, PONG_HELLO + HELLO, HELLO * 3]
    wire, off = pack_streams(streams)
    res = _check_batch(codec, streams)
    f = res.frames
    assert int(f[0]["kind"]) == K.FK_MESSAGE and int(f[0]["payload_len"]) == 5
    assert int(f[0]["mask"]) == 0x3D21FA37 and int(f[0]["mode"]) == 1
    # frame 2 (after the masked PONG, which takes msgID 0 -- Q5) is MsgID 1
    assert int(f[1]["kind"]) == K.FK_PONG and int(f[2]["msg_id"]) == 1


def test_rfc6455_unmasked_examples_stall(codec):
    # §5.7 single-frame unmasked text and fragmented unmasked text: netman never completes them (Q3)
    res = _check_batch(codec, [bytes.fromhex("810548656c6c6f"), bytes.fromhex("010348656c80026c6f")])
    assert [int(x) for x in res.seg["status"]] == [K.SEG_STALLED, K.SEG_STALLED]


@pytest.mark.parametrize("compact", [False, True])
def test_fuzz_single_batch(codec, compact):
    streams = [random_stream(1000 + i, n_units=int(5 + i % 40)) for i in range(400)]
    _check_batch(codec, streams, compact=compact)


@pytest.mark.parametrize("compact,mode", [(False, 3), (True, 3), (False, 256), (True, 256), (False, 64), (True, 64),
                                          (False, 65), (True, 65), (False, 16), (True, 16), (False, 32), (True, 32),
                                          (False, 66), (True, 66), (False, 257), (True, 257)])
def test_fuzz_walk_geometries(codec_lib, monkeypatch, compact, mode):
    """Every walk geometry forced on the same fuzz batches (5..44 units with text and errors, and
    1..6 units): the fused walk with 64- and 256-lane blocks (16 LDS records per lane, longer
    segments re-walked, the rest emitted cooperatively), 256-lane blocks whose first wave walks and
    all four emit (mode 65), 64-lane blocks whose first 16 / 32 lanes walk (modes 16, 32: several
    walking waves per CU), 256-lane blocks whose 64 walking columns are spread 16 per wave (mode
    66), one segment per lane with 4 LDS records per lane (mode 257: 3 blocks per CU), and the tiled
    walk for many segments (mode 3)."""
    monkeypatch.setitem(K.CFG_DEFAULTS, "walk_mode", mode)
    c = K.Codec(0, max_batch_bytes=64 << 20, max_segs=1 << 14, max_frames=1 << 18)
    try:
        streams = [random_stream(7000 + i, n_units=int(5 + i % 40), text_p=0.5) for i in range(400)]
        _check_batch(c, streams, compact=compact)
        assert c.walk_info()[0] == mode          # the pinned geometry really ran (round-4 ADVICE)
        streams = [random_stream(7500 + i, n_units=int(1 + i % 6)) for i in range(300)]
        _check_batch(c, streams, compact=compact)
        assert c.walk_info()[0] == mode
    finally:
        c.close()


def _run_streams(seed, n):
    """Segments built from runs of equal-size masked BIN frames (the quad pre-pass speculates 16
    headers per round trip at the last stride): run lengths 1..40, sizes across the 7/16-bit length
    forms, a TEXT or PING frame between runs, and some segments cut inside a header or payload."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        parts = []
        for _ in range(int(rng.integers(1, 5))):
            size = int(rng.choice([0, 1, 5, 60, 125, 126, 300, 1000, 4096]))
            parts += [synth.frame(2, bytes(rng.integers(0, 256, size, dtype=np.uint8)), rng=rng)
                      for _ in range(int(rng.integers(1, 41)))]
            r = rng.random()
            if r < 0.2:
                parts.append(synth.frame(1, "ok ü".encode() * int(rng.integers(1, 4)), rng=rng))
            elif r < 0.3:
                parts.append(synth.frame(9, b"ping", rng=rng))
        s = b"".join(parts)
        if rng.random() < 0.2:
            s = s[:int(rng.integers(1, len(s) + 1))]
        out.append(s)
    return out


@pytest.mark.parametrize("compact,pre", [(False, "1"), (True, "1"), (False, "0")])
def test_quad_prepass_runs(codec_lib, monkeypatch, compact, pre):
    """The fused walk's quad pre-pass (mode 65) on runs of equal frames, stride changes, non-BIN
    frames that end a run, and segments cut mid-frame: records, bytes and carried state equal the
    oracle's, and equal the serial walk's (walk_flags WSC_WALK_NO_QUAD_PRE)."""
    monkeypatch.setitem(K.CFG_DEFAULTS, "walk_mode", 65)
    monkeypatch.setitem(K.CFG_DEFAULTS, "walk_flags", 0 if pre == "1" else K.WALK_NO_QUAD_PRE)
    c = K.Codec(0, max_batch_bytes=64 << 20, max_segs=1 << 14, max_frames=1 << 18)
    try:
        for rep in range(2):   # the second decode starts from the first one's stride hint
            _check_batch(c, _run_streams(4242 + rep, 600), compact=compact)
    finally:
        c.close()


@pytest.mark.parametrize("cache", ["1", "0"])
def test_tiled_walk_header_cache(codec_lib, monkeypatch, cache):
    """The tiled walk (mode 3) with and without its per-segment header cache (walk_flags
    WSC_WALK_NO_HDR_CACHE), on the fuzz corpus and on runs of equal frames."""
    monkeypatch.setitem(K.CFG_DEFAULTS, "walk_mode", 3)
    monkeypatch.setitem(K.CFG_DEFAULTS, "walk_flags", 0 if cache == "1" else K.WALK_NO_HDR_CACHE)
    c = K.Codec(0, max_batch_bytes=64 << 20, max_segs=1 << 14, max_frames=1 << 18)
    try:
        _check_batch(c, [random_stream(8000 + i, n_units=int(1 + i % 9), text_p=0.3) for i in range(500)])
        _check_batch(c, _run_streams(77, 400), compact=True)
    finally:
        c.close()


@pytest.mark.parametrize("mode", ["65", "3"])
def test_nontemporal_header_loads(codec_lib, monkeypatch, mode):
    """The walk's non-temporal header loads (COMPACT batches by default) forced on in-place
    batches too (walk_flags WSC_WALK_HDR_NT): the same records and bytes as the oracle's."""
    monkeypatch.setitem(K.CFG_DEFAULTS, "walk_mode", int(mode))
    monkeypatch.setitem(K.CFG_DEFAULTS, "walk_flags", K.WALK_HDR_NT)
    c = K.Codec(0, max_batch_bytes=64 << 20, max_segs=1 << 14, max_frames=1 << 18)
    try:
        _check_batch(c, [random_stream(9100 + i, n_units=int(1 + i % 30), text_p=0.3) for i in range(400)])
        _check_batch(c, _run_streams(91, 300), compact=True)
    finally:
        c.close()


def _close_streams():
    from fuzz_streams import close_in_chain_stream, CLOSE_PAYLOADS
    streams = [close_in_chain_stream(11000 + i) for i in range(600)]
    for mode in (0, 1, 2):   # every CLOSE payload class in every messageMode
        for p in CLOSE_PAYLOADS:
            streams.append((synth.frame(mode, b"ab", fin=False) if mode else b"") + synth.frame(8, p, mask=0x0BADF00D))
    return streams


@pytest.mark.parametrize("compact,inline_max", [(False, 256), (True, 256), (False, 0)])
def test_close_inside_text_and_bin_chains(codec_lib, monkeypatch, compact, inline_max):
    """FIN=1 CLOSE frames inside TEXT / BIN chains (and outside any): the reason rule depends on
    messageMode (websocket.go:153-172 + websocket_frame.go:49,71-73).  inline_max 0 defers every
    other text check to the chip-wide UTF-8 kernel (the CLOSE itself is always checked in the walk)."""
    monkeypatch.setitem(K.CFG_DEFAULTS, "u8_inline_max", inline_max)
    c = K.Codec(0, max_batch_bytes=16 << 20, max_segs=1 << 12, max_frames=1 << 16)
    try:
        _check_batch(c, _close_streams(), compact=compact)
    finally:
        c.close()


def test_fuzz_text_heavy(codec):
    streams = [random_stream(5000 + i, n_units=30, text_p=0.9, err_p=0.02) for i in range(300)]
    _check_batch(codec, streams)


@pytest.mark.parametrize("compact", [False, True])
def test_edge_lengths(codec, compact):
    streams = []
    for n in [0, 1, 2, 3, 4, 5, 15, 16, 17, 125, 126, 127, 1023, 1024, 1025, 65535, 65536, 65537, 1 << 20]:
        streams.append(synth.frame(2, bytes(np.random.default_rng(n).bytes(n)), mask=0xDEADBEEF))
        streams.append(synth.frame(2, b"\x00" * n, mask=0))
        streams.append(synth.frame(2, b"\xff" * n, mask=0xFFFFFFFF, ext=8))
    streams.append(b"")
    streams.append(b"\x82")                         # incomplete header
    streams.append(synth.frame(2, b"abc")[:-1])     # incomplete payload
    _check_batch(codec, streams, compact=compact)


@pytest.mark.parametrize("compact", [False, True])
def test_tiny_frames_many_per_piece(codec, compact):
    """Frames of 0-40 B: several spans per 16-byte piece (the tail loop), more than 64 spans per
    4 KiB window (the serial fallback), fragments of 0-8 B with PINGs between them, and runs that
    end on the last bytes of the wire (the partial last window)."""
    rng = np.random.default_rng(77)
    streams = []
    s = b"".join(synth.frame(2, rng.bytes(int(rng.integers(0, 9))), mask=int(rng.integers(0, 2**32)))
                 for _ in range(2000))
    streams.append(s)
    for i in range(300):
        fr = []
        for _ in range(int(rng.integers(1, 21))):
            fr.append(synth.frame(2, rng.bytes(int(rng.integers(0, 41))), mask=int(rng.integers(0, 2**32))))
        streams.append(b"".join(fr))
    for i in range(100):   # fragmented: 0x02 FIN=0, 0x00 ..., 0x00 FIN=1 with tiny parts and PINGs
        parts = [rng.bytes(int(rng.integers(0, 9))) for _ in range(int(rng.integers(2, 12)))]
        out = bytearray()
        for j, p in enumerate(parts):
            out += synth.frame(2 if j == 0 else 0, p, fin=j == len(parts) - 1, mask=int(rng.integers(0, 2**32)))
            if rng.random() < 0.3:
                out += synth.frame(9, rng.bytes(int(rng.integers(0, 6))), mask=int(rng.integers(0, 2**32)))
        streams.append(bytes(out))
    streams.append(b"".join(synth.frame(2, bytes([k]) * k, mask=0x01020304) for k in (15, 16, 17, 1, 31, 32, 33)))
    _check_batch(codec, streams, compact=compact)


def test_max_frame_len(codec_lib):
    c = K.Codec(0, max_batch_bytes=8 << 20, max_segs=64, max_frames=4096, max_frame_len=1000)
    streams = [synth.frame(2, b"a" * 1000), synth.frame(2, b"a" * 1001), synth.frame(10, b"b" * 5000),
               synth.frame(1, b"ok") + synth.frame(2, b"c" * 70000)]
    wire, off = pack_streams(streams)
    res = c.decode_host(wire, off)
    for i, s in enumerate(streams):
        compare_segment(i, s, int(off[i]), res, O.run(s, max_frame_len=1000), wire_after=wire)
    assert int(res.seg[1]["err"]) == K.ERR_TOO_LARGE
    c.close()


@pytest.mark.parametrize("compact", [False, True])
def test_session_carry_over(codec_lib, compact):
    """streams fed in random chunks across several batched decodes == oracle on the whole stream"""
    rng = np.random.default_rng(7)
    sess = K.Session(0, compact=compact, max_batch_bytes=16 << 20, max_segs=1024, max_frames=1 << 16)
    streams = [random_stream(9000 + i, n_units=25) for i in range(120)]
    conns = [sess.open() for _ in streams]
    splits = [random_splits(rng, len(s), int(rng.integers(0, 6))) for s in streams]
    got = {c: [] for c in conns}
    rounds = max(len(sp) for sp in splits)
    prev = [0] * len(streams)
    for r in range(rounds):
        for i, (c, s, sp) in enumerate(zip(conns, streams, splits)):
            if r < len(sp):
                sess.feed(c, s[prev[i]:sp[r]])
                prev[i] = sp[r]
        sess.decode()
        for c in conns:
            got[c].extend(events_of_session(sess, c))
    for i, (c, s) in enumerate(zip(conns, streams)):
        ref = [e.key() for e in O.run(s).events]
        assert got[c] == ref, f"stream {i}: {got[c][:5]} vs {ref[:5]}"
    sess.close()


@pytest.mark.gpu
def test_header_split_across_feeds_is_header_complete(codec_lib):
    """Q1/Q2 at the device boundary (documented divergence): the reference's parseHeadBytes /
    parsePayloadLength read the extended length and the mask with one Read each
    (websocket.go:214-302) and desync when a read returns fewer bytes.  The codec only decodes a
    frame once its whole header is in, so a stream fed with the cut at EVERY header byte gives the
    events of the whole stream -- and those differ from the reference's own chunked behaviour
    (the oracle run with the same cut), which is the divergence DESIGN.md lists."""
    frames = [synth.frame(2, b"x" * 200, mask=0x01020304),          # 16-bit length, 8-byte header
              synth.frame(1, "é".encode() * 40000, mask=0x0a0b0c0d),  # 64-bit length, 14-byte header
              synth.frame(2, b"abc", mask=0x11223344)]                # 7-bit length, 6-byte header
    tail = synth.frame(2, b"y", mask=5)
    sess = K.Session(0, max_batch_bytes=1 << 20, max_segs=64, max_frames=1024)
    diverged = 0
    for f in frames:
        hl = {126: 8, 127: 14}.get(f[1] & 0x7F, 6)
        s = f + tail
        whole = [e.key() for e in O.run(s).events]
        for cut in range(1, hl):
            c = sess.open()
            sess.feed(c, s[:cut])
            sess.decode()
            got = events_of_session(sess, c)
            assert got == [], f"cut {cut}: events before the header is complete: {got}"
            sess.feed(c, s[cut:])
            sess.decode()
            got += events_of_session(sess, c)
            assert got == whole, f"header {hl} B cut at {cut}: {got[:3]} vs {whole[:3]}"
            ref_chunked = [e.key() for e in O.run(s, chunk_ends=[cut, len(s)]).events]
            diverged += ref_chunked != [e.key() for e in O.run(s).events]
            sess.remove(c)
    assert diverged > 0   # the reference does desync on some of these cuts (Q1/Q2)
    sess.close()


def test_decode_packet_mirror(codec_lib):
    sess = K.Session(0, max_batch_bytes=1 << 20, max_segs=16, max_frames=1024)
    c = sess.open()
    sess.feed(c, HELLO + synth.frame(9, b"ping!") + synth.frame(0x2, b"\x01\x02", fin=True)
              + synth.frame(1, b"\xff"))
    sess.decode()
    m, err = sess.DecodePacket(c)
    assert err is None and m.IsText() and m.Bytes() == b"Hello" and m.ID() == 0
    m, err = sess.DecodePacket(c)          # PING answered -> (nil, nil)
    assert m is None and err is None
    m, err = sess.DecodePacket(c)
    assert m.IsBinary() and m.ID() == 2    # the PING consumed msgID 1 (Q5)
    m, err = sess.DecodePacket(c)
    assert m is None and err is K.WebsocketMustUtf8 and K.close_code_for(err) == 1007
    m, err = sess.DecodePacket(c)
    assert err is K.EAGAIN
    sess.close()


def test_device_resident_uniform_64k(codec_lib):
    torch = pytest.importorskip("torch")
    cfg = synth.uniform_batch(1024, 65536, 4, seed=synth.SEED_BASE + 99)
    c = K.Codec(0, max_batch_bytes=128 << 20, max_segs=4096, max_frames=1 << 16)
    dev = torch.device("cuda:0")
    wire = torch.from_numpy(cfg["wire"]).to(dev)
    seg_off = torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev)
    n = len(cfg["seg_off"]) - 1
    st_out = torch.zeros(n * K.STATE_BYTES, dtype=torch.uint8, device=dev)
    seg_out = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
    frames = torch.zeros((1 << 16) * 32, dtype=torch.uint8, device=dev)
    summ = torch.zeros(32, dtype=torch.uint8, device=dev)
    b = c.make_batch(wire, seg_off, None, st_out, seg_out, frames, summ)
    c.decode(b)
    c.sync()
    ref = synth.unmask_reference(cfg["wire"], cfg["payload_off"], cfg["plen"], cfg["mask"])
    assert np.array_equal(wire.cpu().numpy().copy(), ref)
    # XOR is an involution: a second decode restores the masked bytes exactly
    c.decode(b)
    c.sync()
    assert np.array_equal(wire.cpu().numpy().copy(), cfg["wire"])
    fr = frames.cpu().numpy().copy().view(K.FRAME_DTYPE)[:1024]
    assert (fr["kind"] == K.FK_MESSAGE).all() and (fr["msg_id"] == np.tile(np.arange(4), 256)).all()
    c.close()


# ---- golden fixtures through the device path --------------------------------------------------
def test_golden_known_answers_gpu(codec_lib):
    from golden_io import kat_cases, event_matches
    cases = kat_cases()
    sess = K.Session(0, max_batch_bytes=4 << 20, max_segs=64, max_frames=4096)
    conns = []
    for _, stream, _ in cases:
        c = sess.open()
        sess.feed(c, stream)
        conns.append(c)
    sess.decode()
    for (name, _, expect), c in zip(cases, conns):
        evs = sess.events(c)
        assert len(evs) == len(expect), (name, evs)
        for e, ev in zip(expect, evs):
            assert event_matches(e, ev), (name, e, ev)
    sess.close()


@pytest.mark.parametrize("compact", [False, True])
def test_golden_aiohttp_streams_gpu(codec, compact):
    from golden_io import aiohttp_cases
    streams = [s for _, s, _ in aiohttp_cases()]
    _check_batch(codec, streams, compact=compact)


# ---- BASELINE.json configs at full size (size-independent properties + vectorised reference) --
def _device_batch(c, cfg, torch, compact=False):
    dev = torch.device("cuda:0")
    n = len(cfg["seg_off"]) - 1
    t = dict(wire=torch.from_numpy(cfg["wire"]).to(dev),
             seg_off=torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev),
             st_out=torch.zeros(n * K.STATE_BYTES, dtype=torch.uint8, device=dev),
             seg_out=torch.zeros(n * 32, dtype=torch.uint8, device=dev),
             frames=torch.zeros((cfg["n_frames"] + 16) * 32, dtype=torch.uint8, device=dev),
             summ=torch.zeros(32, dtype=torch.uint8, device=dev))
    if compact:
        t["arena"] = torch.zeros(len(cfg["wire"]) + 64, dtype=torch.uint8, device=dev)
        t["frame_dst"] = torch.zeros(cfg["n_frames"] + 16, dtype=torch.int64, device=dev)
    b = c.make_batch(t["wire"], t["seg_off"], None, t["st_out"], t["seg_out"], t["frames"], t["summ"],
                     compact=compact, arena=t.get("arena"), frame_dst=t.get("frame_dst"))
    return b, t


def _device_result(t, cfg, compact=False):
    """the device batch's outputs as a DecodeResult (host copies)"""
    summ = t["summ"].cpu().numpy().copy().view(K.SUMMARY_DTYPE)[0]
    assert K.Codec.summary_status(summ) == K.WSC_OK
    nf = int(summ["n_frames"])
    return K.DecodeResult(seg=t["seg_out"].cpu().numpy().copy().view(K.SEG_RESULT_DTYPE),
                          state=t["st_out"].cpu().numpy().copy().view(K.CONN_STATE_DTYPE),
                          frames=t["frames"].cpu().numpy().copy().view(K.FRAME_DTYPE)[:nf], summary=summ,
                          frame_dst=t["frame_dst"].cpu().numpy().copy().view(np.uint64)[:nf] if compact else None,
                          arena=t["arena"].cpu().numpy().copy() if compact else None)


def _oracle_sample(cfg, res, after, compact=False, n=2000, must=(), seed=0):
    """record-by-record and byte-by-byte comparison with the oracle (O.run on the segment's own
    masked bytes) for n sampled segments + the segments in `must` + the first and last ones"""
    n_segs = len(cfg["seg_off"]) - 1
    rng = np.random.default_rng(seed)
    pick = set(rng.choice(n_segs, size=min(n, n_segs), replace=False).tolist()) | set(int(x) for x in must)
    pick |= {0, n_segs - 1}
    for i in sorted(pick):
        a, b = int(cfg["seg_off"][i]), int(cfg["seg_off"][i + 1])
        stream = bytes(cfg["wire"][a:b])
        compare_segment(i, stream, a, res, O.run(stream), wire_after=after, compact=compact)
    return len(pick)


@pytest.mark.parametrize("per_seg", [16, 1])   # 64 k connections x 16 frames, and 1 frame per segment
def test_config1_1m_x_1k_frames(codec_lib, per_seg):
    torch = pytest.importorskip("torch")
    cfg = synth.uniform_batch(1 << 20, 1024, per_seg, seed=synth.SEED_BASE + 1)
    c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=(1 << 20) // per_seg, max_frames=(1 << 20) + 16)
    b, t = _device_batch(c, cfg, torch)
    c.decode(b)
    c.sync()
    after = t["wire"].cpu().numpy().copy()
    assert np.array_equal(after, synth.unmask_uniform(cfg))
    res = _device_result(t, cfg)
    fr = res.frames
    assert len(fr) == 1 << 20 and (fr["kind"] == K.FK_MESSAGE).all() and (fr["hdr_len"] == 8).all()
    assert _oracle_sample(cfg, res, after, n=2000 // per_seg * per_seg) >= 2000
    c.close()


@pytest.mark.parametrize("per_seg", [16, 1])
def test_config2_mixed_power_law(codec_lib, per_seg):
    torch = pytest.importorskip("torch")
    cfg = synth.mixed_batch(frames_per_seg=per_seg)
    c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=len(cfg["seg_off"]) - 1, max_frames=cfg["n_frames"] + 16)
    b, t = _device_batch(c, cfg, torch)
    c.decode(b)
    c.sync()
    after = t["wire"].cpu().numpy().copy()
    ref = synth.unmask_reference(cfg["wire"], cfg["payload_off"], cfg["plen"], cfg["mask"])
    assert np.array_equal(after, ref)
    # every segment that holds a 1 MiB frame (6 / 8 / 14-byte headers side by side), + 2000 more
    big = np.nonzero(cfg["plen"] == 1048576)[0] // per_seg
    res = _device_result(t, cfg)
    assert _oracle_sample(cfg, res, after, must=big, seed=2) >= 2000
    c.close()


def test_config3_shard_1m_x_4k_frames(codec_lib):
    """one GPU's shard of configs[3] (8M x 4 KiB over 8 GPUs): 1M frames, 4 GiB payload"""
    torch = pytest.importorskip("torch")
    from netman_amd import shard
    cfg = synth.uniform_batch(1 << 20, 4096, 16, seed=shard.shard_seed(synth.SEED_BASE + 3, 0))
    c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=1 << 16, max_frames=(1 << 20) + 16)
    b, t = _device_batch(c, cfg, torch)
    c.decode(b)
    c.sync()
    assert np.array_equal(t["wire"].cpu().numpy().copy(), synth.unmask_uniform(cfg))
    c.decode(b)                      # involution: decoding again restores the masked wire
    c.sync()
    assert np.array_equal(t["wire"].cpu().numpy().copy(), cfg["wire"])
    c.close()


@pytest.mark.parametrize("ping_p", [0.0, 0.1])
def test_config4_fragmented_reassembly(codec_lib, ping_p):
    """configs[4]: 64k connections x one fragmented message, reassembled contiguously (COMPACT)"""
    torch = pytest.importorskip("torch")
    cfg = synth.fragmented_batch(n_conns=65536, seed=synth.SEED_BASE + 4, ping_p=ping_p)
    c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=1 << 16, max_frames=cfg["n_frames"] + 16)
    b, t = _device_batch(c, cfg, torch, compact=True)
    c.decode(b)
    c.sync()
    assert np.array_equal(t["wire"].cpu().numpy().copy(), cfg["wire"])      # COMPACT leaves the wire alone
    fr = t["frames"].cpu().numpy().copy().view(K.FRAME_DTYPE)[: cfg["n_frames"]]
    dst = t["frame_dst"].cpu().numpy().copy()[: cfg["n_frames"]].view(np.uint64)
    arena = t["arena"].cpu().numpy().copy()
    segr = t["seg_out"].cpu().numpy().copy().view(K.SEG_RESULT_DTYPE)
    ref = synth.unmask_reference(cfg["wire"], cfg["payload_off"], cfg["plen"], cfg["mask"])
    data_frames = fr["kind"] != K.FK_PING
    assert (segr["status"] == K.SEG_OPEN).all() and (fr["kind"][data_frames] != K.FK_ERROR).all()
    msg_end = np.nonzero(fr["kind"] == K.FK_MESSAGE)[0]
    assert len(msg_end) == 65536
    # arena layout: per connection [message bytes, contiguous][control payloads], in order
    pieces = []
    fb = segr["frame_begin"].astype(np.int64)
    fc = segr["frame_count"].astype(np.int64)
    for cn in range(65536):
        ks = range(fb[cn], fb[cn] + fc[cn])
        for want_ping in (False, True):
            for i in ks:
                if (fr["kind"][i] == K.FK_PING) == want_ping:
                    p, L = int(cfg["payload_off"][i]), int(cfg["plen"][i])
                    pieces.append(ref[p:p + L])
    expect = np.concatenate(pieces)
    sm = t["summ"].cpu().numpy().copy().view(K.SUMMARY_DTYPE)[0]
    assert int(sm["data_bytes"]) + int(sm["ctrl_bytes"]) == len(expect)
    assert np.array_equal(arena[: len(expect)], expect)
    # frame_dst points at each payload
    assert int((dst != 0).sum()) >= cfg["n_frames"] - 65536, ((dst != 0).sum(), dst[:20], fr[:3])
    for i in range(0, cfg["n_frames"], 997):
        p, L = int(cfg["payload_off"][i]), int(cfg["plen"][i])
        assert np.array_equal(arena[int(dst[i]):int(dst[i]) + L], ref[p:p + L]), \
            (i, int(dst[i]), p, L, fr[i - 2:i + 3], dst[i - 2:i + 3], cfg["plen"][i - 2:i + 3])
    # record by record against the oracle (MsgIDs across PINGs, Q5) on 2,000 sampled connections
    res = _device_result(t, cfg, compact=True)
    assert _oracle_sample(cfg, res, t["wire"].cpu().numpy().copy(), compact=True, seed=4) >= 2000
    c.close()


def test_compact_decode_is_deterministic(codec_lib):
    """repeated decodes of one batch give identical records (look-back hand-off under load)"""
    torch = pytest.importorskip("torch")
    cfg = synth.fragmented_batch(n_conns=65536, seed=synth.SEED_BASE + 44, ping_p=0.1)
    c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=1 << 16, max_frames=cfg["n_frames"] + 16)
    b, t = _device_batch(c, cfg, torch, compact=True)
    first = None
    for _ in range(20):
        c.decode(b)
        c.sync()
        snap = (t["frames"].cpu().numpy().copy(), t["frame_dst"].cpu().numpy().copy(),
                t["seg_out"].cpu().numpy().copy(), t["summ"].cpu().numpy().copy())
        if first is None:
            first = snap
        else:
            for x, y in zip(first, snap):
                assert np.array_equal(x, y)
    sm = first[3].view(K.SUMMARY_DTYPE)[0]
    assert int(sm["overflow"]) == 0 and int(sm["n_frames"]) == cfg["n_frames"]
    c.close()


def test_session_undrained_events_survive_next_decode(codec_lib):
    """messages are handed out as zero-copy views into the pinned staging; events not drained
    before the next wsc_session_decode must still carry their own bytes afterwards"""
    sess = K.Session(0, max_batch_bytes=1 << 20, max_segs=16, max_frames=1024)
    a, b = sess.open(), sess.open()
    pa = [bytes([i]) * (100 + i) for i in range(5)]
    sess.feed(a, b"".join(synth.frame(2, p, mask=0x01020304 + i) for i, p in enumerate(pa)))
    sess.feed(b, synth.frame(9, b"ping-b"))
    sess.decode()
    first = sess.next_event(a)                        # drained: valid until the next decode
    assert first.data == pa[0]
    sess.feed(a, synth.frame(2, b"\xee" * 5000, mask=0xAABBCCDD))
    sess.feed(b, synth.frame(1, "καλημέρα".encode()))
    sess.decode()                                     # reuses the staging
    rest = sess.events(a)
    assert [e.data for e in rest] == pa[1:] + [b"\xee" * 5000]
    eb = sess.events(b)
    assert eb[0].type == K.EV_PONG and eb[0].data == b"ping-b"
    assert eb[1].type == K.EV_MESSAGE and eb[1].data == "καλημέρα".encode()
    sess.close()


# ---- split pipeline (wsc_decode_split): walk on a CU-masked stream, unmask on others ----------
@pytest.mark.parametrize("compact,layout,inline_max,staged", [
    (False, "bench", 256, False), (True, "bench", 256, False), (False, "rest2", 256, False),
    (True, "rest2", 256, False), (False, "bench", 0, False), (True, "rest2", 0, False),
    (False, "bench", 256, True), (True, "bench", 0, True), (False, "rest2", 0, True), (True, "bench", 256, True)])
def test_decode_split_pipeline_matches_oracle(codec_lib, compact, layout, inline_max, staged):
    """two contexts in flight, walk stream on 16 CUs; the unmasks on one stream over every CU (the
    bench's pipeline) or on one stream per context over the other CUs; every round re-arms the
    wires and decodes both batches back to back, so one batch's walk runs beside the other's
    unmask; each is compared with the oracle.  inline_max 0 sends every text check to the
    chip-wide UTF-8 kernel (which runs on the unmask stream).  staged: wsc_decode_walk, the host
    waits for the walk, wsc_decode_finish (the check is skipped when nothing was deferred, the
    unmask signals the host instead of recording an event)"""
    import os
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    sets = [[random_stream(7000 + 400 * j + i, n_units=10) for i in range(300)] for j in range(2)]
    ctxs, bats, ts, packed = [], [], [], []
    for streams in sets:
        wire, off = pack_streams(streams)
        c = K.Codec(0, max_batch_bytes=len(wire) + 4096, max_segs=len(streams), max_frames=1 << 15,
                    u8_inline_max=inline_max)
        n = len(streams)
        t = dict(wire=torch.from_numpy(wire.copy()).to(dev), seg_off=torch.from_numpy(off.view(np.int64)).to(dev),
                 st_out=torch.zeros(n * K.STATE_BYTES, dtype=torch.uint8, device=dev),
                 seg_out=torch.zeros(n * 32, dtype=torch.uint8, device=dev),
                 frames=torch.zeros((1 << 15) * 32, dtype=torch.uint8, device=dev),
                 summ=torch.zeros(32, dtype=torch.uint8, device=dev))
        if compact:
            t["arena"] = torch.zeros(len(wire) + 64, dtype=torch.uint8, device=dev)
            t["frame_dst"] = torch.zeros(1 << 15, dtype=torch.int64, device=dev)
        ctxs.append(c)
        ts.append(t)
        packed.append((wire, off, streams))
        bats.append(c.make_batch(t["wire"], t["seg_off"], None, t["st_out"], t["seg_out"], t["frames"], t["summ"],
                                 compact=compact, arena=t.get("arena"), frame_dst=t.get("frame_dst")))
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    ws = ctxs[0].stream_create(K.cu_mask(range(16), n_cu))
    if layout == "bench":
        us = [ctxs[0].stream_create(None)]
    else:
        us = [ctxs[0].stream_create(K.cu_mask(range(16, n_cu), n_cu)) for _ in range(2)]
    with pytest.raises(K.WscError):
        ctxs[0].decode_split(bats[0], ws, ws)
    try:
        for _ in range(3):
            for t, (wire, _, _) in zip(ts, packed):
                t["wire"].copy_(torch.from_numpy(wire))
            torch.cuda.synchronize()
            for j in range(2):
                if staged:
                    ctxs[j].decode_walk(bats[j], ws)
                    ctxs[j].walk_wait()
                    ctxs[j].decode_finish(bats[j], us[j % len(us)])
                else:
                    ctxs[j].decode_split(bats[j], ws, us[j % len(us)])
            torch.cuda.synchronize()
            for j, (wire, off, streams) in enumerate(packed):
                t = ts[j]
                summ = t["summ"].cpu().numpy().copy().view(K.SUMMARY_DTYPE)[0]
                nf = int(summ["n_frames"])
                res = K.DecodeResult(
                    seg=t["seg_out"].cpu().numpy().copy().view(K.SEG_RESULT_DTYPE),
                    state=t["st_out"].cpu().numpy().copy().view(K.CONN_STATE_DTYPE),
                    frames=t["frames"].cpu().numpy().copy().view(K.FRAME_DTYPE)[:nf], summary=summ,
                    frame_dst=t["frame_dst"].cpu().numpy().copy().view(np.uint64)[:nf] if compact else None,
                    arena=t["arena"].cpu().numpy().copy() if compact else None)
                after = t["wire"].cpu().numpy().copy()
                if compact:
                    assert np.array_equal(after, wire)
                for i, s in enumerate(streams):
                    compare_segment(i, s, int(off[i]), res, O.run(s), wire_after=after, compact=compact)
    finally:
        torch.cuda.synchronize()
        for s in [ws] + us:
            ctxs[0].stream_destroy(s)
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("inline_max", [256, 0])
def test_staged_pipeline_back_to_back(codec_lib, monkeypatch, inline_max):
    """COMPACT (the wire is only read), two contexts, eight staged decodes per context with no
    host synchronisation between them: each context's next walk must wait (on the host, for the
    unmask's pinned done word) until its previous unmask has read the spans and window index it
    overwrites.  A race would corrupt the arena; the last decode of each is checked with the oracle."""
    monkeypatch.setitem(K.CFG_DEFAULTS, "u8_inline_max", inline_max)
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    ctxs, bats, ts, packed = [], [], [], []
    for j in range(2):
        streams = [random_stream(9100 + 500 * j + i, n_units=12) for i in range(400)]
        wire, off = pack_streams(streams)
        c = K.Codec(0, max_batch_bytes=len(wire) + 4096, max_segs=len(streams), max_frames=1 << 15)
        n = len(streams)
        t = dict(wire=torch.from_numpy(wire.copy()).to(dev), seg_off=torch.from_numpy(off.view(np.int64)).to(dev),
                 st_out=torch.zeros(n * K.STATE_BYTES, dtype=torch.uint8, device=dev),
                 seg_out=torch.zeros(n * 32, dtype=torch.uint8, device=dev),
                 frames=torch.zeros((1 << 15) * 32, dtype=torch.uint8, device=dev),
                 summ=torch.zeros(32, dtype=torch.uint8, device=dev),
                 arena=torch.zeros(len(wire) + 64, dtype=torch.uint8, device=dev),
                 frame_dst=torch.zeros(1 << 15, dtype=torch.int64, device=dev))
        ctxs.append(c)
        ts.append(t)
        packed.append((wire, off, streams))
        bats.append(c.make_batch(t["wire"], t["seg_off"], None, t["st_out"], t["seg_out"], t["frames"], t["summ"],
                                 compact=True, arena=t["arena"], frame_dst=t["frame_dst"]))
    torch.cuda.synchronize()
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    ws = ctxs[0].stream_create(K.cu_mask(range(16), n_cu))
    us = ctxs[0].stream_create(None)
    try:
        for i in range(16):
            j = i % 2
            ctxs[j].decode_walk(bats[j], ws)
            ctxs[j].walk_wait()
            ctxs[j].decode_finish(bats[j], us)
        torch.cuda.synchronize()
        for j, (wire, off, streams) in enumerate(packed):
            t = ts[j]
            summ = t["summ"].cpu().numpy().copy().view(K.SUMMARY_DTYPE)[0]
            nf = int(summ["n_frames"])
            res = K.DecodeResult(
                seg=t["seg_out"].cpu().numpy().copy().view(K.SEG_RESULT_DTYPE),
                state=t["st_out"].cpu().numpy().copy().view(K.CONN_STATE_DTYPE),
                frames=t["frames"].cpu().numpy().copy().view(K.FRAME_DTYPE)[:nf], summary=summ,
                frame_dst=t["frame_dst"].cpu().numpy().copy().view(np.uint64)[:nf],
                arena=t["arena"].cpu().numpy().copy())
            after = t["wire"].cpu().numpy().copy()
            assert np.array_equal(after, wire)
            for i, s in enumerate(streams):
                compare_segment(i, s, int(off[i]), res, O.run(s), wire_after=after, compact=True)
            assert ctxs[j].error_flags() == 0
    finally:
        torch.cuda.synchronize()
        for s in (ws, us):
            ctxs[0].stream_destroy(s)
        for c in ctxs:
            c.close()


# ---- multi-GPU sharding: shards decoded independently == the unsharded decode ----
@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_decode_equals_unsharded(codec, world):
    """one global batch of fuzz connections split with shard.split_batch (connection c -> rank
    c mod world), every shard decoded on its own (device 0 stands in for device r), the shards'
    records and bytes merged back by connection: identical to decoding the whole batch at once,
    and to the oracle -- no cross-shard state exists (no collective needed)"""
    from netman_amd import shard
    streams = [random_stream(13000 + i, n_units=int(3 + i % 25)) for i in range(240)]
    wire, off = pack_streams(streams)
    whole_wire = wire.copy()
    whole = codec.decode_host(whole_wire, off)
    assert K.Codec.summary_status(whole.summary) == K.WSC_OK
    merged_wire = np.empty_like(wire)
    for r in range(world):
        w, so, mine = shard.split_batch(wire, off, world, r)
        w = w.copy()
        res = codec.decode_host(w, so)
        for j, g in enumerate(mine):
            a, b = int(off[g]), int(off[g + 1])
            merged_wire[a:b] = w[int(so[j]):int(so[j + 1])]
            # records: same fields as the unsharded decode's, offsets rebased to the global batch
            sr, wr = res.seg[j], whole.seg[g]
            for f in ("consumed", "frame_count", "status", "close_code", "err"):
                assert int(sr[f]) == int(wr[f]), (g, f)
            fs = res.frames[int(sr["frame_begin"]):int(sr["frame_begin"]) + int(sr["frame_count"])].copy()
            fw = whole.frames[int(wr["frame_begin"]):int(wr["frame_begin"]) + int(wr["frame_count"])].copy()
            fs["hdr_off"] += np.uint64(a) - so[j]
            fs["seg"] = g
            assert np.array_equal(fs, fw), g
            assert np.array_equal(res.state[j], whole.state[g])
    assert np.array_equal(merged_wire, whole_wire)
    for i, s in enumerate(streams):
        compare_segment(i, s, int(off[i]), whole, O.run(s), wire_after=whole_wire)


@pytest.mark.parametrize("inline_max", [256, 0])
def test_mode65_many_blocks_large_payloads(codec_lib, monkeypatch, inline_max):
    """The configs[2] geometry (mode 65: one walking wave and the quad pre-pass per block, >= 128
    blocks over the whole chip) on 9,000 connections: fuzz streams (text, errors, control frames),
    runs of equal BIN frames, and one in 25 carrying payloads of 17 KiB .. 1 MiB -- whole, cut at
    the segment's end (a streamed piece), as a fragment (FIN=0) or as TEXT (deferred UTF-8).  Every
    segment equals the oracle, record for record and byte for byte.  (It was written for the
    round-6 eager-unmask experiment, DESIGN.md "Round 6", whose helper waves took those payloads.)"""
    monkeypatch.setitem(K.CFG_DEFAULTS, "u8_inline_max", inline_max)
    rng = np.random.default_rng(2606)
    streams = []
    for i in range(9000):
        if i % 25 == 7:
            parts = [synth.frame(2, b"h" * int(rng.integers(0, 300)), rng=rng)]
            for _ in range(int(rng.integers(1, 4))):
                n = int(rng.choice([17 << 10, 64 << 10, 65535, 100003, 1 << 20]))
                body = bytes(rng.integers(0, 256, n, dtype=np.uint8))
                kind = rng.random()
                if kind < 0.6:
                    parts.append(synth.frame(2, body, rng=rng))
                elif kind < 0.75:
                    parts.append(synth.frame(2, body, fin=False, rng=rng) + synth.frame(0, b"end", rng=rng))
                else:
                    parts.append(synth.frame(1, ("é" * (n // 2)).encode(), rng=rng))
            s = b"".join(parts)
            if rng.random() < 0.3:   # the segment ends inside its last payload: a streamed piece
                s = s[:len(s) - int(rng.integers(1, 9000))]
            streams.append(s)
        elif i % 3 == 0:
            streams.append(b"".join(synth.frame(2, bytes(rng.integers(0, 256, 125, dtype=np.uint8)), rng=rng)
                                    for _ in range(int(rng.integers(1, 17)))))
        else:
            streams.append(random_stream(26000 + i, n_units=int(1 + i % 12), text_p=0.3))
    c = K.Codec(0, max_batch_bytes=512 << 20, max_segs=1 << 14, max_frames=1 << 18)
    try:
        res = _check_batch(c, streams)
        mode, blocks = c.walk_info()
        assert mode == 65 and blocks >= 128, (mode, blocks)
        assert c.error_flags() == 0
    finally:
        c.close()
