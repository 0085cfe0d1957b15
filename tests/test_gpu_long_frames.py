"""64-bit payload lengths on the device (websocket.go:291-299 parses the 8-byte length as u64).

A frame of 4 GiB or more is one wsc_frame record with a 40-bit length (payload_len |
payload_len_hi << 32) and several payload spans of at most 2 GiB each, cut at multiples of 4
bytes so every span keeps the frame's key phase.  The big payload is generated and checked on the
device in chunks (no multi-GiB host copies); the oracle cannot run a 4 GiB stream in a test's
time, so the records are checked against what the reference does for these headers (one
Message per FIN BIN frame, MsgID counting, 14-byte header) and the bytes against the pattern.
Lengths of 2^40 and more are always TOO_LARGE (max_frame_len < 2^40): that small case is
compared with the oracle record by record."""
import numpy as np
import pytest

import oracle_ref as O
from gpu_helpers import pack_streams, compare_segment
from netman_amd import codec as K
from netman_amd import synth

pytestmark = pytest.mark.gpu

CHUNK = 256 << 20


def _hdr64(op, n, mask, fin=True):
    return bytes([(0x80 if fin else 0) | op, 0x80 | 127]) + int(n).to_bytes(8, "big") + int(mask).to_bytes(4, "little")


def _pattern(torch, dev, start, n):
    """payload byte i (i from the payload start) = (i * 7 + (i >> 12)) & 0xFF, on the device"""
    i = torch.arange(start, start + n, dtype=torch.int64, device=dev)
    return ((i * 7 + (i >> 12)) & 0xFF).to(torch.uint8)


def _mask_tile(torch, dev, mask, n):
    k = torch.tensor(list(int(mask).to_bytes(4, "little")), dtype=torch.uint8, device=dev)
    return k.repeat((n + 3) // 4)[:n]


@pytest.mark.parametrize("compact,walk_mode", [(False, "0"), (True, "0"), (False, "3")])
def test_frame_over_4gib(codec_lib, monkeypatch, compact, walk_mode):
    torch = pytest.importorskip("torch")
    monkeypatch.setitem(K.CFG_DEFAULTS, "walk_mode", int(walk_mode))
    dev = torch.device("cuda:0")
    big = (4 << 30) + 12345            # > 2^32: 3 spans (2 GiB, 2 GiB, 12345 B)
    mask_big = 0xA1B2C3D4
    pre = synth.frame(2, b"x" * 100, mask=0x01020304)
    post = synth.frame(1, "tail ünïcode".encode(), mask=0x0BADF00D)
    other = [synth.frame(2, bytes(range(200)), mask=0x55AA55AA), synth.frame(1, b"hi", mask=7)]
    hb = _hdr64(2, big, mask_big)
    seg0_len = len(pre) + len(hb) + big + len(post)
    seg1 = b"".join(other)
    n_bytes = seg0_len + len(seg1)
    c = K.Codec(0, max_batch_bytes=n_bytes + 4096, max_segs=4, max_frames=64, max_frame_len=(1 << 40) - 1)
    wire = torch.empty(n_bytes + 64, dtype=torch.uint8, device=dev)
    head = np.frombuffer(pre + hb, dtype=np.uint8)
    wire[:len(head)] = torch.from_numpy(head.copy()).to(dev)
    p0 = len(head)                      # payload start of the big frame
    for o in range(0, big, CHUNK):      # masked pattern, chunk by chunk (CHUNK % 4 == 0: key phase kept)
        n = min(CHUNK, big - o)
        wire[p0 + o:p0 + o + n] = _pattern(torch, dev, o, n) ^ _mask_tile(torch, dev, mask_big, n)
    tail = np.frombuffer(post + seg1, dtype=np.uint8)
    wire[p0 + big:p0 + big + len(tail)] = torch.from_numpy(tail.copy()).to(dev)
    seg_off = torch.tensor([0, seg0_len, n_bytes], dtype=torch.int64, device=dev)
    st_out = torch.zeros(2 * K.STATE_BYTES, dtype=torch.uint8, device=dev)
    seg_out = torch.zeros(2 * 32, dtype=torch.uint8, device=dev)
    frames = torch.zeros(64 * 32, dtype=torch.uint8, device=dev)
    summ = torch.zeros(32, dtype=torch.uint8, device=dev)
    arena = torch.zeros(n_bytes + 64, dtype=torch.uint8, device=dev) if compact else None
    frame_dst = torch.zeros(64, dtype=torch.int64, device=dev) if compact else None
    b = c.make_batch(wire, seg_off, None, st_out, seg_out, frames, summ, compact=compact, arena=arena,
                     frame_dst=frame_dst, n_bytes=n_bytes)
    c.decode(b)
    c.sync()
    sm = summ.cpu().numpy().copy().view(K.SUMMARY_DTYPE)[0]
    assert K.Codec.summary_status(sm) == K.WSC_OK
    assert int(sm["n_frames"]) == 5 and int(sm["n_spans"]) == 1 + 3 + 1 + 2
    fr = frames.cpu().numpy().copy().view(K.FRAME_DTYPE)[:5]
    seg = seg_out.cpu().numpy().copy().view(K.SEG_RESULT_DTYPE)
    assert [int(x) for x in seg["status"]] == [K.SEG_OPEN, K.SEG_OPEN]
    assert int(seg[0]["consumed"]) == seg0_len and int(seg[1]["consumed"]) == len(seg1)
    assert [int(x) for x in fr["kind"]] == [K.FK_MESSAGE] * 5
    assert [int(x) for x in fr["msg_id"]] == [0, 1, 2, 0, 1]
    assert [K.frame_len(x) for x in fr] == [100, big, len("tail ünïcode".encode()), 200, 2]
    assert int(fr[1]["hdr_len"]) == 14 and int(fr[1]["hdr_off"]) == len(pre)
    assert int(fr[1]["payload_len_hi"]) == 1 and int(fr[1]["mask"]) == mask_big
    # payload bytes: the big one chunk by chunk on the device, the small ones on the host
    if compact:
        fd = frame_dst.cpu().numpy().copy().view(np.uint64)[:5]
        dst = [int(x) for x in fd]
        out, base = arena, dst[1]
    else:
        dst = None
        out, base = wire, p0
    for o in range(0, big, CHUNK):
        n = min(CHUNK, big - o)
        assert torch.equal(out[base + o:base + o + n], _pattern(torch, dev, o, n)), f"big payload at {o}"
    host = (arena if compact else wire).cpu().numpy()
    want = [(0, b"x" * 100), (2, "tail ünïcode".encode()), (3, bytes(range(200))), (4, b"hi")]
    for i, data in want:
        if compact:
            p = dst[i]
        else:
            p = int(fr[i]["hdr_off"]) + int(fr[i]["hdr_len"])
        assert bytes(host[p:p + len(data)]) == data, f"frame {i}"
    c.close()


def test_length_2_40_and_more_is_too_large(codec_lib):
    """headers claiming 2^40 .. 2^63 bytes: TOO_LARGE / 1002 with the record length saturated at
    2^40 - 1 (the oracle keeps the u64); 2^40 - 1 itself is a legal limit that only waits for bytes"""
    c = K.Codec(0, max_batch_bytes=1 << 20, max_segs=16, max_frames=1024, max_frame_len=(1 << 40) - 1)
    streams = [synth.frame(2, b"ok", mask=1) + _hdr64(2, 1 << 40, 5) + b"\x00" * 32,
               _hdr64(2, (1 << 63) + 7, 6),
               _hdr64(1, (1 << 40) - 1, 7) + b"\x00" * 10,
               _hdr64(0, 1 << 41, 8, fin=False)]
    wire, off = pack_streams(streams)
    res = c.decode_host(wire, off)
    for i, s in enumerate(streams):
        compare_segment(i, s, int(off[i]), res, O.run(s, max_frame_len=(1 << 40) - 1), wire_after=wire)
    f = res.frames
    assert K.frame_len(f[1]) == (1 << 40) - 1 and int(f[1]["err"]) == K.ERR_TOO_LARGE
    assert [int(x) for x in res.seg["status"]] == [K.SEG_ERROR, K.SEG_ERROR, K.SEG_OPEN, K.SEG_ERROR]
    c.close()


def test_max_frame_len_limit(codec_lib):
    with pytest.raises(K.WscError):
        K.Codec(0, max_batch_bytes=1 << 20, max_segs=4, max_frames=64, max_frame_len=1 << 40)


@pytest.mark.parametrize("compact,bad,big", [(False, False, (2 << 30) + 4100), (False, True, (2 << 30) + 4100),
                                             (True, True, (2 << 30) + 4100), (False, False, (4 << 30) + 4100),
                                             (True, True, (4 << 30) + 4100)])
def test_text_frame_over_1gib(codec_lib, compact, bad, big):
    """a TEXT frame of 2 GiB + 4100 B: three UTF-8 items cut at 1 GiB-aligned wire offsets with
    2-byte characters straddling every cut, most of it folded window by window inside the unmask,
    the item ends in k_u8_check, the three items composed by k_u8_verdict.  With one 0xFF byte at
    1.5 GiB the connection must stop at that frame with 1007 (websocket_frame.go:71-73,
    epoll.go:126-127) and the TEXT frame after it must be left masked (re-masked after the unmask);
    valid, the frame after it is a Message.  The payload is built and checked on the device.
    4 GiB + 4100 B: the payload (starting 24 B into the wire, not window-aligned) is
    cut into 2 GiB spans -- at absolute 2 GiB wire offsets, so no unmask window holds a cut and
    every window inside the text is folded (a cut inside a window left its map unwritten)."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    mask_big = 0x5EC0DE11
    pre = synth.frame(1, "pré".encode(), mask=0x01020304)
    post = synth.frame(1, "après".encode(), mask=0x0BADF00D)
    hb = _hdr64(1, big, mask_big)
    n_bytes = len(pre) + len(hb) + big + len(post)
    c = K.Codec(0, max_batch_bytes=n_bytes + 4096, max_segs=4, max_frames=64, max_frame_len=(1 << 40) - 1)
    wire = torch.empty(n_bytes + 64, dtype=torch.uint8, device=dev)
    head = np.frombuffer(pre + hb, dtype=np.uint8)
    wire[:len(head)] = torch.from_numpy(head.copy()).to(dev)
    p0 = len(head)
    bad_at = (3 << 29) + 1

    def text(o, n):   # "é" = C3 A9 repeated (payload offset o is even at every chunk start)
        i = torch.arange(o, o + n, dtype=torch.int64, device=dev)
        t = torch.where((i & 1) == 0, torch.tensor(0xC3, dtype=torch.uint8, device=dev),
                        torch.tensor(0xA9, dtype=torch.uint8, device=dev))
        if bad and o <= bad_at < o + n:
            t[bad_at - o] = 0xFF
        return t

    for o in range(0, big, CHUNK):
        n = min(CHUNK, big - o)
        wire[p0 + o:p0 + o + n] = text(o, n) ^ _mask_tile(torch, dev, mask_big, n)
    tail = np.frombuffer(post, dtype=np.uint8)
    wire[p0 + big:p0 + big + len(tail)] = torch.from_numpy(tail.copy()).to(dev)
    seg_off = torch.tensor([0, n_bytes], dtype=torch.int64, device=dev)
    st_out = torch.zeros(K.STATE_BYTES, dtype=torch.uint8, device=dev)
    seg_out = torch.zeros(32, dtype=torch.uint8, device=dev)
    frames = torch.zeros(64 * 32, dtype=torch.uint8, device=dev)
    summ = torch.zeros(32, dtype=torch.uint8, device=dev)
    arena = torch.zeros(n_bytes + 64, dtype=torch.uint8, device=dev) if compact else None
    frame_dst = torch.zeros(64, dtype=torch.int64, device=dev) if compact else None
    b = c.make_batch(wire, seg_off, None, st_out, seg_out, frames, summ, compact=compact, arena=arena,
                     frame_dst=frame_dst, n_bytes=n_bytes)
    c.decode(b)
    c.sync()
    sm = summ.cpu().numpy().copy().view(K.SUMMARY_DTYPE)[0]
    assert K.Codec.summary_status(sm) == K.WSC_OK and int(sm["n_frames"]) == 3
    assert int(sm["n_spans"]) == 2 + (1 if big < (4 << 30) else 3)
    seg = seg_out.cpu().numpy().copy().view(K.SEG_RESULT_DTYPE)[0]
    fr = frames.cpu().numpy().copy().view(K.FRAME_DTYPE)[:3]
    assert K.frame_len(fr[1]) == big and int(fr[1]["opcode"]) == 1
    fd = frame_dst.cpu().numpy().copy().view(np.uint64)[:3] if compact else None
    out = arena if compact else wire
    base = int(fd[1]) if compact else p0
    for o in range(0, big, CHUNK):   # the big payload is unmasked either way (nextFrame unmasks first)
        n = min(CHUNK, big - o)
        assert torch.equal(out[base + o:base + o + n], text(o, n)), f"big payload at {o}"
    if bad:
        assert int(seg["status"]) == K.SEG_ERROR and int(seg["close_code"]) == 1007
        assert int(seg["frame_count"]) == 2 and int(fr[1]["kind"]) == K.FK_ERROR
        assert int(seg["consumed"]) == p0 + big
        # the frame after the failing one is never read by the reference: its payload stays masked
        pl = len("après".encode())
        masked = wire[n_bytes - pl:n_bytes].cpu().numpy().tobytes()
        assert masked == post[-pl:], "payload after the failing frame must stay masked (in place)"
        if compact:   # in the arena the later payload is copied masked, as the key-0 span did
            assert arena[int(fd[2]):int(fd[2]) + pl].cpu().numpy().tobytes() == post[-pl:]
    else:
        assert int(seg["status"]) == K.SEG_OPEN and int(seg["frame_count"]) == 3
        assert [int(x) for x in fr["kind"]] == [K.FK_MESSAGE] * 3
        pl = len("après".encode())
        assert wire[n_bytes - pl:n_bytes].cpu().numpy().tobytes() == "après".encode()
    c.close()
