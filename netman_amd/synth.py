"""Synthetic masked client->server WebSocket traffic (RFC 6455 §5.2), generated with numpy.

Used by bench.py and the tests to build the BASELINE.json configs as device-resident batches.
Payload bytes on the wire are uniform random (so the unmasked payload is uniform random too);
masks are uniform random u32; MASK=1, RSV=0 and minimal length encoding unless asked otherwise.
Seeds: 0x57530001 + config index (+ rank for multi-GPU shards), see DESIGN.md.
"""
from __future__ import annotations

import numpy as np

OP_CONT, OP_TEXT, OP_BIN, OP_CLOSE, OP_PING, OP_PONG = 0, 1, 2, 8, 9, 10
SEED_BASE = 0x57530001


def header_len(plen, masked=True, ext=None):
    plen = np.asarray(plen, dtype=np.uint64)
    if ext is None:
        ext = np.where(plen <= 125, 0, np.where(plen <= 65535, 2, 8))
    return 2 + np.asarray(ext) + (4 if masked is True else 4 * np.asarray(masked, dtype=np.int64))


def build_frames(b0, plen, mask, rng, masked=None, ext=None, seg_frames=None, fill=True):
    """Vectorised frame builder.

    b0[i]      first header byte (FIN | RSV | opcode)
    plen[i]    payload length
    mask[i]    mask key as little-endian u32 (wire byte 0 = bits 0..7)
    masked[i]  MASK bit (default all 1)
    ext[i]     forced extended-length width 0/2/8 (default minimal)
    seg_frames frames per segment (default: one segment)
    Returns (wire uint8[], seg_off uint64[n_segs+1], payload_off uint64[n]).
    """
    b0 = np.asarray(b0, dtype=np.uint8)
    plen = np.asarray(plen, dtype=np.uint64)
    mask = np.asarray(mask, dtype=np.uint32)
    n = len(plen)
    if masked is None:
        masked = np.ones(n, dtype=np.uint8)
    masked = np.asarray(masked, dtype=np.uint8)
    if ext is None:
        ext = np.where(plen <= 125, 0, np.where(plen <= 65535, 2, 8)).astype(np.int64)
    ext = np.asarray(ext, dtype=np.int64)
    hl = 2 + ext + 4 * masked.astype(np.int64)
    size = hl.astype(np.uint64) + plen
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(size, out=off[1:])
    total = int(off[-1])
    if fill:
        wire = np.frombuffer(rng.bytes(total), dtype=np.uint8).copy() if total else np.zeros(0, np.uint8)
    else:
        wire = np.zeros(total, dtype=np.uint8)
    h = off[:-1].astype(np.int64)
    len7 = np.where(ext == 0, plen, np.where(ext == 2, 126, 127)).astype(np.uint8)
    wire[h] = b0
    wire[h + 1] = (masked << 7) | len7
    e2 = ext == 2
    if e2.any():
        wire[h[e2] + 2] = ((plen[e2] >> 8) & 0xFF).astype(np.uint8)
        wire[h[e2] + 3] = (plen[e2] & 0xFF).astype(np.uint8)
    e8 = ext == 8
    if e8.any():
        for k in range(8):
            wire[h[e8] + 2 + k] = ((plen[e8] >> np.uint64(56 - 8 * k)) & np.uint64(0xFF)).astype(np.uint8)
    m = masked.astype(bool)
    if m.any():
        mb = h[m] + 2 + ext[m]
        for k in range(4):
            wire[mb + k] = ((mask[m] >> np.uint32(8 * k)) & 0xFF).astype(np.uint8)
    if seg_frames is None:
        seg_off = np.array([0, total], dtype=np.uint64)
    else:
        seg_frames = np.asarray(seg_frames, dtype=np.int64)
        assert seg_frames.sum() == n
        idx = np.zeros(len(seg_frames) + 1, dtype=np.int64)
        np.cumsum(seg_frames, out=idx[1:])
        seg_off = off[idx]
    return wire, seg_off, (off[:-1] + hl.astype(np.uint64))


def set_payload(wire, payload_off, mask, data: bytes):
    """Write `data` as the UNMASKED payload of a frame (stores data ^ mask on the wire)."""
    d = np.frombuffer(data, dtype=np.uint8)
    mb = np.array([(int(mask) >> (8 * k)) & 0xFF for k in range(4)], dtype=np.uint8)
    p = int(payload_off)
    wire[p:p + len(d)] = d ^ np.resize(mb, len(d))


def unmask_reference(wire, payload_off, plen, mask):
    """numpy restatement used for large-size checks in tests (websocket_frame.go:35-39)."""
    out = wire.copy()
    for p, L, m in zip(payload_off.tolist(), plen.tolist(), mask.tolist()):
        if L:
            mb = np.array([(m >> (8 * k)) & 0xFF for k in range(4)], dtype=np.uint8)
            out[p:p + L] ^= np.resize(mb, L)
    return out


# ---- BASELINE.json configs ---------------------------------------------------------------------
def uniform_batch(n_frames, size, frames_per_seg, seed, opcode=OP_BIN):
    """n_frames masked BIN frames of `size` payload bytes, grouped frames_per_seg per segment."""
    rng = np.random.default_rng(seed)
    b0 = np.full(n_frames, 0x80 | opcode, dtype=np.uint8)
    plen = np.full(n_frames, size, dtype=np.uint64)
    mask = rng.integers(0, 2**32, n_frames, dtype=np.uint64).astype(np.uint32)
    nseg = (n_frames + frames_per_seg - 1) // frames_per_seg
    segf = np.full(nseg, frames_per_seg, dtype=np.int64)
    segf[-1] = n_frames - frames_per_seg * (nseg - 1)
    wire, seg_off, poff = build_frames(b0, plen, mask, rng, seg_frames=segf)
    return dict(wire=wire, seg_off=seg_off, payload_off=poff, plen=plen, mask=mask,
                n_frames=n_frames, payload_bytes=int(plen.sum()))


def _splitmix64(x):
    """vectorised splitmix64 finaliser (counter-based: value = f(seed, index), order-free)"""
    x = np.asarray(x, dtype=np.uint64).copy()
    with np.errstate(over="ignore"):
        x += np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def dealt_uniform_batch(n_frames_total, size, frames_per_seg, seed, world, rank, opcode=OP_BIN):
    """Rank `rank`'s shard of ONE global batch of n_frames_total masked frames (configs[3]: 8 M x
    4 KiB over 8 GPUs): global connection segment g (frames_per_seg frames each) goes to rank
    shard.assign_segments(G, world)[g] = g mod world.  Every segment is generated from (seed, g)
    alone -- mask of global frame f = splitmix64(seed ^ f), payload bytes from
    default_rng([seed, g]) -- so the shards of all ranks are exactly split_batch() of the global
    batch (tests/test_shard.py) while each rank only materialises its own segments."""
    from netman_amd.shard import assign_segments
    G = (n_frames_total + frames_per_seg - 1) // frames_per_seg
    mine = np.nonzero(assign_segments(G, world) == rank)[0]
    segf = np.minimum(frames_per_seg, n_frames_total - mine * frames_per_seg).astype(np.int64)
    gframe = np.concatenate([g * frames_per_seg + np.arange(k, dtype=np.int64) for g, k in zip(mine, segf)]) \
        if len(mine) else np.zeros(0, np.int64)
    n = len(gframe)
    b0 = np.full(n, 0x80 | opcode, dtype=np.uint8)
    plen = np.full(n, size, dtype=np.uint64)
    mask = (_splitmix64(np.uint64(seed) ^ gframe.astype(np.uint64)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    wire, seg_off, poff = build_frames(b0, plen, mask, None, seg_frames=segf, fill=False)
    hl = int(header_len(size))
    for j, g in enumerate(mine):   # payload bytes of segment g: a function of (seed, g) only
        a, b = int(seg_off[j]), int(seg_off[j + 1])
        k = int(segf[j])
        pay = np.frombuffer(np.random.default_rng([seed, int(g)]).bytes(k * size), np.uint8).reshape(k, size)
        wire[a:b].reshape(k, hl + size)[:, hl:] = pay
    return dict(wire=wire, seg_off=seg_off, payload_off=poff, plen=plen, mask=mask, segments=mine,
                n_frames=n, payload_bytes=int(plen.sum()))


def utf8_units(rng, n_units):
    """n_units random 4-byte units, each valid UTF-8 on its own: 4 ASCII, 2 x 2-byte (Greek),
    3-byte (CJK) + ASCII, or one 4-byte character (emoji) -- uint8[4 * n_units]."""
    kind = rng.integers(0, 4, n_units)
    u = rng.integers(0x20, 0x7F, (n_units, 4)).astype(np.uint8)
    g = rng.integers(0x3B1, 0x3C9, (n_units, 2))                      # 2-byte: U+03B1..U+03C9
    m2 = kind == 1
    u[m2, 0] = (0xC0 | (g[m2, 0] >> 6)).astype(np.uint8)
    u[m2, 1] = (0x80 | (g[m2, 0] & 0x3F)).astype(np.uint8)
    u[m2, 2] = (0xC0 | (g[m2, 1] >> 6)).astype(np.uint8)
    u[m2, 3] = (0x80 | (g[m2, 1] & 0x3F)).astype(np.uint8)
    c = rng.integers(0x4E00, 0x9FFF, n_units)                        # 3-byte: CJK (+ 1 ASCII)
    m3 = kind == 2
    u[m3, 0] = (0xE0 | (c[m3] >> 12)).astype(np.uint8)
    u[m3, 1] = (0x80 | ((c[m3] >> 6) & 0x3F)).astype(np.uint8)
    u[m3, 2] = (0x80 | (c[m3] & 0x3F)).astype(np.uint8)
    e = rng.integers(0x1F300, 0x1F5FF, n_units)                      # 4-byte: emoji
    m4 = kind == 3
    u[m4, 0] = (0xF0 | (e[m4] >> 18)).astype(np.uint8)
    u[m4, 1] = (0x80 | ((e[m4] >> 12) & 0x3F)).astype(np.uint8)
    u[m4, 2] = (0x80 | ((e[m4] >> 6) & 0x3F)).astype(np.uint8)
    u[m4, 3] = (0x80 | (e[m4] & 0x3F)).astype(np.uint8)
    return u.reshape(-1)


def text_batch(n_frames, size, frames_per_seg, seed, ascii_only=False):
    """n_frames masked TEXT frames whose unmasked payload is valid UTF-8 (`size` bytes each:
    random 1-4 byte characters, or printable ASCII), grouped frames_per_seg per segment."""
    rng = np.random.default_rng(seed)
    b0 = np.full(n_frames, 0x80 | OP_TEXT, dtype=np.uint8)
    plen = np.full(n_frames, size, dtype=np.uint64)
    mask = rng.integers(0, 2**32, n_frames, dtype=np.uint64).astype(np.uint32)
    nseg = (n_frames + frames_per_seg - 1) // frames_per_seg
    segf = np.full(nseg, frames_per_seg, dtype=np.int64)
    segf[-1] = n_frames - frames_per_seg * (nseg - 1)
    wire, seg_off, poff = build_frames(b0, plen, mask, rng, seg_frames=segf, fill=False)
    body_len = size - size % 4
    pool_units = body_len // 4 + 1024
    pool = (rng.integers(0x20, 0x7F, 4 * pool_units).astype(np.uint8) if ascii_only
            else utf8_units(rng, pool_units))
    starts = rng.integers(0, 1024, n_frames) * 4            # unit-aligned: every slice is valid
    pad = np.full(size % 4, 0x61, np.uint8)                  # the tail is ASCII
    # masked payload = body ^ mask bytes (phase restarts at each payload start)
    mb = np.stack([(mask >> np.uint32(8 * k)) & 0xFF for k in range(4)], axis=1).astype(np.uint8)
    for i in range(n_frames):
        body = pool[starts[i]: starts[i] + body_len]
        if len(pad):
            body = np.concatenate([body, pad])
        p = int(poff[i])
        wire[p:p + size] = body ^ np.resize(mb[i], size)
    return dict(wire=wire, seg_off=seg_off, payload_off=poff, plen=plen, mask=mask,
                n_frames=n_frames, payload_bytes=int(plen.sum()))


def mixed_batch(n_frames=262144, seed=SEED_BASE + 2, frames_per_seg=16):
    """configs[2]: sizes {125, 65536, 1048576} with p proportional to 1/size, shuffled."""
    rng = np.random.default_rng(seed)
    sizes = np.array([125, 65536, 1048576], dtype=np.uint64)
    p = 1.0 / sizes.astype(np.float64)
    p /= p.sum()
    plen = sizes[rng.choice(3, size=n_frames, p=p)]
    b0 = np.full(n_frames, 0x82, dtype=np.uint8)
    mask = rng.integers(0, 2**32, n_frames, dtype=np.uint64).astype(np.uint32)
    nseg = (n_frames + frames_per_seg - 1) // frames_per_seg
    segf = np.full(nseg, frames_per_seg, dtype=np.int64)
    segf[-1] = n_frames - frames_per_seg * (nseg - 1)
    wire, seg_off, poff = build_frames(b0, plen, mask, rng, seg_frames=segf)
    return dict(wire=wire, seg_off=seg_off, payload_off=poff, plen=plen, mask=mask,
                n_frames=n_frames, payload_bytes=int(plen.sum()))


def fragmented_batch(n_conns=65536, seed=SEED_BASE + 4, ping_p=0.0, max_frag=8192):
    """configs[4]: per connection one message = chain of L~U{2..16} frames (BIN FIN=0, CONT FIN=0,
    ..., CONT FIN=1), fragment payload ~U{0..max_frag}; optional <=125 B PINGs inserted after a
    fragment with probability ping_p (variant B)."""
    rng = np.random.default_rng(seed)
    L = rng.integers(2, 17, n_conns)
    b0s, lens, segf = [], [], []
    for c in range(n_conns):
        cnt = 0
        for i in range(int(L[c])):
            first, last = i == 0, i == L[c] - 1
            op = OP_BIN if first else OP_CONT
            b0s.append((0x80 if last else 0) | op)
            lens.append(int(rng.integers(0, max_frag + 1)))
            cnt += 1
            if ping_p and not last and rng.random() < ping_p:
                b0s.append(0x80 | OP_PING)
                lens.append(int(rng.integers(0, 126)))
                cnt += 1
        segf.append(cnt)
    b0 = np.array(b0s, dtype=np.uint8)
    plen = np.array(lens, dtype=np.uint64)
    mask = rng.integers(0, 2**32, len(plen), dtype=np.uint64).astype(np.uint32)
    wire, seg_off, poff = build_frames(b0, plen, mask, rng, seg_frames=segf)
    return dict(wire=wire, seg_off=seg_off, payload_off=poff, plen=plen, mask=mask, b0=b0,
                n_frames=len(plen), payload_bytes=int(plen.sum()))


# ---- single frames (tests) -----------------------------------------------------------------------
def frame(op, payload: bytes = b"", fin=True, mask=None, masked=True, rsv=0, ext=None, rng=None):
    """One frame as bytes with an explicit UNMASKED payload."""
    if mask is None:
        rng = rng or np.random.default_rng(0)
        mask = int(rng.integers(0, 2**32))
    n = len(payload)
    if ext is None:
        ext = 0 if n <= 125 else (2 if n <= 65535 else 8)
    out = bytearray([(0x80 if fin else 0) | (rsv << 4) | op])
    len7 = n if ext == 0 else (126 if ext == 2 else 127)
    out.append((0x80 if masked else 0) | len7)
    if ext:
        out += n.to_bytes(ext, "big")
    if masked:
        mb = mask.to_bytes(4, "little")
        out += mb
        out += bytes(b ^ mb[i % 4] for i, b in enumerate(payload))
    else:
        out += payload
    return bytes(out)


def unmask_uniform(cfg):
    """vectorised websocket_frame.go:35-39 for batches whose frames all have one payload size"""
    plen = cfg["plen"]
    P = int(plen[0])
    assert (plen == P).all() and P % 4 == 0
    n = len(plen)
    wire = cfg["wire"]
    stride = len(wire) // n
    hdr = stride - P
    out = wire.copy().reshape(n, stride)
    mb = cfg["mask"].view(np.uint8).reshape(n, 1, 4)
    pay = out[:, hdr:].reshape(n, P // 4, 4)
    pay ^= mb
    return out.reshape(-1)
