// wsc_encode.hip -- gfx950 kernels of the batched server -> client framer.
//
// Replaces websocketProtocol.encode(firstByte, bs) (server/websocket_ctrl.go:23-70): firstByte,
// a minimal length (<=125: 1 byte; <=65535: 126 + u16 BE; else 127 + u64 BE), then the payload,
// unmasked.  Called per message in the reference by Text/Binary (websocket.go:378-398), pong
// (websocket_ctrl.go:140-143) and CloseCode (websocket_ctrl.go:108-109).  Here one launch pair
// frames a whole batch of messages back to back:
//   k_encode_scan  16 consecutive messages per lane: frame sizes, block scan + look-back -> out_off,
//                  and the output-window -> first-message index for the copy kernel.
//   k_encode_copy  one 4 KiB output window per wave, 16 B per lane, 1 KiB per wave instruction:
//                  a window inside one payload is a shifted stream copy (two aligned loads +
//                  alignbyte per 16 B); windows holding frame edges assemble header bytes in
//                  registers and OR in the payload bytes of every frame that overlaps them.
// Byte work, HBM-bound: no MFMA.  Algorithmic bytes per message: len read + (hl + len) written
// + 24 B descriptor + 8 B offset.
#include "wsc_kernels.hpp"
#include "wsc_dev.hpp"

namespace wsc {

__device__ __forceinline__ uint32_t enc_hlen(uint64_t len) { return len <= 125 ? 2u : (len <= 65535 ? 4u : 10u); }

// The header of one frame as 16 little-endian bytes (only the first enc_hlen(len) are used).
__device__ __forceinline__ void enc_header(uint32_t first_byte, uint64_t len, uint32_t (&h)[4]) {
    // written as selects (no branches) so the compiler keeps h in registers
    const bool l7 = len <= 125;                 // websocket_ctrl.go:33-37  one length byte
    const bool l16 = !l7 && len <= 65535;       // :39-49  126, uint16 big-endian
    const bool l64 = !l7 && !l16;               // :51-61  127, uint64 big-endian
    const uint64_t be = __builtin_bswap64(len);
    const uint32_t code = l7 ? (uint32_t)len : (l16 ? 126u : 127u);
    const uint32_t ext = l16 ? ((uint32_t)((len >> 8) & 0xFF) | (uint32_t)(len & 0xFF) << 8)
                             : (l64 ? (uint32_t)(be & 0xFFFF) : 0u);
    h[0] = first_byte | code << 8 | ext << 16;
    h[1] = l64 ? (uint32_t)(be >> 16) : 0u;
    h[2] = l64 ? (uint32_t)(be >> 48) : 0u;
    h[3] = 0;
}

// 16 bytes b = 0..15 with b -> h[b - d] (zero outside h's 16 bytes), for d in (-16, 16): a funnel
// of h with zeros (d >= 0: zeros then h from byte 16 - d; d < 0: h from byte -d then zeros)
__device__ __forceinline__ uint4 enc_place(const uint32_t (&h)[4], int32_t d) {
    const u32x4 H = {h[0], h[1], h[2], h[3]}, Z = {0u, 0u, 0u, 0u};
    const bool pos = d >= 0;
    const u32x4 o = funnel16(pos ? Z : H, pos ? H : Z, pos ? (uint32_t)(16 - d) : (uint32_t)(-d));
    return make_uint4(o.x, o.y, o.z, o.w);
}

// An aligned 16-byte output store.  NT bit 4: a buffer store over the output window with the
// in-place unmask's streaming policy (sc0 nt sc1) instead of a 64-bit global store.
template <int NT>
__device__ __forceinline__ void enc_st(uint8_t* out, uint64_t wbase, uint64_t pa, u32x4 v) {
    if constexpr ((NT & 16) != 0) st16b<19>(win_rsrc(out + wbase, ENC_WIN), (uint32_t)(pa - wbase), v);
    else st16v<NT>(out + pa, v);
}

__device__ __forceinline__ uint4 and4(const uint4& v, const uint32_t (&m)[4]) {
    return make_uint4(v.x & m[0], v.y & m[1], v.z & m[2], v.w & m[3]);
}

// byte masks of [lo, hi) within a 16-byte piece, per dword
__device__ __forceinline__ void piece_mask(uint32_t bl, uint32_t bh, uint32_t (&m)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t l = bl > 4u * j ? bl - 4u * j : 0u;
        const uint32_t hh = bh > 4u * j ? bh - 4u * j : 0u;
        m[j] = l < hh ? bytes_to_mask(l, hh > 4 ? 4 : hh) : 0u;
    }
}

// ---------------------------------------------------------------------------------------------
// Scan: frame sizes -> out_off (exclusive), window index.  Decoupled look-back as in the decoder's
// walk (wsc_kernels.hip): ticket block ids, self-tagged records (below), bounded spin.
// IPT consecutive messages per thread: 1 M messages in 256 blocks instead of 4,096 -- the scan
// went 68 -> 24 us at IPT 16 (8 per thread: 28 us, 32: 30 us).  The host picks the smallest IPT
// that keeps the grid within 256 blocks (wsc_api.cpp enc_scan_ipt): with few, large messages the
// window-index stores (16 per 64 KiB message) are the scan's work, so 16 Ki messages run at IPT 1
// on 64 CUs instead of IPT 16 on 4 (64 KiB encode 0.379 -> 0.360 ms, profiles/r05/ab6_enc_*.log;
// lanes taking messages 64 apart for coalesced loads and stores measured no faster: 1 KiB 0.437
// -> 0.442 ms).
// ---------------------------------------------------------------------------------------------
template <uint32_t IPT>
__global__ __launch_bounds__(256) void k_encode_scan(EncArgs a) {
    __shared__ uint32_t sh_bid;
    __shared__ uint64_t sh_wave[4];
    __shared__ uint64_t sh_prefix;
    if (threadIdx.x == 0)
        sh_bid = __hip_atomic_fetch_add(a.lb_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const uint32_t bid = sh_bid;
    const uint64_t i0 = ((uint64_t)bid * 256 + threadIdx.x) * IPT;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t sz[IPT];
    uint64_t tsz = 0;
#pragma unroll
    for (uint32_t j = 0; j < IPT; ++j) {
        sz[j] = 0;
        if (i0 + j < a.n_msgs) {
            const uint64_t len = a.msgs[i0 + j].len;
            sz[j] = enc_hlen(len) + len;
        }
        tsz += sz[j];
    }
    uint64_t inc = tsz;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(inc, d);
        if (lane >= (uint32_t)d) inc += o;
    }
    if (lane == 63) sh_wave[wave] = inc;
    __syncthreads();
    uint64_t wpre = 0, btot = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if ((uint32_t)q < wave) wpre += sh_wave[q];
        btot += sh_wave[q];
    }
    if (wave == 0) {
        // look-back records: one self-tagged word per block, kind (bits 62-63: 1 aggregate, 2
        // inclusive prefix, 0 not yet -- k_encode_copy re-arms them) over the 62-bit value, one
        // 8-byte agent-scope (sc1) store; a reader's one sc1 load gets status and value together
        // (the decoder's walk does the same with 8-word records, wsc_kernels.hip lb_publish)
        constexpr uint64_t VAL = (1ull << 62) - 1;
        if (lane == 0)
            __hip_atomic_store(a.lb_rec + bid, (bid == 0 ? 2ull : 1ull) << 62 | (btot & VAL), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        uint64_t prefix = 0;
        int64_t j0 = (int64_t)bid - 1;
        uint32_t spins = 0;
        while (j0 >= 0) {
            const int64_t j = j0 - (int64_t)lane;
            const uint64_t r = j >= 0 ? __hip_atomic_load(a.lb_rec + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : 2ull << 62;   // before block 0: an inclusive prefix of zero
            const uint32_t f = (uint32_t)(r >> 62);
            const uint64_t m2 = __ballot(f == 2);
            const uint64_t m0 = __ballot(f == 0);
            const uint32_t first2 = m2 ? (uint32_t)__builtin_ctzll(m2) : 64u;
            const uint64_t need = first2 >= 63 ? ~0ull : ((2ull << first2) - 1);
            if (m0 & need) {
                if (++spins > (1u << 22)) {
                    if (lane == 0) __hip_atomic_fetch_or(a.lb_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            uint64_t v = lane <= first2 ? (r & VAL) : 0ull;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
            prefix += v;
            if (first2 < 64) break;
            j0 -= 64;
        }
        if (lane == 0) {
            if (bid != 0)
                __hip_atomic_store(a.lb_rec + bid, 2ull << 62 | ((prefix + btot) & VAL), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            sh_prefix = prefix;
        }
    }
    __syncthreads();
    uint64_t off = sh_prefix + wpre + (inc - tsz);
#pragma unroll
    for (uint32_t j = 0; j < IPT; ++j) {
        const uint64_t i = i0 + j;
        if (i >= a.n_msgs) break;
        a.out_off[i] = off;
        // windows that start inside this frame: [ceil(off / W), floor((off + sz - 1) / W)]
        uint64_t w = (off + ENC_WIN - 1) >> ENC_WIN_SHIFT;
        uint64_t w_end = ((off + sz[j] - 1) >> ENC_WIN_SHIFT) + 1;
        if (w_end > a.tile_entries) w_end = a.tile_entries;
        for (; w < w_end; ++w) a.tile[w] = (uint32_t)i;
        off += sz[j];
        if (i == a.n_msgs - 1) {
            uint64_t total = off;
            if (__hip_atomic_load(a.lb_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                total = ~0ull;   // invalid
                __hip_atomic_fetch_or(a.sticky, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            a.out_off[a.n_msgs] = total;
        }
    }
}

// General output window, lane-parallel (the decoder's unmask_window_lanes, for frames): the wave
// loads the frames overlapping the window into lanes (frame m + lane), each lane binary-searches
// them (ds_bpermute) for the frame holding its 16-byte piece and assembles the piece from that
// frame and the next -- header bytes from registers, payload bytes by unaligned gathers issued
// together; pieces meeting 3+ frames (frames shorter than 16 B) take a uniform tail loop.  Returns
// false (nothing written) when more than 64 frames overlap the window.
// byte masks from the 17-entry LDS prefix table (the unmask's idea, wsc_unmask.inl): the bytes
// [lo, hi) of a 16-byte piece are pm[hi] & ~pm[lo]
__device__ __forceinline__ void pm_mask(const u32x4* __restrict__ pm, uint32_t lo, uint32_t hi, uint32_t (&m)[4]) {
    const u32x4 h = pm[hi], l = pm[lo];
    m[0] = h[0] & ~l[0]; m[1] = h[1] & ~l[1]; m[2] = h[2] & ~l[2]; m[3] = h[3] & ~l[3];
}

// Two passes: (1) every piece lying inside one payload is a plain gather + store (the common case
// even at 1 KiB frames: ~4 frame edges in 256 pieces); (2) the pieces holding a header or a frame
// edge are compacted into lanes (LDS list, in window order) and assembled together -- one pass
// of the costly header placement per window instead of one per 1 KiB slice (PMC: the slice-wise
// version issued ~600 VALU per window at 1 KiB frames, past the HBM budget).
// Frames base + lane in lanes, absolute output offsets: header start o, payload start p, end e
// (all ~0 past the last frame), source offset of output byte x = so + x, the header's bytes.
struct EncLanes {
    uint64_t o, p, e;
    int64_t so;
    uint32_t h[3];
};
__device__ __forceinline__ EncLanes enc_lanes_load(const EncCopyArgs& a, uint32_t base, uint32_t lane) {
    EncLanes L;
    L.o = L.p = L.e = ~0ull;
    L.so = 0;
    L.h[0] = L.h[1] = L.h[2] = 0;
    if (base + lane < a.n_msgs) {
        const wsc_out_msg mj = a.msgs[base + lane];
        L.o = a.out_off[base + lane];
        L.p = L.o + enc_hlen(mj.len);
        L.e = L.p + mj.len;
        uint32_t h[4];
        enc_header(mj.first_byte, mj.len, h);
        L.h[0] = h[0];
        L.h[1] = h[1];
        L.h[2] = h[2];
        L.so = (int64_t)mj.src_off - (int64_t)L.p;
    }
    return L;
}

template <int NT>
__device__ __forceinline__ bool encode_window_lanes(const EncCopyArgs& a, const EncLanes& L, uint32_t base, uint64_t wbase,
                                                    uint64_t limit, uint32_t lane, const u32x4* __restrict__ pm,
                                                    uint16_t* __restrict__ elist) {
    constexpr uint32_t P = ENC_WIN / 1024;
    constexpr int64_t WB = ENC_WIN;
    auto clip = [](uint64_t x, uint64_t wb) -> int32_t {   // x - wb clamped to [-2^30, WB + 64]
        if (x == ~0ull || x > wb + (uint64_t)(WB + 64)) return (int32_t)WB + 64;
        return x + (1ull << 30) < wb ? -(1 << 30) : (int32_t)((int64_t)x - (int64_t)wb);
    };
    // window-relative header start, payload start, end (lanes before the window's first frame lie
    // before it: the search below never lands on them)
    const int32_t ro = clip(L.o, wbase), rp = clip(L.p, wbase), re = clip(L.e, wbase);
    const uint32_t h[4] = {L.h[0], L.h[1], L.h[2], 0u};
    const int64_t so = L.so;
    const uint32_t nl = (uint32_t)__builtin_popcountll(__ballot(ro < (int32_t)WB));
    if (nl == 64 && __shfl(re, 63) < (int32_t)WB && base + 64 < a.n_msgs) return false;
    const uint32_t so_lo = (uint32_t)so, so_hi = (uint32_t)((uint64_t)so >> 32);

    // binary search: the last frame (lane) whose header starts at or before window byte pr; first
    // step = the power of two with 2*st0 > nl (wave-uniform), as many steps as the window needs
    const int32_t st0 = nl == 0 ? 0 : (nl >= 32 ? 32 : (int32_t)((1u << (32 - __builtin_clz(nl))) >> 1));
    auto find = [&](int32_t pr) -> int32_t {
        int32_t lo = -1;
        for (int32_t st = st0; st >= 1; st >>= 1) {
            const int32_t c = lo + st;
            const int32_t dv = __shfl(ro, c & 63);
            if (c < (int32_t)nl && dv <= pr) lo = c;
        }
        return lo < 0 ? 0 : lo;
    };
    auto store_piece = [&](uint64_t pa, const uint4& v) {
        if (pa + 16 <= limit) {
            enc_st<NT>(a.out, wbase, pa, u32x4{v.x, v.y, v.z, v.w});
        } else {   // the tail piece: never write at or past the total / out_cap
            const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (uint32_t b = 0; b < 16; ++b)
                if (pa + b < limit) a.out[pa + b] = (uint8_t)(d[b >> 2] >> (8 * (b & 3)));
        }
    };
    // ---- pass 1: pieces inside one payload ----
    // all P gathers issued before the first store: one memory round trip for the window (with a
    // load and its store in one iteration the compiler waited on each load in turn -- the branchy
    // edge path of load16_unaligned keeps it from hoisting the next load over the store)
    uint32_t n_edge = 0;
    uint4 v[P];
    bool ins[P];
#pragma unroll
    for (uint32_t k = 0; k < P; ++k) {
        const int32_t pr = (int32_t)(k * 1024 + lane * 16);
        const uint64_t pa = wbase + (uint64_t)pr;
        const int32_t t = find(pr);
        const int32_t fp = __shfl(rp, t & 63), fe = __shfl(re, t & 63);
        const uint32_t sl = __shfl(so_lo, t & 63), sh = __shfl(so_hi, t & 63);
        const bool inside = t < (int32_t)nl && fp <= pr && pr + 16 <= fe && pa + 16 <= limit;
        ins[k] = inside;
        if (inside) v[k] = load16_unaligned(a.src, (int64_t)((uint64_t)sh << 32 | sl) + (int64_t)pa, a.src_bytes);
        const bool edge = !inside && pa < limit;
        const uint64_t em = __ballot(edge);
        if (edge)
            elist[n_edge + __builtin_amdgcn_mbcnt_hi((uint32_t)(em >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)em, 0u))] =
                (uint16_t)(k * 64 + lane);
        n_edge += (uint32_t)__builtin_popcountll(em);
    }
#pragma unroll
    for (uint32_t k = 0; k < P; ++k) {
        const uint64_t pa = wbase + k * 1024u + lane * 16u;
        if (ins[k]) enc_st<NT>(a.out, wbase, pa, u32x4{v[k].x, v[k].y, v[k].z, v[k].w});
    }
    if (n_edge == 0) return true;
    __builtin_amdgcn_wave_barrier();
    // ---- pass 2: pieces holding headers / frame edges, one per lane ----
    // one frame's contribution to a piece: header bytes from registers, payload by a gather
    // (split in two: the payload gathers of a piece's two frames are issued together, then the
    // piece is assembled -- with the gather and its use in one step, the two waited in turn)
    struct Part {
        int32_t fo, fp, fe;
        uint32_t hh[3];
        bool ok;
        uint4 pay;   // the 16 source bytes under the piece (when the payload meets it)
    };
    auto part_load = [&](int32_t t, int32_t pr) -> Part {
        Part q;
        q.fo = __shfl(ro, t & 63);
        q.fp = __shfl(rp, t & 63);
        q.fe = __shfl(re, t & 63);
        q.hh[0] = __shfl(h[0], t & 63);
        q.hh[1] = __shfl(h[1], t & 63);
        q.hh[2] = __shfl(h[2], t & 63);
        const uint32_t sl = __shfl(so_lo, t & 63), sh = __shfl(so_hi, t & 63);
        q.ok = t < (int32_t)nl;
        q.pay = make_uint4(0, 0, 0, 0);
        const int32_t lo = q.fp > pr ? q.fp : pr, hi = q.fe < pr + 16 ? q.fe : pr + 16;
        if (q.ok && lo < hi)
            q.pay = load16_unaligned(a.src, (int64_t)((uint64_t)sh << 32 | sl) + (int64_t)wbase + pr, a.src_bytes);
        return q;
    };
    // one frame's contribution to a piece: header bytes from registers, payload from the gather
    auto part_add = [&](const Part& q, int32_t pr, uint4& acc, bool& ends_inside) {
        ends_inside = false;
        if (!q.ok) return;
        uint32_t msk[4];
        int32_t lo = q.fo > pr ? q.fo : pr, hi = q.fp < pr + 16 ? q.fp : pr + 16;
        if (lo < hi) {
            const uint32_t hh[4] = {q.hh[0], q.hh[1], q.hh[2], 0u};
            pm_mask(pm, (uint32_t)(lo - pr), (uint32_t)(hi - pr), msk);
            const uint4 t4 = and4(enc_place(hh, q.fo - pr), msk);
            acc.x |= t4.x; acc.y |= t4.y; acc.z |= t4.z; acc.w |= t4.w;
        }
        lo = q.fp > pr ? q.fp : pr;
        hi = q.fe < pr + 16 ? q.fe : pr + 16;
        if (lo < hi) {
            pm_mask(pm, (uint32_t)(lo - pr), (uint32_t)(hi - pr), msk);
            const uint4 t4 = and4(q.pay, msk);
            acc.x |= t4.x; acc.y |= t4.y; acc.z |= t4.z; acc.w |= t4.w;
        }
        ends_inside = q.fe < pr + 16;
    };
    auto part = [&](int32_t t, int32_t pr, uint4& acc, bool& ends_inside) { part_add(part_load(t, pr), pr, acc, ends_inside); };
    for (uint32_t base = 0; base < n_edge; base += 64) {
        const bool act = base + lane < n_edge;
        const uint32_t pid = act ? elist[base + lane] : 0u;
        const int32_t pr = (int32_t)((pid >> 6) * 1024 + (pid & 63) * 16);
        const int32_t ta = find(pr);
        uint4 acc = make_uint4(0, 0, 0, 0);
        bool ea, eb;
        const Part qa = part_load(ta, pr), qb = part_load(ta + 1, pr);
        part_add(qa, pr, acc, ea);
        part_add(qb, pr, acc, eb);
        // rare: frames shorter than 16 B -> a third, fourth ... frame in a piece
        int32_t t = ta + 2;
        bool more = act && ea && eb && t < (int32_t)nl;
        while (__ballot(more)) {
            const int32_t fo = __shfl(ro, t & 63);
            more = more && t < (int32_t)nl && fo < pr + 16;
            uint4 tmp = make_uint4(0, 0, 0, 0);
            bool e;
            part(t, pr, tmp, e);
            if (more) { acc.x |= tmp.x; acc.y |= tmp.y; acc.z |= tmp.z; acc.w |= tmp.w; }
            ++t;
        }
        if (act) store_piece(wbase + (uint64_t)pr, acc);
    }
    return true;
}

// The same window in one memory round trip, when it can: every gather of both passes -- the
// pieces inside one payload and the two frames' payload bytes under each edge piece -- is issued
// before any is waited on, as plain 16-byte loads (a lane with nothing to gather reads src + 0).
// Taken when the window has at most 64 edge pieces (a piece meeting a third frame -- frames under
// 16 B -- gathers it in the loop at the end) and every gather lies inside src (a wave-uniform test; load16_unaligned's byte path for the ends
// of src made the compiler wait on each gather in turn).  Returns false, having written nothing,
// when it cannot: encode_window_lanes then takes the window.
template <int NT>
__device__ __forceinline__ bool encode_window_direct(const EncCopyArgs& a, const EncLanes& L, uint32_t base, uint64_t wbase,
                                                     uint64_t limit, uint32_t lane, const u32x4* __restrict__ pm,
                                                     uint16_t* __restrict__ elist) {
    constexpr uint32_t P = ENC_WIN / 1024;
    constexpr int64_t WB = ENC_WIN;
    if (a.src_bytes < 16) return false;
    const int64_t smax = (int64_t)a.src_bytes - 16;
    // (clip and find repeat encode_window_lanes' on purpose: shared as __device__ helpers the kernel
    // compiled to 82 VGPRs, 5 waves per SIMD, and the 1 KiB encode ran 0.429 -> 0.437 ms)
    auto clip = [](uint64_t x, uint64_t wb) -> int32_t {   // as in encode_window_lanes
        if (x == ~0ull || x > wb + (uint64_t)(WB + 64)) return (int32_t)WB + 64;
        return x + (1ull << 30) < wb ? -(1 << 30) : (int32_t)((int64_t)x - (int64_t)wb);
    };
    const int32_t ro = clip(L.o, wbase), rp = clip(L.p, wbase), re = clip(L.e, wbase);
    const uint32_t h[4] = {L.h[0], L.h[1], L.h[2], 0u};
    const uint32_t so_lo = (uint32_t)L.so, so_hi = (uint32_t)((uint64_t)L.so >> 32);
    const uint32_t nl = (uint32_t)__builtin_popcountll(__ballot(ro < (int32_t)WB));
    if (nl == 64 && __shfl(re, 63) < (int32_t)WB && base + 64 < a.n_msgs) return false;
    const int32_t st0 = nl == 0 ? 0 : (nl >= 32 ? 32 : (int32_t)((1u << (32 - __builtin_clz(nl))) >> 1));
    auto find = [&](int32_t pr) -> int32_t {
        int32_t lo = -1;
        for (int32_t st = st0; st >= 1; st >>= 1) {
            const int32_t c = lo + st;
            const int32_t dv = __shfl(ro, c & 63);
            if (c < (int32_t)nl && dv <= pr) lo = c;
        }
        return lo < 0 ? 0 : lo;
    };
    auto src_of = [&](int32_t t) -> int64_t {   // frame t's source offset of output byte x: so + x
        const uint32_t sl = __shfl(so_lo, t & 63), sh = __shfl(so_hi, t & 63);
        return (int64_t)((uint64_t)sh << 32 | sl);
    };
    bool safe = true;
    // pass 1's pieces: inside one payload -> gather address; otherwise listed as an edge piece
    uint32_t n_edge = 0;
    int64_t g1[P];
    bool ins[P];
#pragma unroll
    for (uint32_t k = 0; k < P; ++k) {
        const int32_t pr = (int32_t)(k * 1024 + lane * 16);
        const uint64_t pa = wbase + (uint64_t)pr;
        const int32_t t = find(pr);
        const int32_t fp = __shfl(rp, t & 63), fe = __shfl(re, t & 63);
        const int64_t g = src_of(t) + (int64_t)pa;
        const bool inside = t < (int32_t)nl && fp <= pr && pr + 16 <= fe && pa + 16 <= limit;
        ins[k] = inside;
        g1[k] = inside ? g : 0;
        safe = safe && (!inside || (g >= 0 && g <= smax));
        const bool edge = !inside && pa < limit;
        const uint64_t em = __ballot(edge);
        if (edge)
            elist[n_edge + __builtin_amdgcn_mbcnt_hi((uint32_t)(em >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)em, 0u))] =
                (uint16_t)(k * 64 + lane);
        n_edge += (uint32_t)__builtin_popcountll(em);
    }
    if (n_edge > 64) return false;
    __builtin_amdgcn_wave_barrier();
    // pass 2's pieces, one per lane: the frame holding the piece's first byte (a) and the next (b)
    const bool act = lane < n_edge;
    const uint32_t pid = act ? elist[lane] : 0u;
    const int32_t pr2 = (int32_t)((pid >> 6) * 1024 + (pid & 63) * 16);
    const int32_t ta = find(pr2);
    struct Meta { int32_t fo, fp, fe; uint32_t hh[3]; bool ok; int64_t g; };
    auto meta = [&](int32_t t) -> Meta {
        Meta q;
        q.fo = __shfl(ro, t & 63);
        q.fp = __shfl(rp, t & 63);
        q.fe = __shfl(re, t & 63);
        q.hh[0] = __shfl(h[0], t & 63);
        q.hh[1] = __shfl(h[1], t & 63);
        q.hh[2] = __shfl(h[2], t & 63);
        q.ok = act && t < (int32_t)nl;
        const int32_t lo = q.fp > pr2 ? q.fp : pr2, hi = q.fe < pr2 + 16 ? q.fe : pr2 + 16;
        const int64_t g = src_of(t) + (int64_t)wbase + pr2;
        const bool need = q.ok && lo < hi;
        q.g = need ? g : 0;
        safe = safe && (!need || (g >= 0 && g <= smax));
        return q;
    };
    const Meta qa = meta(ta), qb = meta(ta + 1);
    if (__ballot(!safe)) return false;
    // every gather at once
    auto ld = [&](int64_t g) -> uint4 {
        const u32x4u_ld t = *reinterpret_cast<const u32x4u_ld*>(a.src + g);
        return make_uint4(t.x, t.y, t.z, t.w);
    };
    uint4 v[P];
#pragma unroll
    for (uint32_t k = 0; k < P; ++k) v[k] = ld(g1[k]);
    const uint4 pay_a = ld(qa.g), pay_b = ld(qb.g);
#pragma unroll
    for (uint32_t k = 0; k < P; ++k) {
        const uint64_t pa = wbase + k * 1024u + lane * 16u;
        if (ins[k]) enc_st<NT>(a.out, wbase, pa, u32x4{v[k].x, v[k].y, v[k].z, v[k].w});
    }
    if (n_edge == 0) return true;
    // assemble the edge pieces: header bytes from registers, payload bytes from the gathers
    auto add = [&](const Meta& q, const uint4& pay, uint4& acc) -> bool {
        if (!q.ok) return false;
        uint32_t msk[4];
        int32_t lo = q.fo > pr2 ? q.fo : pr2, hi = q.fp < pr2 + 16 ? q.fp : pr2 + 16;
        if (lo < hi) {
            const uint32_t hh[4] = {q.hh[0], q.hh[1], q.hh[2], 0u};
            pm_mask(pm, (uint32_t)(lo - pr2), (uint32_t)(hi - pr2), msk);
            const uint4 t4 = and4(enc_place(hh, q.fo - pr2), msk);
            acc.x |= t4.x; acc.y |= t4.y; acc.z |= t4.z; acc.w |= t4.w;
        }
        lo = q.fp > pr2 ? q.fp : pr2;
        hi = q.fe < pr2 + 16 ? q.fe : pr2 + 16;
        if (lo < hi) {
            pm_mask(pm, (uint32_t)(lo - pr2), (uint32_t)(hi - pr2), msk);
            const uint4 t4 = and4(pay, msk);
            acc.x |= t4.x; acc.y |= t4.y; acc.z |= t4.z; acc.w |= t4.w;
        }
        return q.fe < pr2 + 16;
    };
    uint4 acc = make_uint4(0, 0, 0, 0);
    const bool ea = add(qa, pay_a, acc);
    const bool eb = add(qb, pay_b, acc);
    // rare: frames shorter than 16 B -> a third, fourth ... frame in a piece (one gather each)
    int32_t t = ta + 2;
    bool more = act && ea && eb && t < (int32_t)nl;
    while (__ballot(more)) {
        const int32_t fo = __shfl(ro, t & 63);
        more = more && t < (int32_t)nl && fo < pr2 + 16;
        Meta q = meta(t);
        q.ok = q.ok && more;
        const uint4 pay = load16_unaligned(a.src, q.g, a.src_bytes);   // (q.g = 0 when unused: a harmless read)
        uint4 tmp = make_uint4(0, 0, 0, 0);
        add(q, pay, tmp);
        acc.x |= tmp.x; acc.y |= tmp.y; acc.z |= tmp.z; acc.w |= tmp.w;
        ++t;
    }
    if (act) {
        const uint64_t pa = wbase + (uint64_t)pr2;
        if (pa + 16 <= limit) {
            enc_st<NT>(a.out, wbase, pa, u32x4{acc.x, acc.y, acc.z, acc.w});
        } else {   // the tail piece: never write at or past the total / out_cap
            const uint32_t d[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
            for (uint32_t b = 0; b < 16; ++b)
                if (pa + b < limit) a.out[pa + b] = (uint8_t)(d[b >> 2] >> (8 * (b & 3)));
        }
    }
    return true;
}

// A window with more than 64 frames: frame by frame from m, every lane assembling its P pieces.
template <int NT>
__device__ __forceinline__ void encode_window_serial(const EncCopyArgs& a, uint32_t m, uint64_t wbase, uint64_t limit,
                                                  uint32_t lane) {
    constexpr uint32_t P = ENC_WIN / 1024;
    const uint32_t lofs = lane * 16u, n = a.n_msgs;
    uint4 acc[P];
#pragma unroll
    for (uint32_t k = 0; k < P; ++k) acc[k] = make_uint4(0, 0, 0, 0);
    for (uint32_t j = m; j < n; ++j) {
        const uint64_t oj = a.out_off[j];
        if (oj >= wbase + ENC_WIN) break;
        const wsc_out_msg mj = a.msgs[j];
        const uint32_t hl = enc_hlen(mj.len);
        uint32_t h[4];
        enc_header(mj.first_byte, mj.len, h);
        const uint64_t pj = oj + hl, ej = pj + mj.len;
#pragma unroll
        for (uint32_t k = 0; k < P; ++k) {
            const uint64_t pa = wbase + k * 1024u + lofs;
            uint32_t msk[4];
            // header bytes [oj, pj)
            uint64_t lo = oj > pa ? oj : pa;
            uint64_t hi = pj < pa + 16 ? pj : pa + 16;
            if (lo < hi) {
                piece_mask((uint32_t)(lo - pa), (uint32_t)(hi - pa), msk);
                const uint4 hv = enc_place(h, (int32_t)((int64_t)oj - (int64_t)pa));
                const uint4 t = and4(hv, msk);
                acc[k].x |= t.x; acc[k].y |= t.y; acc[k].z |= t.z; acc[k].w |= t.w;
            }
            // payload bytes [pj, ej)
            lo = pj > pa ? pj : pa;
            hi = ej < pa + 16 ? ej : pa + 16;
            if (lo < hi) {
                piece_mask((uint32_t)(lo - pa), (uint32_t)(hi - pa), msk);
                const uint4 sv = load16_unaligned(a.src, (int64_t)mj.src_off + ((int64_t)pa - (int64_t)pj), a.src_bytes);
                const uint4 t = and4(sv, msk);
                acc[k].x |= t.x; acc[k].y |= t.y; acc[k].z |= t.z; acc[k].w |= t.w;
            }
        }
        if (ej >= wbase + ENC_WIN) break;   // this frame runs past the window
    }
#pragma unroll
    for (uint32_t k = 0; k < P; ++k) {
        const uint64_t pa = wbase + k * 1024u + lofs;
        if (pa >= limit) continue;
        if (pa + 16 <= limit) {
            enc_st<NT>(a.out, wbase, pa, u32x4{acc[k].x, acc[k].y, acc[k].z, acc[k].w});
        } else {   // the tail piece: never write at or past the total / out_cap
            const uint32_t d[4] = {acc[k].x, acc[k].y, acc[k].z, acc[k].w};
#pragma unroll
            for (uint32_t b = 0; b < 16; ++b)   // unrolled: constant register indices, no scratch
                if (pa + b < limit) a.out[pa + b] = (uint8_t)(d[b >> 2] >> (8 * (b & 3)));
        }
    }
}

// fast path: the window lies inside one payload -> shifted stream copy, non-temporal loads (A/B,
// tools/lib_ab.py: 64 KiB echo batch 0.411 -> 0.396 ms; the lane-parallel windows keep default
// loads: their pieces at frame edges re-read lines a neighbour piece loaded, and nt loads made the
// 1 KiB batch 3.5 % slower)
template <int NT>
__device__ __forceinline__ void encode_window_inside(const EncCopyArgs& a, int64_t so, uint64_t wbase, uint32_t lane) {
    constexpr uint32_t P = ENC_WIN / 1024;
    const uint32_t lofs = lane * 16u;
    uint4 v[P];
#pragma unroll
    for (uint32_t k = 0; k < P; ++k) v[k] = load16u<NT>(a.src, so + (int64_t)(wbase + k * 1024u + lofs), a.src_bytes);
#pragma unroll
    for (uint32_t k = 0; k < P; ++k) enc_st<NT>(a.out, wbase, wbase + k * 1024u + lofs, u32x4{v[k].x, v[k].y, v[k].z, v[k].w});
}

__device__ __forceinline__ void enc_pm_init(u32x4* pm) {
    if (threadIdx.x < 17) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t L = threadIdx.x;
            const uint32_t nb = L > 4u * j ? (L - 4u * j > 4u ? 4u : L - 4u * j) : 0u;
            pm[threadIdx.x][j] = nb == 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Copy: one ENC_WIN-byte output window per wave.
// ---------------------------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(256) void k_encode_copy(EncCopyArgs a) {
    __shared__ u32x4 pm[17];
    __shared__ uint16_t elist[4][ENC_WIN / 16];   // per wave: the window's edge pieces (pass 2)
    enc_pm_init(pm);
    __syncthreads();
    // re-arm the scan's look-back state for the next encode (this launch is ordered after it)
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < a.n_lb; t += gridDim.x * blockDim.x) {
        a.lb_state[t] = 0;
        a.lb_rec[t] = 0;   // (n_lb = scan blocks + 2 >= the records written)
    }
    const uint32_t n = a.n_msgs;
    if (n == 0) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t gw = __builtin_amdgcn_readfirstlane(xcd_run_block(blockIdx.x, gridDim.x, a.xcd_run) * 4 +
                                                       (threadIdx.x >> 6));
    uint64_t limit = a.out_off[n];
    if (limit > a.out_cap) limit = a.out_cap;
    const uint64_t wbase = gw << ENC_WIN_SHIFT;
    if (wbase >= limit || gw >= a.tile_entries) return;
    const uint32_t m = a.tile[gw];
    const wsc_out_msg mm = a.msgs[m];
    const uint64_t o = a.out_off[m];
    // the frames from m in lanes: with small messages (most windows hold frame edges: a.hoist)
    // loaded beside m's own descriptor -- the general path's next round trip; with large ones only
    // when the window is not inside one payload (1 KiB encode 0.4325 -> 0.4279 ms hoisted, 64 KiB
    // 0.3508 -> 0.3446 ms not: interleaved A/B, profiles/r06/enc_direct_ab.log)
    EncLanes L;
    if (a.hoist) L = enc_lanes_load(a, m, lane);
    const uint64_t p0 = o + enc_hlen(mm.len), p1 = p0 + mm.len;
    if (p0 <= wbase && p1 >= wbase + ENC_WIN && wbase + ENC_WIN <= limit) {
        encode_window_inside<NT>(a, (int64_t)mm.src_off - (int64_t)p0, wbase, lane);
        return;
    }
    if (!a.hoist) L = enc_lanes_load(a, m, lane);
    // general path: frame edges in the window -> lane-parallel frame lookup (serial walk over the
    // frames only when more than 64 of them overlap the window)
    if (encode_window_direct<NT>(a, L, m, wbase, limit, lane, pm, elist[threadIdx.x >> 6])) return;
    if (encode_window_lanes<NT>(a, L, m, wbase, limit, lane, pm, elist[threadIdx.x >> 6])) return;
    encode_window_serial<NT>(a, m, wbase, limit, lane);
}

template __global__ void k_encode_scan<1>(EncArgs);
template __global__ void k_encode_scan<4>(EncArgs);
template __global__ void k_encode_scan<16>(EncArgs);
template __global__ void k_encode_copy<3>(EncCopyArgs);

}  // namespace wsc
