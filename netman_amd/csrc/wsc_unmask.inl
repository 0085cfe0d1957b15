// wsc_unmask.inl -- the unmask kernel template (the hot loop, websocket_frame.go:35-39), shared by
// the two translation units that instantiate it (wsc_unmask_inplace.hip, wsc_unmask_compact.hip)
// so that hipcc compiles the variants in parallel.
#pragma once
#include "wsc_kernels.hpp"
#include "wsc_dev.hpp"

namespace wsc {

// ---------------------------------------------------------------------------------------------
// Unmask: the hot loop.  The destination byte range is cut into windows of P KiB; wave w owns
// window w (grid-stride).  tile_first[w] names the first span whose destination ends after the
// window start, so the wave walks only the spans that overlap its window (scalar loads).  Each
// lane holds P pieces of 16 B at dst + w*W + k*1024 + lane*16: every wave instruction touches
// 1 KiB contiguous.  For each overlapping span a lane ORs the span's rotated mask word into the
// bytes of its pieces that the span covers, then XORs and stores once.
// ---------------------------------------------------------------------------------------------

// General window: several spans overlap it (small frames), or it is the last, partial window.
// Builds a per-byte key from every span that overlaps each 16-byte piece.
template <bool COMPACT, int P, int NT>
__device__ __attribute__((noinline)) void unmask_window_general(
    uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t src_bytes, uint64_t total,
    const Span* __restrict__ spans, uint32_t n_spans, uint32_t r, uint64_t wbase, uint32_t lofs) {
    constexpr uint32_t WB = 1024u * P;
    uint4 v[P], key[P];
    uint32_t cov[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        key[k] = make_uint4(0, 0, 0, 0);
        cov[k] = 0;
        v[k] = make_uint4(0, 0, 0, 0);
        if constexpr (!COMPACT) {
            const uint64_t addr = wbase + k * 1024u + lofs;
            if (addr + 16 <= total) v[k] = ld16<NT>(dst + addr);
        }
    }
    for (; r < n_spans; ++r) {
        const Span sp = spans[r];
        if (sp.dst >= wbase + WB) break;
        const uint64_t d0 = sp.dst, d1 = sp.dst + sp.len;
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const uint64_t pa = wbase + k * 1024u + lofs;
            const uint64_t lo = d0 > pa ? d0 : pa;
            const uint64_t hi = d1 < pa + 16 ? d1 : pa + 16;
            if (lo < hi) {
                const uint32_t bl = (uint32_t)(lo - pa), bh = (uint32_t)(hi - pa);
                uint32_t m[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t l = bl > 4u * j ? bl - 4u * j : 0u;
                    const uint32_t hh = bh > 4u * j ? bh - 4u * j : 0u;
                    m[j] = l < hh ? bytes_to_mask(l, hh > 4 ? 4 : hh) : 0u;
                }
                key[k].x |= sp.key & m[0];
                key[k].y |= sp.key & m[1];
                key[k].z |= sp.key & m[2];
                key[k].w |= sp.key & m[3];
                cov[k] |= 1u;
                if constexpr (COMPACT) {
                    const int64_t so = (int64_t)sp.src + ((int64_t)pa - (int64_t)sp.dst);
                    const uint4 sv = load16_unaligned(src, so, src_bytes);
                    v[k].x |= sv.x & m[0];
                    v[k].y |= sv.y & m[1];
                    v[k].z |= sv.z & m[2];
                    v[k].w |= sv.w & m[3];
                }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        if (!cov[k]) continue;
        const uint64_t addr = wbase + k * 1024u + lofs;
        uint4 o = v[k];
        o.x ^= key[k].x; o.y ^= key[k].y; o.z ^= key[k].z; o.w ^= key[k].w;
        if (COMPACT || addr + 16 <= total) {
            st16<NT>(dst + addr, o);
        } else {
            // in-place tail piece past the last full 16 B of the buffer: byte stores
            const uint32_t kd[4] = {key[k].x, key[k].y, key[k].z, key[k].w};
            for (uint32_t j = 0; addr + j < total; ++j)
                dst[addr + j] ^= (uint8_t)(kd[j >> 2] >> (8 * (j & 3)));
        }
    }
}

// 16 source bytes at src + so for the COMPACT gather: two aligned 16-byte loads + alignbyte when
// all 32 bytes lie inside the wire (the common case, no branches), else the guarded byte path.
__device__ __forceinline__ uint4 gather16(const uint8_t* __restrict__ src, int64_t so, uint64_t n) {
    const int64_t c0 = so & ~(int64_t)15;
    if (c0 < 0 || (uint64_t)c0 + 32 > n) return load16_unaligned(src, so, n);
    const uint4 v0 = *reinterpret_cast<const uint4*>(src + c0);
    const uint4 v1 = *reinterpret_cast<const uint4*>(src + c0 + 16);
    const uint32_t sh = (uint32_t)(so - c0), q = sh >> 2, rb = sh & 3;
    const uint32_t d[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t lo = d[j], hi = d[j + 1];
        if (q == 1) { lo = d[j + 1]; hi = d[j + 2]; }
        else if (q == 2) { lo = d[j + 2]; hi = d[j + 3]; }
        else if (q == 3) { lo = d[j + 3]; hi = d[j + 4]; }
        o[j] = __builtin_amdgcn_alignbyte(hi, lo, rb);
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

__device__ __forceinline__ u32x4 range_mask16(int32_t lo, int32_t hi) {
    // byte mask of [lo, hi) within a 16-byte piece (lo, hi already clipped to [0, 16])
    u32x4 m;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int32_t l = lo - 4 * j, h = hi - 4 * j;
        const uint32_t ll = l < 0 ? 0u : (uint32_t)l, hh = h < 0 ? 0u : (uint32_t)h;
        m[j] = ll < hh ? bytes_to_mask(ll, hh > 4 ? 4 : hh) : 0u;
    }
    return m;
}

// lane 0's value, as a wave-uniform (scalar) value
__device__ __forceinline__ uint64_t lane0_u64(uint64_t x) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, 0), hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), 0);
    return (uint64_t)hi << 32 | lo;
}
__device__ __forceinline__ uint32_t lane0_u32(uint32_t x) { return __builtin_amdgcn_readlane(x, 0); }

// The span lane r0 + lane of a window, as loaded (valid = the span exists).
__device__ __forceinline__ bool load_span_lane(const Span* __restrict__ spans, uint32_t n_spans, uint32_t r0,
                                               uint32_t lane, Span& sp) {
    const uint32_t si = r0 + lane;
    if (si < n_spans) {
        sp = spans[si];
        return true;
    }
    sp = Span{0, ~0ull, 0, 0};
    return false;
}

// General window, lane-parallel: the wave loads the window's spans into lanes with one vector
// load (span r0 + lane), then every lane finds the span holding its piece by a 6-step binary
// search over the lanes (ds_bpermute) and takes that span and the next one -- at most 2 spans per
// 16-byte piece unless spans are shorter than 16 B, which a uniform tail loop handles.  No
// dependent scalar loads per span; in COMPACT mode all of a lane's gathers are issued together.
// Returns false (nothing written) when more than 64 spans overlap the window.
template <bool COMPACT, int P, int NT>
__device__ __forceinline__ bool unmask_window_lanes(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                    uint64_t src_bytes, const Span& sp, bool valid,
                                                    uint32_t n_spans, uint32_t r0, uint64_t wbase, uint32_t lane,
                                                    u32x4 (&v)[P]) {
    constexpr int32_t WB = 1024 * P;
    int32_t rd = WB + 64, re = WB + 64;   // window-relative [start, end), clipped to [-1, WB + 64]
    uint32_t key = 0;
    int64_t sd = 0;                       // COMPACT: src - dst
    if (valid) {
        const int64_t d0 = (int64_t)sp.dst - (int64_t)wbase, d1 = d0 + (int64_t)sp.len;
        rd = (int32_t)(d0 < -1 ? -1 : (d0 > WB + 64 ? WB + 64 : d0));
        re = (int32_t)(d1 < -1 ? -1 : (d1 > WB + 64 ? WB + 64 : d1));
        key = sp.key;
        if constexpr (COMPACT) sd = (int64_t)sp.src - (int64_t)sp.dst;
    }
    const uint64_t inwin = __ballot(rd < WB);
    const uint32_t nl = (uint32_t)__builtin_popcountll(inwin);   // spans overlapping the window: lanes 0..nl-1
    if (nl == 64 && __shfl(re, 63) < WB && r0 + 64 < n_spans) return false;
    const uint32_t sd_lo = (uint32_t)sd, sd_hi = (uint32_t)((uint64_t)sd >> 32);

    u32x4 acc[P];
    int32_t ta[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int32_t pr = k * 1024 + (int32_t)lane * 16;
        // largest t < nl with rd[t] <= pr (-1 if none)
        int32_t lo = -1;
#pragma unroll
        for (int st = 32; st >= 1; st >>= 1) {
            const int32_t c = lo + st;
            const int32_t dv = __shfl(rd, c & 63);
            if (c < (int32_t)nl && dv <= pr) lo = c;
        }
        ta[k] = lo < 0 ? 0 : lo;
    }
    // spans A = ta and B = ta + 1 of every piece: parameters first, then all gathers together
    int32_t alo[P], ahi[P], blo[P], bhi[P];
    uint32_t ka[P], kb[P];
    int64_t soa[P], sob[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int32_t pr = k * 1024 + (int32_t)lane * 16;
        const int32_t a = ta[k], b = ta[k] + 1;
        const int32_t da = __shfl(rd, a & 63), ea = __shfl(re, a & 63);
        const int32_t db = __shfl(rd, b & 63), eb = __shfl(re, b & 63);
        ka[k] = __shfl(key, a & 63);
        kb[k] = __shfl(key, b & 63);
        alo[k] = (da > pr ? da : pr) - pr;
        ahi[k] = (ea < pr + 16 ? ea : pr + 16) - pr;
        if (a >= (int32_t)nl) ahi[k] = -1;
        blo[k] = (db > pr ? db : pr) - pr;
        bhi[k] = (eb < pr + 16 ? eb : pr + 16) - pr;
        if (b >= (int32_t)nl) bhi[k] = -1;
        if constexpr (COMPACT) {
            const uint32_t al = __shfl(sd_lo, a & 63), ah = __shfl(sd_hi, a & 63);
            const uint32_t bl = __shfl(sd_lo, b & 63), bh = __shfl(sd_hi, b & 63);
            const int64_t pa = (int64_t)wbase + pr;
            soa[k] = (int64_t)((uint64_t)ah << 32 | al) + pa;
            sob[k] = (int64_t)((uint64_t)bh << 32 | bl) + pa;
        }
    }
    uint4 ga[P], gb[P];
    if constexpr (COMPACT) {
#pragma unroll
        for (int k = 0; k < P; ++k) {
            ga[k] = alo[k] < ahi[k] ? gather16(src, soa[k], src_bytes) : make_uint4(0, 0, 0, 0);
            gb[k] = blo[k] < bhi[k] ? gather16(src, sob[k], src_bytes) : make_uint4(0, 0, 0, 0);
        }
    }
    bool more = false;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const u32x4 ma = alo[k] < ahi[k] ? range_mask16(alo[k], ahi[k]) : u32x4{0, 0, 0, 0};
        const u32x4 mb = blo[k] < bhi[k] ? range_mask16(blo[k], bhi[k]) : u32x4{0, 0, 0, 0};
        const u32x4 key16 = (ka[k] & ma) | (kb[k] & mb);
        if constexpr (COMPACT) {
            const u32x4 sa = u32x4{ga[k].x, ga[k].y, ga[k].z, ga[k].w} & ma;
            const u32x4 sb = u32x4{gb[k].x, gb[k].y, gb[k].z, gb[k].w} & mb;
            acc[k] = (sa | sb) ^ key16;
        } else {
            acc[k] = v[k] ^ key16;
        }
        // span B ends inside the piece and another span follows it there (spans < 16 B)
        more |= bhi[k] == 16 ? false : (bhi[k] >= 0 && ta[k] + 2 < (int32_t)nl);
    }
    if (__ballot(more)) {
        // rare: pieces overlapping 3+ spans; uniform loop over the extra spans t = ta + 2, ...
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const int32_t pr = k * 1024 + (int32_t)lane * 16;
            int32_t t = ta[k] + 2;
            bool act = true;
            while (__ballot(act && t < (int32_t)nl)) {
                const int32_t dt = __shfl(rd, t & 63), et = __shfl(re, t & 63);
                const uint32_t kt = __shfl(key, t & 63);
                const uint32_t tl = __shfl(sd_lo, t & 63), th = __shfl(sd_hi, t & 63);
                act = act && t < (int32_t)nl && dt < pr + 16;
                if (act) {
                    const int32_t l = (dt > pr ? dt : pr) - pr, h = (et < pr + 16 ? et : pr + 16) - pr;
                    if (l < h) {
                        const u32x4 m = range_mask16(l, h);
                        if constexpr (COMPACT) {
                            const int64_t so = (int64_t)((uint64_t)th << 32 | tl) + (int64_t)wbase + pr;
                            const uint4 g = gather16(src, so, src_bytes);
                            acc[k] ^= (u32x4{g.x, g.y, g.z, g.w} & m) ^ (kt & m);
                        } else {
                            acc[k] ^= kt & m;
                        }
                    }
                }
                ++t;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < P; ++k) st16v<NT>(dst + wbase + k * 1024u + lane * 16u, acc[k]);
    return true;
}

// NT bit 0: non-temporal loads, bit 1: non-temporal stores.  In place, `src` is unused (dst is
// both source and destination) so the two restrict pointers never alias in an access.
template <bool COMPACT, int P, int NT, int MINW = 1>
__global__ __launch_bounds__(256, MINW) void k_unmask(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                uint64_t src_bytes, uint64_t dst_bytes_host,
                                                const Span* __restrict__ spans,
                                                const uint32_t* __restrict__ tile_first,
                                                const wsc_summary* __restrict__ summary,
                                                uint32_t* __restrict__ lb_state, uint32_t n_walk_blocks) {
    constexpr uint32_t WB = 1024u * P;
    // re-arm the walk's look-back state for the next decode (this launch is ordered after it):
    // lb_state[0] = ticket, [1] = timeout flag, [2 ...] = per-block flags
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n_walk_blocks + 2; t += gridDim.x * blockDim.x)
        lb_state[t] = 0;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t waves_per_block = blockDim.x >> 6;
    const uint32_t gw = __builtin_amdgcn_readfirstlane(blockIdx.x * waves_per_block + (threadIdx.x >> 6));
    const uint32_t nw = gridDim.x * waves_per_block;
    const uint64_t total = COMPACT ? summary->data_bytes + summary->ctrl_bytes : dst_bytes_host;
    const uint32_t n_spans = summary->n_spans;
    const uint64_t n_win = (total + WB - 1) / WB;
    const uint32_t lofs = lane * 16u;
    if (n_spans == 0) return;

    if constexpr (COMPACT) {
        // Arena windows: the source bytes depend on the span lookup (tile -> spans -> gathers), so
        // the lookup of window i + nw is prefetched while window i is gathered and stored: spans
        // one window ahead (vector), the tile index two ahead (scalar).  Grid-stride over windows.
        uint64_t win = gw;
        if (win >= n_win) return;
        uint32_t r = tile_first[win];
        Span sp;
        bool sv = load_span_lane(spans, n_spans, r, lane, sp);
        uint32_t r_next = win + nw < n_win ? tile_first[win + nw] : 0u;
        while (true) {
            const uint64_t wbase = win * WB;
            const uint64_t nx = win + nw;
            const Span cur = sp;
            const bool cv = sv;
            const uint32_t rc = r;
            if (nx < n_win) {   // prefetch
                r = r_next;
                sv = load_span_lane(spans, n_spans, r, lane, sp);
                r_next = nx + nw < n_win ? tile_first[nx + nw] : 0u;
            }
            const uint64_t s_dst = lane0_u64(cur.dst), s_end = s_dst + lane0_u32(cur.len);
            if (wbase + WB > total) {
                unmask_window_general<COMPACT, P, NT>(dst, src, src_bytes, total, spans, n_spans, rc, wbase, lofs);
            } else if (lane0_u32(cv) && s_dst <= wbase && s_end >= wbase + WB) {
                // one span covers the whole window -> gather with one shift, one rotated key
                const int64_t so = (int64_t)lane0_u64(cur.src) - (int64_t)s_dst;
                const uint32_t key = lane0_u32(cur.key);
                uint4 t[P];
#pragma unroll
                for (int k = 0; k < P; ++k) t[k] = gather16(src, so + (int64_t)(wbase + k * 1024u + lofs), src_bytes);
#pragma unroll
                for (int k = 0; k < P; ++k) st16v<NT>(dst + wbase + k * 1024u + lofs, u32x4{t[k].x, t[k].y, t[k].z, t[k].w} ^ key);
            } else {
                u32x4 vv[P];
                if (!unmask_window_lanes<COMPACT, P, NT>(dst, src, src_bytes, cur, cv, n_spans, rc, wbase, lane, vv))
                    unmask_window_general<COMPACT, P, NT>(dst, src, src_bytes, total, spans, n_spans, rc, wbase, lofs);
            }
            if (nx >= n_win) break;
            win = nx;
        }
        return;
    }

    for (uint64_t win = gw; win < n_win; win += nw) {
        const uint64_t wbase = win * WB;
        if (wbase + WB > total) {   // the last, partial window
            const uint32_t r = tile_first[win];
            unmask_window_general<COMPACT, P, NT>(dst, src, src_bytes, total, spans, n_spans, r, wbase, lofs);
            continue;
        }
        u32x4 v[P];
        // in place the loads do not depend on the span lookup: issue them first
#pragma unroll
        for (int k = 0; k < P; ++k) v[k] = ld16v<NT>(dst + wbase + k * 1024u + lofs);
        // the fast-path test uses scalar loads (lgkmcnt), so it never waits behind the data loads
        const uint32_t r = tile_first[win];
        Span s0 = spans[r < n_spans ? r : n_spans - 1];
        if (r >= n_spans) s0.dst = ~0ull;   // no span starts before the window's end
        if (s0.dst <= wbase && s0.dst + s0.len >= wbase + WB) {
            // fast path: one span covers the whole window -> one rotated key for every dword
#pragma unroll
            for (int k = 0; k < P; ++k) st16v<NT>(dst + wbase + k * 1024u + lofs, v[k] ^ s0.key);
            continue;
        }
        // Several spans overlap the window (small frames) or it holds a frame edge: lane-parallel
        // span lookup; more than 64 spans in one window falls back to the serial span walk.
        Span sp;
        const bool valid = load_span_lane(spans, n_spans, r, lane, sp);
        if (!unmask_window_lanes<COMPACT, P, NT>(dst, src, src_bytes, sp, valid, n_spans, r, wbase, lane, v))
            unmask_window_general<COMPACT, P, NT>(dst, src, src_bytes, total, spans, n_spans, r, wbase, lofs);
    }
}

}  // namespace wsc
