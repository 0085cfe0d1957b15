// wsc_unmask.inl -- the unmask kernel template (the hot loop, websocket_frame.go:35-39), shared by
// the two translation units that instantiate it (wsc_unmask_inplace.hip, wsc_unmask_compact.hip)
// so that hipcc compiles the variants in parallel.
#pragma once
#include <type_traits>
#include "wsc_kernels.hpp"
#include "wsc_dev.hpp"
#include "wsc_u8.hpp"

namespace wsc {

// ---------------------------------------------------------------------------------------------
// Unmask: the hot loop.  The wire is cut into windows of P KiB; wave w owns window w (grid-
// stride).  tile_first[w] names the first span (stream order) whose wire end lies after the
// window start, so the wave looks only at the spans that overlap its window.  Each lane holds P
// pieces of 16 B at wire + w*W + k*1024 + lane*16: every wave instruction touches 1 KiB
// contiguous, and the loads never depend on the span lookup.  A span's key is phased at the wire,
// so every aligned wire dword XORs with one register.  In place the pieces are stored back where
// they came from; COMPACT stores each span's bytes at its arena offset (dst = wire + span.dst -
// span.src): a piece inside one span is one byte-aligned 16-byte store, a piece holding a frame
// edge stores each span's run with at most four stores and skips the header bytes between them.
// ---------------------------------------------------------------------------------------------

// General window: several spans overlap it (small frames), or it is the last, partial window.
// Builds a per-byte key from every span that overlaps each 16-byte piece.
template <bool COMPACT, int P, int NT>
// Inlined (WSC_GENERAL_INLINE=1, the default): as an out-of-line call the general window cost the
// kernel its live registers across the call (in place 116 VGPRs, 4 waves per SIMD; 52 B of spills
// when built for 5).  Inlined, in place needs 84 VGPRs (96 with the UTF-8 fold), COMPACT 72 (80),
// and every P = 4 unmask runs at 5 waves per SIMD without spills: headline 3,064 -> 3,157 GiB/s,
// configs[1] 0.400 -> 0.382 ms, configs[3] 1.357 -> 1.305 ms, 64 KiB TEXT 0.415 -> 0.393 ms
// (profiles/r04_unmask_inline_ab.log).
#ifndef WSC_GENERAL_INLINE
#define WSC_GENERAL_INLINE 1
#endif
#if WSC_GENERAL_INLINE
__device__ __forceinline__
#else
__device__ __attribute__((noinline))
#endif
void unmask_window_general(
    uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t src_bytes, uint64_t total,
    const Span* __restrict__ spans, uint32_t n_spans, uint32_t r, uint64_t wbase, uint32_t lofs) {
    constexpr uint32_t WB = 1024u * P;
    if constexpr (COMPACT) {
        // serial fallback (last window of the wire, > 64 spans in a window): wire pieces (bytes
        // past the wire read as 0, never stored), every overlapping span's run stored at its dst
        u32x4 w[P];
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const uint4 t = load16_unaligned(src, (int64_t)(wbase + k * 1024u + lofs), src_bytes);
            w[k] = u32x4{t.x, t.y, t.z, t.w};
        }
        for (; r < n_spans; ++r) {
            const Span sp = spans[r];
            if (sp.src >= wbase + WB) break;
            const uint64_t s0 = sp.src, s1 = sp.src + sp.len;
#pragma unroll
            for (int k = 0; k < P; ++k) {
                const uint64_t pa = wbase + k * 1024u + lofs;
                const uint64_t lo = s0 > pa ? s0 : pa;
                const uint64_t hi = s1 < pa + 16 ? s1 : pa + 16;
                if (lo < hi) store_run<NT>(dst + sp.dst + (lo - s0), w[k] ^ sp.key, (uint32_t)(lo - pa), (uint32_t)(hi - pa));
            }
        }
        return;
    }
    uint4 v[P], key[P];
    uint32_t cov[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        key[k] = make_uint4(0, 0, 0, 0);
        cov[k] = 0;
        v[k] = make_uint4(0, 0, 0, 0);
        const uint64_t addr = wbase + k * 1024u + lofs;
        if (addr + 16 <= total) v[k] = ld16<NT>(dst + addr);
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
            }
        }
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        if (!cov[k]) continue;
        const uint64_t addr = wbase + k * 1024u + lofs;
        uint4 o = v[k];
        o.x ^= key[k].x; o.y ^= key[k].y; o.z ^= key[k].z; o.w ^= key[k].w;
        if (addr + 16 <= total) {
            st16<NT>(dst + addr, o);
        } else {
            // in-place tail piece past the last full 16 B of the buffer: byte stores
            const uint32_t kd[4] = {key[k].x, key[k].y, key[k].z, key[k].w};
            for (uint32_t j = 0; addr + j < total; ++j)
                dst[addr + j] ^= (uint8_t)(kd[j >> 2] >> (8 * (j & 3)));
        }
    }
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

// Byte masks from a 17-entry LDS table: pm[L] = the first L bytes of a 16-byte piece, so the
// bytes [lo, hi) are pm[hi] & ~pm[lo] (one v_bfi per dword; empty when hi <= lo).  Replaces the
// per-dword shift / compare chains of range_mask16 in the window paths that run per piece:
// the lane-parallel window of small frames was VALU-bound (PMC: 725 VALU instructions per wave
// window at 1 KiB frames, ~77 % of the chip's VALU cycles during the kernel).
__device__ __forceinline__ u32x4 prefix_mask16(uint32_t L) {
    u32x4 m;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t n = L > 4u * j ? (L - 4u * j > 4u ? 4u : L - 4u * j) : 0u;
        m[j] = n == 4 ? 0xFFFFFFFFu : ((1u << (8 * n)) - 1u);
    }
    return m;
}
__device__ __forceinline__ int32_t clamp16(int32_t x) { return x < 0 ? 0 : (x > 16 ? 16 : x); }
__device__ __forceinline__ u32x4 pm_range(const u32x4* __restrict__ pm, int32_t lo, int32_t hi) {
    const u32x4 h = pm[clamp16(hi)], l = pm[clamp16(lo)];
    return h & ~l;
}

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
// load (span r0 + lane), then every lane finds the span holding its piece by a binary search over
// the lanes (ds_bpermute; as many steps as the window has spans need) and takes that span and the
// next one -- at most 2 spans per 16-byte piece unless spans are shorter than 16 B, which a
// uniform tail loop handles.  No dependent scalar loads per span.  v[] holds the window's wire
// pieces.  Returns false (nothing written) when more than 64 spans overlap the window.
template <bool COMPACT, int P, int NT>
__device__ __forceinline__ bool unmask_window_lanes(uint8_t* __restrict__ dst, const Span& sp, bool valid,
                                                    uint32_t n_spans, uint32_t r0, uint64_t wbase, uint32_t lane,
                                                    const u32x4 (&v)[P], const u32x4* __restrict__ pm) {
    constexpr int32_t WB = 1024 * P;
    int32_t rd = WB + 64, re = WB + 64;   // window-relative wire [start, end), clipped to [-1, WB + 64]
    uint32_t key = 0;
    int64_t sd = 0;                       // COMPACT: dst - src
    if (valid) {
        const int64_t d0 = (int64_t)sp.src - (int64_t)wbase, d1 = d0 + (int64_t)sp.len;
        rd = (int32_t)(d0 < -1 ? -1 : (d0 > WB + 64 ? WB + 64 : d0));
        re = (int32_t)(d1 < -1 ? -1 : (d1 > WB + 64 ? WB + 64 : d1));
        key = sp.key;
        if constexpr (COMPACT) sd = (int64_t)sp.dst - (int64_t)sp.src;
    }
    const uint64_t inwin = __ballot(rd < WB);
    const uint32_t nl = (uint32_t)__builtin_popcountll(inwin);   // spans overlapping the window: lanes 0..nl-1
    if (nl == 64 && __shfl(re, 63) < WB && r0 + 64 < n_spans) return false;
    const uint32_t sd_lo = (uint32_t)sd, sd_hi = (uint32_t)((uint64_t)sd >> 32);
    // binary search: first step = the power of two with 2*st0 > nl (wave-uniform), at most 32 (a
    // piece past span 62 still finds span 63 as its span B)
    const int32_t st0 = nl == 0 ? 0 : (nl >= 32 ? 32 : (int32_t)((1u << (32 - __builtin_clz(nl))) >> 1));

    int32_t ta[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int32_t pr = k * 1024 + (int32_t)lane * 16;
        // largest t < nl with rd[t] <= pr (-1 if none)
        int32_t lo = -1;
        for (int32_t st = st0; st >= 1; st >>= 1) {
            const int32_t c = lo + st;
            const int32_t dv = __shfl(rd, c & 63);
            if (c < (int32_t)nl && dv <= pr) lo = c;
        }
        ta[k] = lo < 0 ? 0 : lo;
    }
    // spans A = ta and B = ta + 1 of every piece
    int32_t alo[P], ahi[P], blo[P], bhi[P];
    uint32_t ka[P], kb[P];
    int64_t da[P], db[P];   // COMPACT: arena address of the piece's byte 0 under span A / B
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int32_t pr = k * 1024 + (int32_t)lane * 16;
        const int32_t a = ta[k], b = ta[k] + 1;
        const int32_t dA = __shfl(rd, a & 63), eA = __shfl(re, a & 63);
        const int32_t dB = __shfl(rd, b & 63), eB = __shfl(re, b & 63);
        ka[k] = __shfl(key, a & 63);
        kb[k] = __shfl(key, b & 63);
        alo[k] = (dA > pr ? dA : pr) - pr;
        ahi[k] = (eA < pr + 16 ? eA : pr + 16) - pr;
        if (a >= (int32_t)nl) ahi[k] = -1;
        blo[k] = (dB > pr ? dB : pr) - pr;
        bhi[k] = (eB < pr + 16 ? eB : pr + 16) - pr;
        if (b >= (int32_t)nl) bhi[k] = -1;
        if constexpr (COMPACT) {
            const uint32_t al = __shfl(sd_lo, a & 63), ah = __shfl(sd_hi, a & 63);
            const uint32_t bl = __shfl(sd_lo, b & 63), bh = __shfl(sd_hi, b & 63);
            const int64_t pa = (int64_t)wbase + pr;
            da[k] = (int64_t)((uint64_t)ah << 32 | al) + pa;
            db[k] = (int64_t)((uint64_t)bh << 32 | bl) + pa;
        }
    }
    bool more = false;
    if constexpr (COMPACT) {
        // pieces inside one span: one 16-byte store each, issued first
        bool part = false;
#pragma unroll
        for (int k = 0; k < P; ++k) {
            if (alo[k] == 0 && ahi[k] == 16) st16u<NT>(dst + da[k], v[k] ^ ka[k]);
            else part |= alo[k] < ahi[k] || blo[k] < bhi[k];
            more |= bhi[k] == 16 ? false : (bhi[k] >= 0 && ta[k] + 2 < (int32_t)nl);
        }
        if (__ballot(part)) {
            // frame edges: each span's run of the piece at its own arena offset
#pragma unroll
            for (int k = 0; k < P; ++k) {
                if (alo[k] == 0 && ahi[k] == 16) continue;
                if (alo[k] < ahi[k]) store_run<NT>(dst + da[k] + alo[k], v[k] ^ ka[k], alo[k], ahi[k]);
                if (blo[k] < bhi[k]) store_run<NT>(dst + db[k] + blo[k], v[k] ^ kb[k], blo[k], bhi[k]);
            }
        }
    } else {
        u32x4 acc[P];
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const u32x4 ma = pm_range(pm, alo[k], ahi[k]);
            const u32x4 mb = pm_range(pm, blo[k], bhi[k]);
            acc[k] = v[k] ^ ((ka[k] & ma) | (kb[k] & mb));
            // span B ends inside the piece and another span follows it there (spans < 16 B)
            more |= bhi[k] == 16 ? false : (bhi[k] >= 0 && ta[k] + 2 < (int32_t)nl);
        }
        if (__ballot(more)) {
#pragma unroll
            for (int k = 0; k < P; ++k) {
                const int32_t pr = k * 1024 + (int32_t)lane * 16;
                int32_t t = ta[k] + 2;
                bool act = true;
                while (__ballot(act && t < (int32_t)nl)) {
                    const int32_t dt = __shfl(rd, t & 63), et = __shfl(re, t & 63);
                    const uint32_t kt = __shfl(key, t & 63);
                    act = act && t < (int32_t)nl && dt < pr + 16;
                    if (act) {
                        const int32_t l = (dt > pr ? dt : pr) - pr, h = (et < pr + 16 ? et : pr + 16) - pr;
                        acc[k] ^= kt & pm_range(pm, l, h);
                    }
                    ++t;
                }
            }
        }
        if constexpr (NT >= 16) {
            const __amdgpu_buffer_rsrc_t rs = win_rsrc(dst + wbase, 1024u * P);
#pragma unroll
            for (int k = 0; k < P; ++k) st16b<(NT >> 4)>(rs, k * 1024u + lane * 16u, acc[k]);
        } else {
#pragma unroll
            for (int k = 0; k < P; ++k) st16v<NT>(dst + wbase + k * 1024u + lane * 16u, acc[k]);
        }
        return true;
    }
    if (__ballot(more)) {
        // COMPACT, rare: pieces overlapping 3+ spans; uniform loop over the extra spans t = ta + 2, ...
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
                        const int64_t d = (int64_t)((uint64_t)th << 32 | tl) + (int64_t)wbase + pr;
                        store_run<NT>(dst + d + l, v[k] ^ kt, (uint32_t)l, (uint32_t)h);
                    }
                }
                ++t;
            }
        }
    }
    return true;
}

#ifndef WSC_COMPACT_EDGE2   // (-DWSC_COMPACT_EDGE2=0: the one-pass unmask_window_lanes<true>, for A/B)
#define WSC_COMPACT_EDGE2 1
#endif
// COMPACT, lane-parallel, in two passes (the encoder's edge pass, wsc_encode.hip): (1) every piece
// lying inside one span is one byte-aligned 16-byte store at its arena offset, and the pieces that
// meet a span edge are listed -- id and wire bytes -- in the wave's LDS stage; (2) one lane per
// listed piece stores the run of each span it meets.  The per-span run stores (store_run: a byte
// shift and up to four partial stores) then run once per wave for all of a window's edge pieces
// instead of once per 1 KiB slice for every lane, and the kernel needs 88 VGPRs instead of 110 (5
// waves per SIMD instead of 4).  Measured (profiles/r04_compact_edge2_ab.log, same box): configs[4]
// unmask 0.895 -> 0.859 ms (5.44 -> 5.63 TB/s), decode 0.956 -> 0.919 ms, pipelined 1.018 ->
// 0.916 ms per batch.  stage: 288 uint4 per wave (256 pieces' bytes, then 256 u16 ids).  Same
// results as unmask_window_lanes<true>.
template <int P, int NT>
__device__ __forceinline__ bool unmask_window_lanes_c(uint8_t* __restrict__ dst, const Span& sp, bool valid,
                                                      uint32_t n_spans, uint32_t r0, uint64_t wbase, uint32_t lane,
                                                      const u32x4 (&v)[P], uint4* __restrict__ stage) {
    constexpr int32_t WB = 1024 * P;
    static_assert(P * 64 <= 256, "stage holds 256 pieces");
    int32_t rd = WB + 64, re = WB + 64;   // window-relative wire [start, end), clipped to [-1, WB + 64]
    uint32_t key = 0;
    int64_t sd = 0;                       // dst - src
    if (valid) {
        const int64_t d0 = (int64_t)sp.src - (int64_t)wbase, d1 = d0 + (int64_t)sp.len;
        rd = (int32_t)(d0 < -1 ? -1 : (d0 > WB + 64 ? WB + 64 : d0));
        re = (int32_t)(d1 < -1 ? -1 : (d1 > WB + 64 ? WB + 64 : d1));
        key = sp.key;
        sd = (int64_t)sp.dst - (int64_t)sp.src;
    }
    const uint64_t inwin = __ballot(rd < WB);
    const uint32_t nl = (uint32_t)__builtin_popcountll(inwin);
    if (nl == 64 && __shfl(re, 63) < WB && r0 + 64 < n_spans) return false;
    const uint32_t sd_lo = (uint32_t)sd, sd_hi = (uint32_t)((uint64_t)sd >> 32);
    const int32_t st0 = nl == 0 ? 0 : (nl >= 32 ? 32 : (int32_t)((1u << (32 - __builtin_clz(nl))) >> 1));
    auto find = [&](int32_t pr) -> int32_t {   // largest t < nl with rd[t] <= pr (0 if none)
        int32_t lo = -1;
        for (int32_t st = st0; st >= 1; st >>= 1) {
            const int32_t c = lo + st;
            const int32_t dv = __shfl(rd, c & 63);
            if (c < (int32_t)nl && dv <= pr) lo = c;
        }
        return lo < 0 ? 0 : lo;
    };
    uint16_t* const ids = reinterpret_cast<uint16_t*>(stage + 256);
    // ---- pass 1: pieces inside one span ----
    uint32_t n_edge = 0;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int32_t pr = k * 1024 + (int32_t)lane * 16;
        const int32_t a = find(pr);
        const int32_t dA = __shfl(rd, a & 63), eA = __shfl(re, a & 63), dB = __shfl(rd, (a + 1) & 63);
        const uint32_t ka = __shfl(key, a & 63), al = __shfl(sd_lo, a & 63), ah = __shfl(sd_hi, a & 63);
        const bool inside = a < (int32_t)nl && dA <= pr && pr + 16 <= eA;
        if (inside) st16u<NT>(dst + ((int64_t)((uint64_t)ah << 32 | al) + (int64_t)wbase + pr), v[k] ^ ka);
        const bool meets = (a < (int32_t)nl && dA < pr + 16 && eA > pr) || (a + 1 < (int32_t)nl && dB < pr + 16);
        const bool edge = !inside && meets;
        const uint64_t em = __ballot(edge);
        if (edge) {
            const uint32_t slot = n_edge + __builtin_amdgcn_mbcnt_hi((uint32_t)(em >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)em, 0u));
            ids[slot] = (uint16_t)(k * 64 + lane);
            stage[slot] = make_uint4(v[k][0], v[k][1], v[k][2], v[k][3]);
        }
        n_edge += (uint32_t)__builtin_popcountll(em);
    }
    if (n_edge == 0) return true;
    __builtin_amdgcn_wave_barrier();
    // ---- pass 2: one edge piece per lane, each span it meets ----
    for (uint32_t base = 0; base < n_edge; base += 64) {
        const bool act = base + lane < n_edge;
        const uint32_t pid = act ? ids[base + lane] : 0u;
        const int32_t pr = (int32_t)((pid >> 6) * 1024 + (pid & 63) * 16);
        const uint4 xs = act ? stage[base + lane] : make_uint4(0, 0, 0, 0);
        const u32x4 x = {xs.x, xs.y, xs.z, xs.w};
        int32_t t = find(pr);
        bool go = act;
        while (__ballot(go)) {
            const int32_t dt = __shfl(rd, t & 63), et = __shfl(re, t & 63);
            const uint32_t kt = __shfl(key, t & 63), tl = __shfl(sd_lo, t & 63), th = __shfl(sd_hi, t & 63);
            go = go && t < (int32_t)nl && dt < pr + 16;
            if (go) {
                const int32_t l = (dt > pr ? dt : pr) - pr, h = (et < pr + 16 ? et : pr + 16) - pr;
                if (l < h)
                    store_run<NT>(dst + ((int64_t)((uint64_t)th << 32 | tl) + (int64_t)wbase + pr + l), x ^ kt,
                                  (uint32_t)l, (uint32_t)h);
            }
            ++t;
        }
    }
    __builtin_amdgcn_wave_barrier();   // (the stage is reused by the wave's next window)
    return true;
}

// Deferred text (k_u8_check runs after this kernel): a window the walk flagged lies inside one
// UTF-8 item, so the wave that has just unmasked it folds its DFA map from the registers (text is
// read from HBM once) and publishes it in win_map; the check reads only the items' partial windows.
// The workgroup's LDS tables are built by the first wave that meets a text window (binary windows
// never touch them); the others wait on the LDS state word.
struct U8Block {
    U8Lds t;
    uint4 stage[4][U8_STAGE];
    uint32_t state;   // 0 none, 1 building, 2 ready
};
// (namespace scope: allocated only in the kernels that reach it, the U8 instantiations)
__shared__ U8Block g_u8b;
// COMPACT edge stage of the binary variants (unmask_window_lanes_c; U8 variants use g_u8b.stage)
__shared__ uint4 c_stage[4][288];

#ifndef WSC_FOLD_NCH   // independent DFA chains per 64-byte lane chunk in the fold (A/B: tools/build_variant.sh)
#define WSC_FOLD_NCH 4
#endif
// The fold of a window whose first 4 KiB the caller has written to the wave's stage: tables (built
// once per workgroup), then the map of every 4 KiB group.  COMPACT calls it out of line: its window
// loop keeps more registers live, and the fold inlined there pushed it past 128 VGPRs (spill)
template <int P>
__device__ __forceinline__ void fold_staged(const u32x4* v, uint32_t key, U8Win u8w, uint64_t win, uint32_t lane);
static inline __device__ __attribute__((noinline)) void fold_staged4(U8Win u8w, uint64_t win, uint32_t lane);
template <bool OUTLINE, int P>
__device__ __forceinline__ void fold_text_window(const u32x4 (&v)[P], uint32_t key, U8Win u8w, uint64_t win,
                                                 uint32_t lane) {
    uint4* sw = g_u8b.stage[(threadIdx.x >> 6) & 3];
    // the first 4 KiB goes to the wave's stage before anything else: the unmasked registers are
    // dead from here on (the table build would otherwise hold them)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t o = 1024u * k + 16u * lane;
        const u32x4 x = v[k] ^ key;
        sw[(o >> 6) * 5 + ((o >> 4) & 3)] = make_uint4(x[0], x[1], x[2], x[3]);
    }
    if constexpr (OUTLINE && P == 4) {
        fold_staged4(u8w, win, lane);
    } else {
        fold_staged<P>(v, key, u8w, win, lane);
    }
}
template <int P>
__device__ __forceinline__ void fold_staged(const u32x4* v, uint32_t key, U8Win u8w, uint64_t win, uint32_t lane) {
    U8Block& b = g_u8b;
    uint4* sw = b.stage[(threadIdx.x >> 6) & 3];
    auto stage_write = [&](int g) {   // groups after the first (P = 8)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t o = 1024u * k + 16u * lane;
            const u32x4 x = v[4 * g + k] ^ key;
            sw[(o >> 6) * 5 + ((o >> 4) & 3)] = make_uint4(x[0], x[1], x[2], x[3]);
        }
    };
    uint32_t prev = 0;
    if (lane == 0) prev = __hip_atomic_compare_exchange_strong(&b.state, &prev, 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_WORKGROUP) ? 0u : prev;
    prev = (uint32_t)__builtin_amdgcn_readfirstlane((int)prev);
    if (prev == 0) {
#pragma unroll 1
        for (uint32_t byte = lane; byte < 256; byte += 64) u8_tables_init(b.t, byte);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&b.state, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
        while (__hip_atomic_load(&b.state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 2u) __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    uint64_t m = u8m_id();
#pragma unroll
    for (int g = 0; g < P / 4; ++g) {
        if (g) stage_write(g);
        __builtin_amdgcn_wave_barrier();
        u32x4 q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 t = sw[lane * 5 + k];
            q[k] = u32x4{t.x, t.y, t.z, t.w};
        }
        __builtin_amdgcn_wave_barrier();
        bool plain;
        const uint64_t pm = u8_chunk_map<WSC_FOLD_NCH, U8P_NONE>(b.t, q, 0u, 64u, plain);
        m = u8m_then(m, u8_wave_map(pm, plain, lane));
    }
    if (lane == 0) {
        u8w.map[win] = m;
        u8w.flag[win] = 0u;   // consumed (flags are only ever set by the walk)
    }
}

static inline __device__ __attribute__((noinline)) void fold_staged4(U8Win u8w, uint64_t win, uint32_t lane) {
    fold_staged<4>(nullptr, 0u, u8w, win, lane);
}

// A COMPACT window inside one span: its 4 KiB go to the arena at d0 (= arena offset of window byte
// 0), which is 16-byte aligned only when the span's arena and wire offsets agree mod 16.  With
// WSC_COMPACT_ALIGNED the wave stores aligned 16-byte chunks instead of byte-aligned ones: lane l's
// chunk of slice k holds the last m bytes of the previous piece (lane l - 1, or lane 63 of slice
// k - 1: a lane shuffle) and the first 16 - m of its own (m = d0 & 15); the window's first
// 16 - m bytes and its last m bytes are byte runs (store_run).  Every arena byte is written once.
#ifndef WSC_COMPACT_ALIGNED
#define WSC_COMPACT_ALIGNED 0
#endif
template <int NT>
__device__ __forceinline__ void compact_window_aligned(uint8_t* d0, const u32x4 (&v)[4], uint32_t key, uint32_t lane) {
    const uint32_t m = (uint32_t)(reinterpret_cast<uintptr_t>(d0) & 15);
    if (m == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) st16v<NT>(d0 + 1024u * k + 16u * lane, v[k] ^ key);
        return;
    }
    u32x4 x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = v[k] ^ key;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        u32x4 p;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t up = (uint32_t)__shfl_up((int)x[k][j], 1);
            const uint32_t wrap = k ? (uint32_t)__builtin_amdgcn_readlane((int)x[k ? k - 1 : 0][j], 63) : 0u;
            p[j] = lane == 0 ? wrap : up;
        }
        if (k == 0 && lane == 0) {
            store_run<NT>(d0, x[0], 0u, 16u - m);   // the window's first bytes, up to the first boundary
        } else {
            st16v<NT>(d0 + 1024u * k + 16u * lane - m, funnel16(p, x[k], 16u - m));
        }
    }
    if (lane == 63) store_run<NT>(d0 + 4096u - m, x[3], 16u - m, 16u);   // its last m bytes
}

// NT bit 0: non-temporal loads, bit 1: non-temporal stores.  In place `src` is unused (dst is
// both source and destination) so the two restrict pointers never alias in an access; COMPACT
// reads `src` (the wire) and writes `dst` (the arena).  `total` = wire bytes.
template <bool COMPACT, int P, int NT, bool U8>
__device__ __forceinline__ void unmask_all(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                           uint64_t src_bytes, uint64_t total,
                                           const Span* __restrict__ spans,
                                           const uint32_t* __restrict__ tile_first,
                                           const wsc_summary* __restrict__ summary,
                                           uint32_t* __restrict__ lb_state, uint32_t n_walk_blocks, U8Win u8w) {
    constexpr uint32_t WB = 1024u * P;
    static_assert(NT < 16 || !COMPACT, "buffer-instruction windows are the in-place path");
    __shared__ u32x4 pm[17];
    // U8: the launch may meet flagged text windows (the host could not rule them out); binary
    // batches whose walk the host has seen use the variant without the fold and its LDS (g_u8b)
    if (threadIdx.x < 17) pm[threadIdx.x] = prefix_mask16(threadIdx.x);
    if constexpr (U8) if (threadIdx.x == 0) g_u8b.state = 0;
    __syncthreads();
    // re-arm the walk's look-back state for the next decode (this launch is ordered after it):
    // lb_state[0] = ticket, [1] = timeout flag, [3 ...] = per-block flags; and the UTF-8 item
    // counter of the OTHER parity (the next decode's; this decode's is read by k_u8_check after
    // this launch, and re-armed by the next decode's unmask)
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n_walk_blocks + 2; t += gridDim.x * blockDim.x)
        lb_state[t] = 0;
    if (u8w.lb_rec)   // ... and its look-back records (8 words per block)
        for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < 8 * n_walk_blocks; t += gridDim.x * blockDim.x)
            u8w.lb_rec[t] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0 && u8w.rearm) *u8w.rearm = 0;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t waves_per_block = blockDim.x >> 6;
    // XCD runs of 4R consecutive windows (xcd_run_block, wsc_dev.hpp).  Measured: R = 8 streams the
    // headline 1 GiB unmask in 0.319 ms instead of 0.335 (6.73 TB/s), configs[3] 1.316 vs 1.368 ms.
    const uint32_t bid = xcd_run_block(blockIdx.x, gridDim.x, u8w.xcd_run);
    const uint32_t gw = __builtin_amdgcn_readfirstlane(bid * waves_per_block + (threadIdx.x >> 6));
    const uint32_t nw = gridDim.x * waves_per_block;
    const uint32_t n_spans = summary->n_spans;
    const uint64_t n_win = (total + WB - 1) / WB;
    const uint32_t lofs = lane * 16u;
    if (n_spans == 0) return;
    const uint8_t* __restrict__ rd = COMPACT ? src : dst;

    for (uint64_t win = gw; win < n_win; win += nw) {
        const uint64_t wbase = win * WB;
        if (wbase + WB > total) {   // the last, partial window
            const uint32_t r = tile_first[win];
            unmask_window_general<COMPACT, P, NT>(dst, src, src_bytes, total, spans, n_spans, r, wbase, lofs);
            continue;
        }
        u32x4 v[P];
        // the loads do not depend on the span lookup: issue them first
        [[maybe_unused]] __amdgpu_buffer_rsrc_t rs;
        if constexpr (NT >= 16) {
            rs = win_rsrc(dst + wbase, WB);
#pragma unroll
            for (int k = 0; k < P; ++k) v[k] = ld16b<(NT & 1) ? 2 : 0>(rs, k * 1024u + lofs);
        } else {
#pragma unroll
            for (int k = 0; k < P; ++k) v[k] = ld16v<NT>(rd + wbase + k * 1024u + lofs);
        }
        // the fast-path test uses scalar loads (lgkmcnt), so it never waits behind the data loads
        const uint32_t r = tile_first[win];
        [[maybe_unused]] uint32_t text = 0;
        if constexpr (U8) text = u8w.flag[win];   // (beside tile_first: same scalar wait)
        Span s0 = spans[r < n_spans ? r : n_spans - 1];
        if (r >= n_spans) s0.src = ~0ull;   // no span starts before the window's end
        if (s0.src <= wbase && s0.src + s0.len >= wbase + WB) {
            // fast path: one span covers the whole window -> one rotated key for every dword
            if constexpr (COMPACT && WSC_COMPACT_ALIGNED && P == 4) {
                compact_window_aligned<NT>(dst + (s0.dst - s0.src) + wbase, v, s0.key, lane);
            } else if constexpr (COMPACT) {
                uint8_t* d = dst + (s0.dst - s0.src) + wbase + lofs;
#pragma unroll
                for (int k = 0; k < P; ++k) st16u<NT>(d + k * 1024u, v[k] ^ s0.key);
            } else if constexpr (NT >= 16) {
#pragma unroll
                for (int k = 0; k < P; ++k) st16b<(NT >> 4)>(rs, k * 1024u + lofs, v[k] ^ s0.key);
            } else {
#pragma unroll
                for (int k = 0; k < P; ++k) st16v<NT>(dst + wbase + k * 1024u + lofs, v[k] ^ s0.key);
            }
            if constexpr (U8) if (text) fold_text_window<COMPACT, P>(v, s0.key, u8w, win, lane);
            continue;
        }
        // Several spans overlap the window (small frames) or it holds a frame edge: lane-parallel
        // span lookup; more than 64 spans in one window falls back to the serial span walk.
        Span sp;
        const bool valid = load_span_lane(spans, n_spans, r, lane, sp);
        bool done;
        if constexpr (COMPACT && WSC_COMPACT_EDGE2 && P == 4) {
            uint4* stage;
            if constexpr (U8) stage = g_u8b.stage[(threadIdx.x >> 6) & 3];   // (the fold's stage: fast-path windows only)
            else stage = c_stage[(threadIdx.x >> 6) & 3];
            done = unmask_window_lanes_c<P, NT>(dst, sp, valid, n_spans, r, wbase, lane, v, stage);
        } else {
            done = unmask_window_lanes<COMPACT, P, NT>(dst, sp, valid, n_spans, r, wbase, lane, v, pm);
        }
        if (!done) unmask_window_general<COMPACT, P, NT>(dst, src, src_bytes, total, spans, n_spans, r, wbase, lofs);
    }
}

// fin_host (staged pipeline): the last workgroup to finish writes fin_seq to the host-visible
// word (fin_signal, wsc_dev.hpp), after every workgroup has done all its reads of the walk's spans
// / window index -- the host then lets the next walk reuse them (wsc_api.cpp fin_wait).  The
// workgroups that re-armed lb_state release it before counting (the next walk may run while this
// grid's tail drains).
template <bool COMPACT, int P, int NT, int MINW = 1, bool U8 = false>
#ifndef WSC_UNMASK_WPE   // waves per SIMD the P = 4 unmask kernels are built for (with the general window inlined)
#define WSC_UNMASK_WPE 5
#endif
__global__ __launch_bounds__(256, (P == 4 ? WSC_UNMASK_WPE : 2) * MINW) void k_unmask(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                uint64_t src_bytes, uint64_t total,
                                                const Span* __restrict__ spans,
                                                const uint32_t* __restrict__ tile_first,
                                                const wsc_summary* __restrict__ summary,
                                                uint32_t* __restrict__ lb_state, uint32_t n_walk_blocks,
                                                uint32_t* fin_ctr, uint32_t* fin_host, uint32_t fin_seq, U8Win u8w) {
    unmask_all<COMPACT, P, NT, U8>(dst, src, src_bytes, total, spans, tile_first, summary, lb_state, n_walk_blocks, u8w);
    if (fin_host == nullptr) return;
    __syncthreads();
    if (threadIdx.x == 0) {
        if (blockIdx.x * blockDim.x < 8 * n_walk_blocks + 2) __threadfence();   // lb_state re-arm visible first
        fin_signal(fin_ctr, fin_host, fin_seq);
    }
}

}  // namespace wsc
