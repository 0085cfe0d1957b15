// wsc_u8check.inl -- chip-wide UTF-8 verdicts: the work of k_u8_check (wsc_kernels.hip) as a
// device function of (workgroup, workgroups), so that another launch can host it.
#pragma once
#include "wsc_kernels.hpp"
#include "wsc_dev.hpp"
#include "wsc_u8.hpp"

namespace wsc {

// ---------------------------------------------------------------------------------------------
// Chip-wide UTF-8 (utf8.Valid, websocket_frame.go:71-73, websocket.go:170-172) for the text the
// walk deferred, in one launch after the unmask.  The unmask has folded the map of every unmask
// window lying inside an item (win_map).  k_u8_check reads only the items' partial windows at
// their ends, folds them (each lane one 64-byte chunk, waves compose lanes), composes head, window
// maps and tail per item: a whole TEXT message (one piece, SELF) is decided on the spot (its
// ordinal min-folded into the segment's first failure), any other item publishes its map.
// Decoupled verdicts, in the same launch: every published item counts itself into its segment
// (U8Seg.done); the lane whose item completes a segment composes the segment's published maps in
// frame order with the states the walk recorded and applies the verdict: the first failing frame
// becomes WSC_FK_ERROR / 1007, the segment stops there, and the spans of later frames -- already
// unmasked -- are XORed again by the wave, so the bytes are left as the reference leaves them
// (never read).  No second launch and no grid-wide wait.  Maps: wsc_u8.hpp.
// Cross-XCD hand-off (L2 is per XCD): maps are published with agent-scope (sc1) stores and the
// failures with agent-scope atomics, drained (s_waitcnt) before the segment's counter increment;
// the completing lane reads them with agent-scope atomic RMWs (MI355X_MICROARCH.md "Valid forms").
// ---------------------------------------------------------------------------------------------

// One item's result: U8R_DEAD (an unused pool slot), U8R_PASS / U8R_FAIL (a single-piece TEXT
// message: nothing is written when it passes), U8R_COMP (any other item: its map is published,
// then counted into its segment once drained).
enum : uint32_t { U8R_DEAD = 0, U8R_PASS = 1, U8R_FAIL = 2, U8R_COMP = 3 };
__device__ __forceinline__ uint32_t u8_store(const U8Args& a, uint32_t it, const U8Item& self, uint64_t acc) {
    if (self.seg == U8_DEAD) return U8R_DEAD;
    if (self.kind == U8K_SELF && self.first && self.last) return u8m_get(acc, 0) != 0 ? U8R_FAIL : U8R_PASS;
    __hip_atomic_store(a.maps + it, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return U8R_COMP;
}
// `cnt` composite items counted into their segment, after the lane's map stores are drained:
// `ret` = the count before them, `n` = the segment's composite items (ret + cnt == n: they
// complete it -- the lane composes the segment's chains).  The caller reads ret / n late.
__device__ __forceinline__ void u8_count(const U8Args& a, uint32_t seg, uint32_t cnt, uint32_t& ret, uint32_t& n) {
    n = a.seg[seg].n;
    ret = __hip_atomic_fetch_add(&a.seg[seg].done, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A segment's composite items composed in frame order with the walk's states (one lane, once all
// are published): the first failing composite frame's ordinal, 0xFFFFFFFF if none -- then an open
// text chain (continueBuffer and/or a streamed frame's pieces) carries its DFA state.  Single-piece
// SELF items never sit inside a chain and are skipped.
__device__ __forceinline__ uint32_t u8_comp_verdict(const U8Args& a, uint32_t s, const U8Seg& g) {
    uint32_t cur = 0, start = 0;   // states 0..7, 0xFF = reject
    uint32_t pcur = 0;             // an open streamed PONG's state (its own chain, Q6)
    uint64_t fm = u8m_id();
    uint32_t j = g.head;
    for (uint32_t c = 0; c < a.items_cap && j != 0xFFFFFFFFu; ++c) {
        const U8Item x = a.items[j];
        if (x.kind == U8K_SELF && x.first && x.last) { j = x.next; continue; }
        const uint64_t m = __hip_atomic_fetch_add(a.maps + j, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (x.first) {
            if (x.kind >= U8K_PONG) start = x.s_in > 7 ? 0xFFu : (uint32_t)x.s_in;   // known at the walk
            else start = x.kind == U8K_SELF ? 0u : (x.s_in != 0xFF ? (x.s_in > 7 ? 0xFFu : (uint32_t)x.s_in) : cur);
            fm = u8m_id();
        }
        fm = u8m_then(fm, m);
        if (x.last) {
            const uint32_t end = u8m_get(fm, start);
            if (x.kind == U8K_PART) {
                cur = end;
            } else if (x.kind == U8K_PONG) {
                pcur = end;
            } else {
                if (end != 0) return x.ordinal;
                if (x.kind == U8K_CHAIN) cur = 0;
            }
        }
        j = x.next;
    }
    if (g.pending_end & 5u) {
        wsc_conn_state* so = a.state_out + s;
        if ((g.pending_end & 1u) && (so->cont_len || so->frame_rem)) so->cont_utf8 = (uint8_t)(cur > 7 ? 8u : cur);
        if (g.pending_end & 4u) so->frame_utf8 = (uint8_t)(pcur > 7 ? 8u : pcur);
        // a single-piece TEXT item of this segment may fail concurrently (u8_fail, another wave),
        // and a closed connection carries no open state (round-4 ADVICE): store, full fence, then
        // look at the segment's failure minimum -- u8_fail sets it (seq_cst) before it zeroes the
        // state, so whichever side runs second leaves the state zero
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        if (__hip_atomic_load(&a.seg[s].minfail, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT) != 0xFFFFFFFFu) {
            so->cont_utf8 = 0;
            so->frame_utf8 = 0;
        }
    }
    return 0xFFFFFFFFu;
}

// Frame `ord` of segment s fails utf8.Valid (one lane): CloseCode(1007) there (epoll.go:126-127),
// nothing after it is read.  Failures of one segment may be found in any order, so each takes
// part only if it lowers the segment's minimum: its record becomes WSC_FK_ERROR, the segment's
// consumed bytes and frame count are min-folded (a smaller failure always gives smaller values),
// and the spans between this frame's end and the previous minimum's end are re-masked (those past
// the previous minimum's end were re-masked when it took part).  Returns that wire range
// [lo, hi) (empty: nothing to re-mask).
__device__ __forceinline__ void u8_fail(const U8Args& a, uint32_t s, uint32_t ord, uint64_t& lo, uint64_t& hi) {
    lo = hi = 0;
    const uint32_t old = __hip_atomic_fetch_min(&a.seg[s].minfail, ord, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT);
    if (ord >= old) return;   // an earlier frame already failed
    const uint32_t fbase = a.seg[s].fbase;
    auto frame_end = [&](uint32_t o) {
        const wsc_frame* f = a.frames + fbase + o;
        return f->hdr_off + f->hdr_len + (f->payload_len | (uint64_t)f->payload_len_hi << 32);
    };
    wsc_frame* f = a.frames + fbase + ord;
    f->kind = WSC_FK_ERROR;
    f->err = WSC_ERR_MUST_UTF8;
    const uint64_t fend = frame_end(ord);
    wsc_seg_result* r = a.seg_out + s;
    __hip_atomic_fetch_min(&r->consumed, fend - a.seg_off[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_min(&r->frame_count, ord + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    r->status = WSC_SEG_ERROR;
    r->close_code = 1007;
    r->err = WSC_ERR_MUST_UTF8;
    // a closed connection carries no frame in progress (as the walk's own terminal paths leave it)
    wsc_conn_state* so = a.state_out + s;
    so->status = WSC_SEG_ERROR;
    so->frame_rem = 0;
    so->frame_len = 0;
    so->frame_mask = 0;
    so->frame_hdr = 0;
    so->frame_utf8 = 0;
    so->cont_utf8 = 0;
    lo = fend;
    hi = old == 0xFFFFFFFFu ? ~0ull : frame_end(old);
}

// The segment's spans that start in [lo, hi) were unmasked although the reference never reads
// them: XOR them again, the whole wave 16 B per lane (1 KiB per step).  The key is phased at the
// wire (byte x takes key byte x & 3), in place and in the arena alike.
__device__ __forceinline__ void u8_remask(const U8Args& a, uint32_t seg, uint64_t lo, uint64_t hi, uint32_t lane) {
    const U8Seg g = a.seg[seg];
    for (uint32_t k = 0; k < g.nspans; ++k) {
        const Span sp = a.spans[g.sbase + k];
        if (sp.src < lo || sp.src >= hi) continue;
        uint8_t* d = a.out + sp.dst;
        for (uint32_t i = lane * 16u; i < sp.len; i += 1024u) {
            const uint32_t key = rotr32(sp.key, 8u * (uint32_t)((sp.src + i) & 3));
            if (sp.len - i >= 16) {
                u32x4u* p = reinterpret_cast<u32x4u*>(d + i);
                const u32x4u v = *p;
                *p = u32x4u{v.x ^ key, v.y ^ key, v.z ^ key, v.w ^ key};
            } else {
                for (uint32_t j = 0; i + j < sp.len; ++j) d[i + j] ^= (uint8_t)(key >> (8 * (j & 3)));
            }
        }
    }
}

// 5 waves per SIMD (96 VGPRs).  Each lane folds a 64-byte chunk (4 x 16 B loads) into one map, so
// the wave-level composition (DPP row levels + 4 readlanes) is paid once per 64 bytes instead of
// per 16: PMC showed the 16-byte-piece version at 12.5 VALU per text byte, VALU-bound (77 % of
// the chip's VALU cycles).
// The check's work for workgroup `bid` of `nblk` check workgroups.  T / stage: the workgroup's LDS
// tables and per-wave stages.
// WSC_CHECK_PREFETCH 1: a small unit's data loads go out one unit ahead.  Off: the second 16-VGPR
// buffer pushed the kernel past 128 VGPRs into 20 B of spills; without it 127 VGPRs and none, and
// 1 KiB TEXT 0.218 -> 0.214 ms, 64 KiB 0.417 -> 0.413 ms (profiles/r04_check_variants_ab.log;
// built for 5 waves per SIMD instead, 96 VGPRs with 112-188 B of spills, the check ran 2.5-5x slower)
#ifndef WSC_CHECK_PREFETCH
#define WSC_CHECK_PREFETCH 0
#endif
// WPB: waves per workgroup (4: 256-thread workgroups; 16: one 1024-thread workgroup per CU, a
// quarter of the workgroups to dispatch for the same waves)
template <uint32_t NCH, uint32_t WPB = 4>
__device__ __forceinline__ void u8_check_run(const U8Args& a, U8Lds& T, uint4 (*stage)[U8_STAGE], uint32_t bid,
                                             uint32_t nblk) {
    // (items past the capacity were dropped by the walk: only a batch whose records overflowed
    // allocates that many, and its verdicts are skipped below)
    const uint32_t n_items = *a.count < a.items_cap ? *a.count : a.items_cap;
    const uint32_t lane = threadIdx.x & 63;
    // a batch whose records overflowed is invalid as a whole (the caller re-decodes it): its
    // verdicts are not applied -- the failing frame or its later spans may lie past the capacity
    const bool ovf = a.summary->overflow != 0;
    // failing frames of this wave (ordinal `ord` of segment `seg` on the lanes where `f`): each
    // applied by its lane, the spans it hands back re-masked by the whole wave
    auto rd64 = [](uint64_t v, uint32_t l) {
        return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l) << 32 |
               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
    };
    auto fail_settle = [&](bool f, uint32_t seg, uint32_t ord) {
        uint64_t pend = __ballot(f && !ovf);
        while (pend) {
            const uint32_t l = (uint32_t)__builtin_ctzll(pend);
            pend &= pend - 1;
            const uint32_t sg = (uint32_t)__builtin_amdgcn_readlane((int)seg, (int)l);
            uint64_t lo = 0, hi = 0;
            if (lane == l) u8_fail(a, sg, ord, lo, hi);
            lo = rd64(lo, l);
            hi = rd64(hi, l);
            if (lo < hi) u8_remask(a, sg, lo, hi, lane);
        }
    };
    // segments whose composite items this wave completed: their chains composed (one lane each,
    // serial over the segment's items), a failing frame applied as above
    auto settle = [&](bool trig, uint32_t seg) {
        uint32_t ord = 0xFFFFFFFFu;
        if (trig && !ovf) ord = u8_comp_verdict(a, seg, a.seg[seg]);
        fail_settle(ord != 0xFFFFFFFFu, seg, ord);
    };
    if (bid * WPB < n_items) {   // (nothing deferred, or fewer units than waves: only the signal)
    if (threadIdx.x < 256) u8_tables_init(T, threadIdx.x);
    __syncthreads();
    const uint32_t gw = __builtin_amdgcn_readfirstlane(bid * WPB + (threadIdx.x >> 6));
    const uint32_t nw = nblk * WPB;
    // Global loads stay coalesced (piece k of a step: 16 B per lane at base_k + 16 * lane, 1 KiB
    // per instruction); a per-wave LDS stage turns them into one contiguous 64-byte chunk per lane.
    // Strided 16-byte global loads at a 64-byte lane stride measured slower.
    uint4* const sw = stage[threadIdx.x >> 6];
    const uint64_t W = 1ull << a.win_shift;
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    // An item reads its head [0, hl) and tail [tb, len); the unmask windows between them
    // (w0 .. w0 + nwin - 1) were folded by the unmask.  An item without a whole window is all head.
    struct Geo { uint32_t hl, tb, nwin; uint64_t w0; };
    auto geo = [&](const U8Item& x) -> Geo {
        const uint64_t s = x.src, e = s + x.len;
        const uint64_t A = (s + W - 1) & ~(W - 1), B = e & ~(W - 1);
        Geo g;
        if (A < B) {
            g.hl = (uint32_t)(A - s);
            g.tb = (uint32_t)(B - s);
            g.w0 = A >> a.win_shift;
            g.nwin = (uint32_t)((B - A) >> a.win_shift);
        } else {
            g.hl = x.len;
            g.tb = x.len;
            g.w0 = 0;
            g.nwin = 0;
        }
        return g;
    };
    auto first_step = [&](const Geo& g, uint32_t len) -> uint32_t { return g.hl ? 0u : (g.tb < len ? g.tb : NONE); };
    auto next_step = [&](const Geo& g, uint32_t len, uint32_t b0) -> uint32_t {
        if (b0 < g.hl) return b0 + 4096 < g.hl ? b0 + 4096 : (g.tb < len ? g.tb : NONE);
        return b0 + 4096 < len ? b0 + 4096 : NONE;
    };
    // the step's mask: phase 0 at item offset b0 (in place the wire is already unmasked)
    auto mask_at = [&](const U8Item& x, uint32_t b0) -> uint32_t {
        return a.unmasked ? 0u : rotr32(x.mask, 8u * (b0 & 3));
    };
    // a 4 KiB step of item x at item offset b0, bytes [b0, lim) (coalesced; others read as 0)
    auto fetch = [&](const U8Item& x, uint32_t b0, uint32_t lim, u32x4 (&q)[4]) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t o = b0 + 1024u * k + 16u * lane;
            const uint4 t = o < lim ? load16_unaligned(a.wire, (int64_t)(x.src + o), a.n_bytes) : make_uint4(0, 0, 0, 0);
            q[k] = u32x4{t.x, t.y, t.z, t.w};
        }
    };
    auto chunk_len = [](uint32_t len, uint32_t off) -> uint32_t {
        return off < len ? (len - off >= 64 ? 64u : len - off) : 0u;
    };
    // A unit is 4 consecutive items.  Units of small items (<= 1 KiB each: 1 KiB text frames) take
    // one step: row r (16 lanes x 64 B) holds item r, and lanes 0, 16, 32, 48 publish the 4 items'
    // maps.  Other units walk their items' steps in order, the next step's loads -- the next
    // item's first step too -- issued before the current step is folded.  (A ticket counter for
    // dynamic balance measured far slower: 64 k same-address atomics; a second pass striding big
    // items one by one paid a scan of every unit's lengths per wave.)
    // Other units walk their items' steps in order, the next step's loads -- the next item's first
    // step too -- issued before the current step is folded.
    auto unit_large = [&](uint32_t i0, uint32_t cnt) {
        // (prefetch within an item only: carrying the next item's geometry and first step across
        // the fold held ~15 more VGPRs, past 128)
        for (uint32_t j = 0; j < cnt; ++j) {
            const U8Item item = a.items[i0 + j];
            const Geo g = geo(item);
            uint32_t b0 = first_step(g, item.len);
            u32x4 nxt[4];
            if (b0 != NONE) fetch(item, b0, b0 < g.hl ? g.hl : item.len, nxt);
            // the windows between head and tail, folded by the unmask: each lane composes a run
            // of ceil(nwin / 64) of them, the wave composes the lanes in order
            uint64_t mids = u8m_id();
            if (g.nwin) {
                const uint32_t k = (g.nwin + 63) / 64;
                uint64_t m = u8m_id();
                for (uint32_t q = 0; q < k; ++q)
                    if (lane * k + q < g.nwin) m = u8m_then(m, a.win_map[g.w0 + (uint64_t)lane * k + q]);
                mids = u8_wave_map(m, false, lane);
            }
            uint64_t acc = u8m_id();
            bool mids_in = false;
            while (b0 != NONE) {
                u32x4 cur4[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) cur4[k] = nxt[k];
                const uint32_t nb = next_step(g, item.len, b0);
                if (nb != NONE) fetch(item, nb, nb < g.hl ? g.hl : item.len, nxt);
                u8_restage(sw, cur4, lane);
                const uint32_t lim = b0 < g.hl ? g.hl : item.len;
                bool plain;
                const uint64_t pm = u8_chunk_map<NCH, U8P_WAVE>(T, cur4, mask_at(item, b0), chunk_len(lim, b0 + lane * 64), plain);
                const uint64_t wm = u8_wave_map(pm, plain, lane);
                if (b0 >= g.hl && !mids_in) {   // the first tail step: the windows come before it
                    acc = u8m_then(acc, mids);
                    mids_in = true;
                }
                acc = u8m_then(acc, wm);
                b0 = nb;
            }
            if (!mids_in) acc = u8m_then(acc, mids);
            uint32_t res = U8R_DEAD, ret = 0, n = 0;
            if (lane == 0) res = u8_store(a, i0 + j, item, acc);
            res = (uint32_t)__builtin_amdgcn_readfirstlane((int)res);
            fail_settle(lane == 0 && res == U8R_FAIL, item.seg, item.ordinal);
            if (res == U8R_COMP) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the map before the count
                if (lane == 0) u8_count(a, item.seg, 1u, ret, n);
            }
            settle(lane == 0 && res == U8R_COMP && ret + 1 == n, item.seg);
        }
    };
    const uint32_t n_units = (n_items + 3) / 4;
    // A small unit's 4 items as the step needs them (uniform, scalar loads); entries past the last
    // item have len 0.
    struct UnitS { uint64_t src[4]; uint32_t len[4], mask[4]; };
    auto unit_items = [&](uint32_t u, UnitS& x) {
        const uint32_t i0 = 4 * u, cnt = n_items - i0 < 4 ? n_items - i0 : 4u;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const U8Item it = a.items[i0 + (k < cnt ? k : 0u)];
            x.src[k] = it.src;
            x.len[k] = k < cnt ? it.len : 0u;
            x.mask[k] = it.mask;
        }
    };
    auto unit_small = [](const UnitS& x) -> bool {
        return x.len[0] <= 1024 && x.len[1] <= 1024 && x.len[2] <= 1024 && x.len[3] <= 1024;
    };
    // piece k of a small unit's step = item k's KiB (16 B per lane, coalesced)
    auto unit_data = [&](const UnitS& x, u32x4 (&q)[4]) {
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint4 t = 16u * lane < x.len[k] ? load16_unaligned(a.wire, (int64_t)(x.src[k] + 16u * lane), a.n_bytes)
                                                  : make_uint4(0, 0, 0, 0);
            q[k] = u32x4{t.x, t.y, t.z, t.w};
        }
    };
    // Software pipeline over a wave's units: the next unit's items are loaded one unit ahead, and
    // (small units) its data loads go out before this unit's verdict atomics, so the dependent
    // round trips of consecutive units overlap (1 KiB text: 4 per unit otherwise)
    UnitS xc, xn;
    u32x4 qc[4] = {};
    bool cur_small = false;
    // the previous small unit's counts, settled one unit later (after the next unit's loads are
    // out): the counter round trip is then never waited for on its own
    bool pact = false;
    uint32_t pret = 0, pn = 0, pseg = 0, pcnt = 0;
    if (gw < n_units) {
        unit_items(gw, xc);
        cur_small = unit_small(xc);
        if (cur_small && WSC_CHECK_PREFETCH) unit_data(xc, qc);
    }
    if (gw + nw < n_units) unit_items(gw + nw, xn);
    for (uint32_t u = gw; u < n_units; u += nw) {
        const uint32_t i0 = 4 * u;
        const uint32_t cnt = n_items - i0 < 4 ? n_items - i0 : 4u;
        const uint32_t un = u + nw;
        bool nsmall = false;
        u32x4 qn[4] = {};
        if (cur_small) {
            if (!WSC_CHECK_PREFETCH) unit_data(xc, qc);
            // restaged so that row r (lanes 16r..16r+15) holds item r in 64-byte chunks (items
            // <= 1 KiB hold no window).  The row's full item is needed only by the verdict: its
            // load overlaps the fold.
            const uint32_t r = lane >> 4;
            const U8Item xr = a.items[i0 + (r < cnt ? r : 0u)];
            const uint32_t rlen = r < cnt ? xr.len : 0u;   // (row r's fields from its item: no selects)
            const uint32_t rmask = xr.mask;
            u8_restage(sw, qc, lane);
            const uint32_t off = (lane & 15) * 64;
            bool plain;
            const uint64_t pm = u8_chunk_map<NCH, U8P_LANE>(T, qc, a.unmasked ? 0u : rmask, chunk_len(rlen, off), plain);
            const uint64_t rm = u8_row_maps(pm, lane);
            if (un < n_units) {
                nsmall = unit_small(xn);
                if (nsmall && WSC_CHECK_PREFETCH) unit_data(xn, qn);
            }
            settle(pact && pret + pcnt == pn, pseg);
            // the unit's items: failures applied at once; composite items counted per run of
            // rows on one segment (a walk pool hands a segment 4 consecutive slots), one counter
            // atomic per run
            uint32_t res = U8R_DEAD;
            if ((lane & 15) == 0 && r < cnt) res = u8_store(a, i0 + r, xr, rm);
            fail_settle(res == U8R_FAIL, xr.seg, xr.ordinal);
            const bool ok = res == U8R_COMP;
            if (__ballot(ok)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // maps before counts
            const uint64_t okm = __ballot(ok);
            uint32_t rs[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) rs[q] = (uint32_t)__builtin_amdgcn_readlane((int)xr.seg, 16 * q);
            auto row_ok = [&](uint32_t q) { return ((okm >> (16 * q)) & 1) != 0; };
            pact = false;
            pcnt = 0;
            if (ok) {
                const uint32_t sg = xr.seg;
                const bool head = !(r > 0 && row_ok(r - 1) && rs[r - 1] == sg);
                if (head) {
                    uint32_t run = 1;
                    while (r + run < 4 && row_ok(r + run) && rs[r + run] == sg) ++run;
                    u8_count(a, sg, run, pret, pn);
                    pact = true;
                    pcnt = run;
                }
            }
            pseg = xr.seg;
        } else {
            settle(pact && pret + pcnt == pn, pseg);
            pact = false;
            unit_large(i0, cnt);
            if (un < n_units) {
                nsmall = unit_small(xn);
                if (nsmall && WSC_CHECK_PREFETCH) unit_data(xn, qn);
            }
        }
        xc = xn;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) qc[k] = qn[k];
        cur_small = nsmall;
        if (un + nw < n_units) unit_items(un + nw, xn);
    }
    settle(pact && pret + pcnt == pn, pseg);
    }
}

}  // namespace wsc
