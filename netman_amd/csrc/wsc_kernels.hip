// wsc_kernels.hip -- gfx950 kernels of the WebSocket frame decoder.
//
//   k_walk_fused<COMPACT,KR,G> header walk + per-frame decode state machine, one lane per G segments
//                         (server/websocket.go:82-302, server/websocket_frame.go:13-103 minus the
//                         byte loops).  Count, block scan + decoupled look-back, then emit frame
//                         records, payload spans and the window->span index, in one launch.
//   k_unmask<COMPACT,P,NT> the hot loop (websocket_frame.go:35-39): XOR-unmask every payload span,
//                         byte-tile decomposed, 16 B per lane access, 1 KiB per wave instruction.
//   utf8.Valid (websocket_frame.go:71-73, websocket.go:170-172): payloads up to u8_inline_max run
//   inside the walk's counting pass on the still-masked wire, so a connection whose text is invalid
//   stops at that frame.  Larger ones are deferred: the unmask folds the windows it unmasks
//   (wsc_unmask.inl), k_u8_check the partial windows and applies 1007 (below).
#include "wsc_kernels.hpp"
#include "wsc_dev.hpp"
#include "wsc_u8.hpp"
#include "wsc_u8check.inl"

namespace wsc {


// ---------------------------------------------------------------------------------------------
// Header walk
// ---------------------------------------------------------------------------------------------

__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// close-code validity, websocket_ctrl.go:160-177 (+ reservedCode, websocket.go:31)
__device__ __forceinline__ bool close_code_ok(uint32_t code) {
    if (code < 1000 || code >= 5000) return false;
    if (code >= 1016 && code <= 2999) return false;
    if (code == 1004 || code == 1005 || code == 1006 || code == 1015) return false;
    return true;
}

// Walk one segment's frames (one lane).  Pass 1 (EMIT=false) only counts; pass 2 (EMIT=true)
// writes frame records, payload spans, the window->span index and the segment's results at the
// output offsets `base` (exclusive prefix over segments) for its counts `own` (pass 1 result).
// COMPACT arena layout per segment: [data payloads][control payloads] at base.bytes0+base.bytes1.
// UTF-8 (Go utf8.Valid semantics): a 9-state DFA, state 0 = between characters, 8 = reject
// (u8_step, wsc_u8.hpp).
// Run the DFA over n payload bytes that are still MASKED on the wire: byte i of the payload is
// w[p + i] ^ (mask >> 8*(i & 3)).  4-byte ASCII groups are skipped while between characters.
__device__ __attribute__((noinline)) uint32_t u8_run_masked(uint32_t s, const uint8_t* __restrict__ w, uint64_t p, uint64_t n,
                                  uint32_t mask) {
    uint64_t i = 0;
    while (i < n && s != 8) {
        if (s == 0 && ((p + i) & 3) == 0 && i + 4 <= n) {
            const uint32_t v = *reinterpret_cast<const uint32_t*>(w + p + i) ^ rotr32(mask, 8u * (uint32_t)(i & 3));
            if ((v & 0x80808080u) == 0) { i += 4; continue; }
        }
        s = u8_step(s, (uint32_t)w[p + i] ^ ((mask >> (8u * (uint32_t)(i & 3))) & 0xFFu));
        ++i;
    }
    return s;
}

// Header fetch: the longest masked header is 14 bytes, so ONE byte-aligned 16-byte load at the
// frame's first byte covers it (gfx950 takes unaligned dwordx4 addresses); the last 16 bytes of the
// buffer are read byte by byte (nothing past n).  Bytes past the segment end are never used
// (every use is guarded by `avail`).
// nt (WalkArgs.hdr_nt; the host sets it for COMPACT batches): a non-temporal load.  Measured
// (profiles/r04_hdr_nt_ab.log, r04_hdr_nt_policy_ab.log; FETCH bytes unchanged): the configs[4]
// (COMPACT) walk 91 -> 65 us, decode -2.5 %; in place the unmask re-reads the header lines and
// loses what the walk gains (configs[1], [2], [3]: walk -2..-6 us, unmask +2..+6 us).
__device__ __forceinline__ uint4 hdr_load(const uint8_t* __restrict__ w, uint64_t n, uint64_t pos, bool nt) {
    return nt ? load16u<1>(w, (int64_t)pos, n) : load16_unaligned(w, (int64_t)pos, n);
}
__device__ __forceinline__ void hdr_bytes(const uint4& hd, uint32_t (&h)[14]) {
    const uint32_t d[4] = {hd.x, hd.y, hd.z, hd.w};
#pragma unroll
    for (int k = 0; k < 14; ++k) h[k] = (d[k >> 2] >> (8 * (k & 3))) & 0xFFu;
}

// Output side of the walk: everything a frame writes (record, arena offset, span, window index)
// and what a segment writes at its end.  Shared by the LDS replay and the re-walking emitter so
// both produce identical outputs.
struct EmitCtx {
    uint32_t s;
    uint64_t seg_start, seg_end;
    uint64_t abase;          // COMPACT: this segment's arena offset
    uint32_t sbase;          // first span index of this segment
    uint32_t fbase;          // first frame index of this segment
    uint64_t own_bytes0;     // COMPACT: data bytes of this segment (control payloads follow)
    uint32_t own_spans0;
    uint32_t nf, ns0, ns1;
    uint64_t nb0, nb1;
    uint64_t nx0, nx1;       // next window start not yet assigned, per region
};

template <bool COMPACT>
__device__ __forceinline__ EmitCtx emit_begin(const WalkArgs& a, uint32_t s, uint64_t seg_start,
                                              uint64_t seg_end, const SegCount& base, const SegCount& own) {
    EmitCtx e;
    e.s = s;
    e.seg_start = seg_start;
    e.seg_end = seg_end;
    e.abase = base.bytes0 + base.bytes1;
    e.sbase = base.spans0 + base.spans1;
    e.fbase = base.frames;
    e.own_bytes0 = own.bytes0;
    e.own_spans0 = own.spans0;
    e.nf = e.ns0 = e.ns1 = 0;
    e.nb0 = e.nb1 = 0;
    // spans are emitted in stream order in both modes and the window index is keyed by wire
    // offset: the unmask reads the wire window by window (COMPACT stores each run at its arena dst)
    const uint64_t W = 1ull << a.win_shift;
    e.nx0 = (seg_start + W - 1) & ~(W - 1);
    e.nx1 = 0;
    return e;
}

template <bool COMPACT>
__device__ __forceinline__ void emit_frame(const WalkArgs& a, EmitCtx& e, const wsc_frame& fr, uint64_t plen,
                                           bool have_span, uint32_t region) {
    const uint32_t fi = e.fbase + e.nf;
    if (fi < a.frames_cap) {
        // two 16-byte stores (the record is 32 B)
        const uint4 r0 = make_uint4((uint32_t)fr.hdr_off, (uint32_t)(fr.hdr_off >> 32), fr.payload_len, fr.mask);
        const uint4 r1 = make_uint4(fr.seg, fr.msg_id,
                                    (uint32_t)fr.opcode | (uint32_t)fr.fin << 8 | (uint32_t)fr.kind << 16 |
                                        (uint32_t)fr.mode << 24,
                                    (uint32_t)fr.err | (uint32_t)fr.hdr_len << 8 | (uint32_t)fr.flags << 16 |
                                        (uint32_t)fr.payload_len_hi << 24);
        reinterpret_cast<uint4*>(a.frames + fi)[0] = r0;
        reinterpret_cast<uint4*>(a.frames + fi)[1] = r1;
        if constexpr (COMPACT) {
            uint64_t d = ~0ull;
            if (fr.flags & WSC_FF_UNMASKED) d = region ? e.abase + e.own_bytes0 + e.nb1 : e.abase + e.nb0;
            a.frame_dst[fi] = d;
        }
    }
    if (have_span) {
        // a payload of 4 GiB or more is cut at absolute SPAN_CHUNK-aligned wire offsets (the key
        // is wire-phased, so every piece keeps it); span_chunks() counted them the same way
        const uint64_t src0 = fr.hdr_off + fr.hdr_len;
        const uint32_t nch = span_chunks(src0, plen);
        uint64_t dst0 = src0;
        if (COMPACT && region) dst0 = e.abase + e.own_bytes0 + e.nb1;
        else if (COMPACT) dst0 = e.abase + e.nb0;
        // the key is phased at the wire: every aligned wire dword XORs with one register
        const uint32_t key = rotr32(fr.mask, 8u * ((uint32_t)(0u - (uint32_t)src0) & 3u));
        for (uint32_t c = 0; c < nch; ++c) {
            const uint64_t cs = c == 0 ? src0 : ((src0 >> 31) + c) << 31;
            const uint64_t ce = c + 1 == nch ? src0 + plen : ((src0 >> 31) + c + 1) << 31;
            Span sp;
            sp.src = cs;
            sp.dst = dst0 + (cs - src0);
            sp.len = (uint32_t)(ce - cs);
            sp.key = key;
            const uint32_t idx = e.sbase + e.ns0 + e.ns1 + c;   // stream order
            if (idx < a.spans_cap) a.spans[idx] = sp;
            const uint64_t dend = sp.src + sp.len;
            uint64_t& nx = e.nx0;
            if (nx < dend) {   // windows [nx, dend) start inside this span: consecutive entries
                uint64_t t = nx >> a.win_shift;
                const uint64_t t_end = ((dend - 1) >> a.win_shift) + 1;
                nx = t_end << a.win_shift;
                for (; t < t_end && (t & 3); ++t) a.tile_first[t] = idx;
                const uint4 q = make_uint4(idx, idx, idx, idx);
                for (; t + 4 <= t_end; t += 4) *reinterpret_cast<uint4*>(a.tile_first + t) = q;
                for (; t < t_end; ++t) a.tile_first[t] = idx;
            }
        }
        if (COMPACT && region) { e.ns1 += nch; e.nb1 += plen; }
        else { e.ns0 += nch; e.nb0 += plen; }
    }
    e.nf += 1;
}

// the walk's final per-connection state (from the counting pass)
struct WalkEnd {
    uint64_t pos, cont;
    uint64_t last_dend;      // wire end of the segment's last payload span (seg_start if none)
    uint64_t frem, flen;     // the in-progress (streamed) data frame: payload still to come, length
    uint32_t fmask, fhdr;    // ... its mask phased to the next payload byte, FIN << 7 | opcode
    uint32_t msg, mode, status, close_code, err, u8dfa;
    uint32_t pdfa;           // an in-progress PONG under TEXT mode: DFA state of its bytes so far
    bool replay;             // counting pass: the LDS records hold the whole segment
};

// the carried state a walk leaves (websocket.go:38-56 subset + the streamed frame)
__device__ __forceinline__ wsc_conn_state end_state(const WalkEnd& w) {
    wsc_conn_state o;
    o.cont_len = w.cont;
    o.msg_id = w.msg;
    o.message_mode = (uint8_t)w.mode;
    o.cont_utf8 = (w.cont || w.frem) ? (uint8_t)w.u8dfa : 0;
    o.status = (uint8_t)w.status;
    o.frame_hdr = w.frem ? (uint8_t)w.fhdr : 0;
    o.frame_rem = w.frem;
    o.frame_len = w.frem ? w.flen : 0;
    o.frame_mask = w.frem ? w.fmask : 0;
    o.frame_utf8 = (w.frem && (w.fhdr & 0xFu) == 10u) ? (uint8_t)w.pdfa : 0;
    o.pad[0] = o.pad[1] = o.pad[2] = 0;
    return o;
}

template <bool COMPACT>
__device__ __forceinline__ void emit_end(const WalkArgs& a, EmitCtx& e, const WalkEnd& w) {
    const uint64_t W = 1ull << a.win_shift;
    // windows that start in this segment's region(s) after its last span
    for (; e.nx0 < e.seg_end; e.nx0 += W) a.tile_first[e.nx0 >> a.win_shift] = e.sbase + e.ns0 + e.ns1;
    wsc_seg_result r;
    r.consumed = w.pos - e.seg_start;
    r.frame_begin = e.fbase;
    r.frame_count = e.nf;
    r.status = w.status;
    r.close_code = w.close_code;
    r.err = w.err;
    r.pad = 0;
    a.seg_out[e.s] = r;
    a.state_out[e.s] = end_state(w);
}


// LDS record of the counting pass: header offset in the segment, payload length, mask, and the
// frame's fields packed into one word -- opcode 0-3, fin 4, kind 5-8, mode 9-10, err 11-13,
// hdr_len 14-17, flags 18-25, region 26, have_span 27, the lane's segment (tag) 28-31
__device__ __forceinline__ uint4 rec_pack(const wsc_frame& fr, uint64_t seg_start, bool have_span,
                                          uint32_t region) {
    const uint32_t bits = (uint32_t)fr.opcode | (uint32_t)fr.fin << 4 | (uint32_t)fr.kind << 5 |
                          (uint32_t)fr.mode << 9 | (uint32_t)fr.err << 11 | (uint32_t)fr.hdr_len << 14 |
                          (uint32_t)fr.flags << 18 | region << 26 | (uint32_t)have_span << 27;
    return make_uint4((uint32_t)(fr.hdr_off - seg_start), fr.payload_len, fr.mask, bits);
}

// Walk one segment's frames (one lane).  Pass 1 (EMIT=false) counts, decides utf8 verdicts and
// keeps up to `cap` frame records in LDS (lrec / lrec2, stride LS); pass 2 (EMIT=true, only for
// segments with more frames) re-walks and writes every output at the offsets `base` (exclusive
// prefix over segments).
//
// The header chain is serial, so the walk fetches SPEC_D headers per memory round trip: the
// next header and the ones at +stride, +2*stride, ... (stride = the last frame's size).  A
// speculative header is used only when its address is the real next position, so results never
// depend on the guess; frames that repeat their size (the common case on one connection) cost
// one round trip per SPEC_D frames.  All loads of a round are waited together.
// Depth 2 by default: the chain of one walking wave per CU is bound by its own instruction
// latency (one wave per SIMD, nothing to interleave), and the header queue's register shifts grow
// with the depth -- measured (profiles/r03_walk_spec_ab*.log): configs[4] walk 76 -> 61 us,
// configs[2] 34.7 -> 33.7 us at depth 2 vs 4; 8 and 16 are slower still.
#ifndef WSC_WALK_SPEC
#define WSC_WALK_SPEC 2
#endif

// A segment's inputs loaded ahead by the caller (the tiled walk pipelines them across tiles): its
// bounds, its carried state and the 16 bytes at its first frame.
struct SegIn {
    uint64_t start, end;
    uint4 hdr;
    wsc_conn_state st;
};

// What the quad pre-pass (quad_prefix, below) already walked of a segment: its leading run of
// plain complete BIN messages, recorded in LDS.  The serial walk continues after it.  Offsets are
// relative to the segment start (the pre-pass runs only on segments < 4 GiB).
struct PreState {
    uint32_t nf, ns, nb;   // frames recorded, spans, payload bytes (region 0)
    uint32_t pos, pend;    // where the walk continues; wire end of the last span
    uint32_t msg, stride;  // msgID after the run; the stride it speculated with last
    bool full;             // the run reached the segment's end (< 2 bytes left): no serial walk
};

// A frame the pre-pass takes -- a plain complete masked BIN message, the serial walk's `fast`
// path -- as the record walk_segment would keep for it (rec_pack, tag 0: one segment per lane)
__device__ __forceinline__ uint4 pre_record(uint64_t hdr_off, uint32_t plen, uint32_t mask, uint32_t hl,
                                            uint64_t seg_start) {
    wsc_frame fr{};
    fr.hdr_off = hdr_off;
    fr.payload_len = plen;
    fr.mask = mask;
    fr.opcode = 2;
    fr.fin = 1;
    fr.kind = WSC_FK_MESSAGE;
    fr.mode = 2;
    fr.err = WSC_ERR_NONE;
    fr.hdr_len = (uint8_t)hl;
    fr.flags = WSC_FF_UNMASKED;
    return rec_pack(fr, seg_start, plen != 0, 0);
}

// What walk_segment returns for a segment the pre-pass walked to its end (a connection with no
// fragmented message or frame open, status OPEN: the pre-pass runs only then) -- mode 0 after a
// FIN message, msgID advanced, no text, nothing in progress.  Its LDS records hold the segment.
__device__ __forceinline__ WalkEnd pre_end(const PreState& p, uint64_t seg_start, uint32_t status) {
    WalkEnd we{};
    we.pos = seg_start + p.pos;
    we.cont = 0;
    we.last_dend = seg_start + p.pend;
    we.frem = we.flen = 0;
    we.fmask = we.fhdr = 0;
    we.msg = p.msg;
    we.mode = 0;
    we.status = status;
    we.close_code = we.err = 0;
    we.u8dfa = we.pdfa = 0;
    we.replay = true;
    return we;
}
template <bool EMIT, bool COMPACT, uint32_t LS = 64, int SPEC_D = WSC_WALK_SPEC, bool PURE = false>
__device__ __forceinline__ SegCount walk_segment(const WalkArgs& a, uint32_t s, const SegCount& base,
                                                 const SegCount& own, uint4* lrec, WalkEnd* wend,
                                                 uint4* lrec2 = nullptr, uint32_t cap = 0, uint32_t tag = 0,
                                                 const PreState* pre = nullptr, const SegIn* in = nullptr,
                                                 uint4* hc_out = nullptr) {
    // in: the segment's bounds and first 16 bytes, loaded ahead by the caller (the tiled walk);
    // hc_out: its header cache -- the counting pass stores the 16 bytes at the segment's first
    // frame (one coalesced 16 B store per lane), the emitting pass loads them from there instead
    // of re-reading a scattered wire line per segment
    const uint8_t* __restrict__ w = a.wire;
    const uint64_t seg_start = in ? in->start : a.seg_off[s];
    const uint64_t seg_end = in ? in->end : a.seg_off[s + 1];

    wsc_conn_state st = {};
    if (in) st = in->st;
    else if (a.state_in) st = a.state_in[s];
    uint64_t cont = st.cont_len;
    uint32_t msg = st.msg_id;
    uint32_t mode = st.message_mode;
    uint32_t status = st.status;
    // a data frame whose payload is still arriving (its header was in an earlier batch):
    // websocket_frame.go:16-31 -- nextFrame reads what is there into rBuffer, completes later
    uint64_t frem = st.frame_rem, flen = st.frame_len;
    uint32_t fmask = st.frame_mask, fhdr = st.frame_hdr;
    // a streamed PONG under messageMode TEXT: the DFA state of its payload so far (its own utf8.Valid,
    // websocket_frame.go:71 with Q6; the message's state u8dfa is untouched by it)
    uint32_t pdfa = st.frame_utf8;
    uint32_t close_code = 0, err_out = 0;
    uint32_t nf = 0, ns0 = 0, ns1 = 0, sflags = 0;
    uint64_t nb0 = 0, nb1 = 0;
    EmitCtx e{};
    if constexpr (EMIT) e = emit_begin<COMPACT>(a, s, seg_start, seg_end, base, own);

    // UTF-8 verdicts are decided by the counting pass (payload read on the still-masked wire) and
    // replayed by the emitting pass: u8fail = ordinal of the first frame that fails, u8dfa = DFA
    // state after the continueBuffer and the in-progress frame's bytes (carried to the next batch).
    uint32_t u8fail = 0xFFFFFFFFu;
    uint32_t u8dfa = (cont || frem) ? st.cont_utf8 : 0u;
    bool u8_pending = false;                      // a text chain has a deferred (chip-wide) part
    uint32_t u8_head = 0xFFFFFFFFu, u8_last = 0xFFFFFFFFu, u8_n = 0, u8_ncomp = 0;
    bool u8_comp = false;                         // an item whose verdict needs the segment's composition
    bool p8_open = false;                         // the segment ends inside a PONG whose piece was deferred
    uint32_t pool_next = 0, pool_end = 0;         // the segment's unused item slots
    auto dead_fill = [&](uint32_t i, uint32_t e) {
        for (; i < e; ++i)
            if (i < a.u8items_cap) {
                U8Item d{};
                d.seg = U8_DEAD;
                d.next = 0xFFFFFFFFu;
                a.u8items[i] = d;
            }
    };
    if constexpr (EMIT) {
        u8fail = a.u8info[2 * s];
        u8dfa = a.u8info[2 * s + 1] & 0xFFu;
        pdfa = a.u8info[2 * s + 1] >> 8;
    }

    uint64_t pos = seg_start;
    uint64_t pend = seg_start;   // wire end of the last payload span so far (window index, emit)

    // LDS records of the counting pass for the emit: rec_pack + the frame's position among the
    // segment's outputs (MsgID, span ordinal, arena offset in its region, previous span end)
    auto record = [&](const wsc_frame& fr, bool have_span, uint32_t region, uint64_t plen) {
        if (lrec && nf < cap) {
            uint4 r = rec_pack(fr, seg_start, have_span, region);
            r.w |= tag << 28;   // the lane's segment the frame belongs to
            lrec[nf * LS] = r;
            lrec2[nf * LS] = make_uint4(fr.msg_id, ns0 + ns1, (uint32_t)(COMPACT && region ? nb1 : nb0),
                                        (uint32_t)(pend - seg_start));
        }
        if (have_span) pend = fr.hdr_off + fr.hdr_len + plen;
    };

    // A text payload validated chip-wide (after the unmask): item slots from the segment's pool,
    // window flags for the unmask's fold, the segment's item list.  Counting pass only.
    // kind: U8K_*; PONG pieces (U8K_PONG / U8K_PONG_END) bring their own entry state p_in
    auto defer = [&](uint64_t src, uint64_t n, uint32_t mk, uint8_t kind, uint32_t p_in, uint32_t hl) {
        // large text (or a chain already deferred): validated chip-wide by k_u8_check,
        // which also applies the verdict; the walk goes on as if it were valid
        const bool part = kind == U8K_PART, chain = kind == U8K_CHAIN, pong = kind >= U8K_PONG;
        if constexpr (PURE) {   // a count without side effects: only the chain state the walk keys on
            if (part) u8_pending = true;
            if (chain) u8_pending = false;
            return;
        }
        const uint8_t s_in = pong ? (uint8_t)p_in : (part || chain) ? (u8_pending ? 0xFF : (uint8_t)u8dfa) : 0;
        // a payload up to U8_PIECE is one piece; longer ones are cut at absolute
        // U8_PIECE-aligned wire offsets.  Either way every unmask window that lies
        // inside a text payload lies inside one item (its map is folded by the unmask
        // that has just unmasked it, win_flag / win_map)
        const uint32_t pieces = n <= U8_PIECE ? 1u : (uint32_t)((src + n - 1) / U8_PIECE - src / U8_PIECE + 1);
        // Item slots come from a per-segment pool: a same-address atomic per frame sat on
        // the header chain (1 KiB TEXT: 16 of them per lane, ~3 us each), so a refill
        // takes up to 4 slots (the frames of this size the segment still holds),
        // wave-aggregated (rank = the slots of the refilling lanes below).  Unused slots
        // become dead items at the segment's end (k_u8_check skips them).
        if (pool_end - pool_next < pieces) {
            dead_fill(pool_next, pool_end);   // (only > 1 GiB frames leave slots here)
            const uint64_t more = (seg_end - (src + n)) / (hl + n + 1);
            const uint32_t want = pieces + (uint32_t)(more < 3 ? more : 3);
            const uint32_t rq = pieces > 4 ? pieces : (want < 4 ? want : 4u);
            uint32_t base;
            const uint64_t act = __ballot(true);
            if (__ballot(rq > 4) == 0) {
                const uint64_t m0 = __ballot(rq & 1), m1 = __ballot(rq & 2), m2 = __ballot(rq & 4);
                auto below = [](uint64_t m) {
                    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                };
                const uint32_t leader = (uint32_t)__builtin_ctzll(act);
                uint32_t b = 0;
                if (lane_id() == leader)
                    b = __hip_atomic_fetch_add(a.u8count,
                                               (uint32_t)(__builtin_popcountll(m0) + 2 * __builtin_popcountll(m1) +
                                                          4 * __builtin_popcountll(m2)),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                base = (uint32_t)__builtin_amdgcn_readlane((int)b, (int)leader) + below(m0) + 2 * below(m1) +
                       4 * below(m2);
            } else {
                base = __hip_atomic_fetch_add(a.u8count, rq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (base == 0 && a.u8host) {   // the first deferral tells the host the check has work
                __hip_atomic_store(a.u8host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __threadfence_system();
            }
            pool_next = base;
            pool_end = base + rq;
        }
        const uint32_t b0 = pool_next;
        pool_next += pieces;
        // capacity (wsc_create): frames + 4 x segments (pool slots) + 4 x bytes / U8_PIECE
        const uint64_t W = 1ull << a.win_shift;
        for (uint32_t p = 0; p < pieces; ++p) {
            const uint32_t idx = b0 + p;
            U8Item it;
            const uint64_t ps = p == 0 ? src : (src / U8_PIECE + p) * U8_PIECE;
            const uint64_t pe0 = pieces == 1 ? src + n : (src / U8_PIECE + p + 1) * U8_PIECE;
            const uint64_t pe = pe0 < src + n ? pe0 : src + n;
            it.src = ps;
            it.len = (uint32_t)(pe - ps);
            it.mask = rotr32(mk, 8u * (uint32_t)((ps - src) & 3));   // phase 0 at the piece
            if (a.win_flag) {   // windows inside the piece: folded by the unmask
                uint64_t wi = (ps + W - 1) >> a.win_shift;
                const uint64_t we = pe >> a.win_shift;
                for (; wi < we && (wi & 3); ++wi) a.win_flag[wi] = 1u;
                for (; wi + 4 <= we; wi += 4) *reinterpret_cast<uint4*>(a.win_flag + wi) = make_uint4(1, 1, 1, 1);
                for (; wi < we; ++wi) a.win_flag[wi] = 1u;
            }
            it.seg = s;
            it.ordinal = nf;
            it.next = 0xFFFFFFFFu;
            it.kind = kind;
            it.s_in = s_in;
            it.first = p == 0;
            it.last = p + 1 == pieces;
            if (idx < a.u8items_cap) {
                a.u8items[idx] = it;
                if (u8_last != 0xFFFFFFFFu) a.u8items[u8_last].next = idx;
                else u8_head = idx;
                u8_last = idx;
                u8_n += 1;
                if (part || chain || pong || pieces != 1) u8_ncomp += 1;   // counted by k_u8_check
            }
        }
        if (part || chain || pong || pieces != 1) u8_comp = true;
        if (part) u8_pending = true;
        if (chain) u8_pending = false;   // the message completes here
    };

    // The end of every frame record: utf8.Valid (TEXT messages, websocket_frame.go:71-73, across
    // fragments, pieces and batches; control payloads inside a TEXT message, Q6; close reasons,
    // websocket.go:170-172), then the record and the segment's counts.  `plen` = the payload
    // bytes this record covers (a streamed frame's piece).
    auto finish = [&](wsc_frame& fr, uint64_t plen, bool have_span, uint32_t region) {
        if (fr.flags & (WSC_FF_U8_PART | WSC_FF_U8_SELF | WSC_FF_U8_CHAIN | WSC_FF_U8_REASON)) {
            sflags |= SEGF_UTF8;
            if constexpr (!EMIT) {
                const bool part = (fr.flags & WSC_FF_U8_PART) != 0, chain = (fr.flags & WSC_FF_U8_CHAIN) != 0;
                const uint64_t src = fr.hdr_off + fr.hdr_len, n = plen;
                const uint32_t mk = fr.mask;
                if (fr.flags & WSC_FF_U8_REASON) {
                    // CLOSE reason, websocket.go:153-172 (<= 125 B: always checked here).  Under
                    // messageMode == TEXT nextFrame first runs utf8.Valid over the whole payload
                    // (websocket_frame.go:71-73); if that fails the error is swallowed (:156) and
                    // the stand-in reason has DataLen = fragmentLength, already zeroed by reset()
                    // (frame.go:49), so payload[2:] is NOT checked -- only the code is.
                    const bool skip = fr.mode == 1 && u8_run_masked(0, w, src, n, mk) != 0;
                    if (!skip && u8_run_masked(0, w, src + 2, n - 2, rotr32(mk, 16)) != 0) u8fail = nf;
                } else if (n > a.u8_inline_max || ((part || chain) && u8_pending)) {
                    defer(src, n, mk, part ? U8K_PART : (chain ? U8K_CHAIN : U8K_SELF), 0, fr.hdr_len);
                } else {
                    bool ok = true;
                    if (part) u8dfa = u8_run_masked(u8dfa, w, src, n, mk);
                    else if (chain) ok = u8_run_masked(u8dfa, w, src, n, mk) == 0;
                    else ok = u8_run_masked(0, w, src, n, mk) == 0;
                    if (!ok) u8fail = nf;
                }
            }
        }
        // a streamed PONG's piece under messageMode TEXT (Q6): its payload alone must be valid once
        // complete; each piece continues the PONG's own DFA (carried in frame_utf8 across batches)
        const bool pong_u8 = fr.opcode == 10 && fr.mode == 1 && (fr.kind == WSC_FK_PIECE || (fr.flags & WSC_FF_HEAD_PREV));
        if (pong_u8) {
            sflags |= SEGF_UTF8;
            if constexpr (!EMIT) {
                const bool end = fr.kind != WSC_FK_PIECE;
                const uint32_t p_in = (fr.flags & WSC_FF_HEAD_PREV) ? pdfa : 0u;   // fresh at its header
                const uint64_t src = fr.hdr_off + fr.hdr_len;
                if (plen > a.u8_inline_max) {   // chip-wide: the check composes it (and carries it if open)
                    defer(src, plen, fr.mask, end ? U8K_PONG_END : U8K_PONG, p_in, fr.hdr_len);
                    p8_open = !end;
                    pdfa = 0;
                } else {
                    pdfa = u8_run_masked(p_in, w, src, plen, fr.mask);
                    p8_open = false;
                    if (end && pdfa != 0) u8fail = nf;
                }
                if (end) pdfa = 0;
            }
        }
        if ((fr.flags & (WSC_FF_U8_PART | WSC_FF_U8_SELF | WSC_FF_U8_CHAIN | WSC_FF_U8_REASON)) || pong_u8) {
            if (nf == u8fail) {   // -> CloseCode(1007) (epoll.go:126-127); nothing after it is read
                fr.kind = WSC_FK_ERROR;
                fr.err = WSC_ERR_MUST_UTF8;
                status = WSC_SEG_ERROR; close_code = 1007; err_out = WSC_ERR_MUST_UTF8;
            }
        }
        // continueBuffer (and a streamed frame's bytes) consumed by the message
        if constexpr (!EMIT) if (fr.flags & (WSC_FF_CONT_MSG | WSC_FF_U8_CHAIN)) u8dfa = 0;
        if constexpr (COMPACT) if (region) fr.flags |= WSC_FF_CTRL_ARENA;
        if (plen > 0xFFFFFFFFull) sflags |= SEGF_LONG;

        if constexpr (EMIT) emit_frame<COMPACT>(a, e, fr, plen, have_span, region);
        else record(fr, have_span, region, plen);
        nf += 1;
        if (have_span) {
            // (control payloads: <= 125 B, but a PONG's -- and its pieces' -- have no bound)
            if (COMPACT && region) { ns1 += span_chunks(fr.hdr_off + fr.hdr_len, plen); nb1 += plen; }
            else { ns0 += span_chunks(fr.hdr_off + fr.hdr_len, plen); nb0 += plen; }
        }
    };

    // The segment starts with the rest of a streamed data frame's payload: consume what is here
    // as one piece.  The piece that completes the frame takes the frame's kind -- FIN=1: the
    // message (continueBuffer || earlier pieces || this one, websocket_frame.go:52-91); FIN=0: a
    // fragment appended to continueBuffer (:92-99) -- earlier ones are WSC_FK_PIECE.
    auto resume = [&]() {
        const uint64_t have = seg_end - pos;
        const uint64_t take = have < frem ? have : frem;
        const uint32_t op = fhdr & 0xFu, fin = fhdr >> 7;
        wsc_frame fr;
        fr.hdr_off = pos;
        fr.payload_len = (uint32_t)take;
        fr.payload_len_hi = (uint8_t)(take >> 32);
        fr.mask = fmask;
        fr.seg = s;
        fr.msg_id = msg;
        fr.opcode = (uint8_t)op;
        fr.fin = (uint8_t)fin;
        fr.mode = (uint8_t)mode;
        fr.err = 0;
        fr.hdr_len = 0;
        fr.flags = WSC_FF_UNMASKED | WSC_FF_HEAD_PREV;
        const bool text = mode == 1 && op != 10;   // (a PONG's own check: finish, Q6)
        if (take < frem) {
            fr.kind = WSC_FK_PIECE;
            if (text) fr.flags |= WSC_FF_U8_PART;
        } else if (op == 10) {   // the PONG is complete: read and discarded (websocket.go:203-205), Q5
            fr.kind = WSC_FK_PONG;
            msg += 1;
        } else if (fin) {
            fr.kind = WSC_FK_MESSAGE;
            if (op == 0 && cont >= 1) { fr.flags |= WSC_FF_CONT_MSG; cont = 0; }
            if (text) fr.flags |= WSC_FF_U8_CHAIN;   // from the state after continueBuffer + pieces
            mode = 0;
            msg += 1;
        } else {
            fr.kind = WSC_FK_FRAG;
            if (text) fr.flags |= WSC_FF_U8_PART;
            cont += flen;
        }
        frem -= take;
        fmask = rotr32(fmask, 8u * (uint32_t)(take & 3));
        finish(fr, take, take > 0, op == 10 ? 1u : 0u);   // (COMPACT: a PONG's bytes in the control region)
        pos += take;
    };

    // One frame at `pos` from its 32-byte header window; returns false when the walk stops
    // (terminal status, or the frame is incomplete and is carried to the next batch).
    auto step = [&](const uint4& hd) -> bool {
        const uint64_t avail = seg_end - pos;
        if (avail < 2) return false;
        uint32_t h[14];
        hdr_bytes(hd, h);
        const uint32_t fin = h[0] >> 7;
        const uint32_t rsv = (h[0] >> 4) & 7;
        const uint32_t op = h[0] & 0xF;
        const uint32_t masked = h[1] >> 7;
        const uint32_t len7 = h[1] & 0x7F;

        wsc_frame fr;
        fr.hdr_off = pos;
        fr.payload_len = 0;
        fr.payload_len_hi = 0;
        fr.mask = 0;
        fr.seg = s;
        fr.msg_id = msg;
        fr.opcode = (uint8_t)op;
        fr.fin = (uint8_t)fin;
        fr.kind = WSC_FK_ERROR;
        fr.mode = (uint8_t)mode;
        fr.err = 0;
        fr.hdr_len = 2;
        fr.flags = 0;

        uint64_t next = pos;
        bool have_span = false;
        uint32_t region = 0;
        uint64_t plen = 0, take = 0;   // take: payload bytes this record covers

        if (rsv) {  // websocket.go:229-231, checked as soon as the 2 bytes are in
            fr.err = WSC_ERR_RSV_FAIL;
            status = WSC_SEG_ERROR; close_code = 1002; err_out = WSC_ERR_RSV_FAIL;
            next = pos + 2;
        } else {
            const uint32_t mode_h = (op == 1 || op == 2) ? op : mode;   // :234-236
            fr.mode = (uint8_t)mode_h;
            const uint32_t ext = len7 == 126 ? 2 : (len7 == 127 ? 8 : 0);
            if (avail < 2 + ext) return false;                           // wait for the length
            if (ext == 2) plen = (h[2] << 8) | h[3];
            else if (ext == 8) {
                plen = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) plen = (plen << 8) | h[2 + k];
            } else plen = len7;
            if (!masked) {  // Q3: the reference never completes this header
                fr.kind = WSC_FK_STALL;
                fr.hdr_len = (uint8_t)(2 + ext);
                status = WSC_SEG_STALLED;
                next = pos + 2 + ext;
            } else {
                const uint32_t hl = 2 + ext + 4;
                if (avail < hl) return false;                            // wait for the mask
                uint32_t mask = 0;
                if (ext == 0) mask = h[2] | h[3] << 8 | h[4] << 16 | h[5] << 24;
                else if (ext == 2) mask = h[4] | h[5] << 8 | h[6] << 16 | h[7] << 24;
                else mask = h[10] | h[11] << 8 | h[12] << 16 | h[13] << 24;
                fr.hdr_len = (uint8_t)hl;
                fr.mask = mask;
                {   // 40-bit record length; longer is always TOO_LARGE (max_frame_len < 2^40): saturated
                    const uint64_t rl = plen < (1ull << 40) ? plen : (1ull << 40) - 1;
                    if (rl > 0xFFFFFFFFull) sflags |= SEGF_LONG;
                    fr.payload_len = (uint32_t)rl;
                    fr.payload_len_hi = (uint8_t)(rl >> 32);
                }
                const uint64_t pstart = pos + hl;

                // opcode switch, websocket.go:136-208
                uint32_t err = 0, kind = WSC_FK_ERROR;
                bool payload = false;
                if (op == 0) {
                    if (mode_h < 1) err = WSC_ERR_OPCODE_FAIL;
                    else { payload = true; kind = fin ? WSC_FK_MESSAGE : WSC_FK_FRAG; }
                } else if (op == 1 || op == 2) {
                    if (cont >= 1) err = WSC_ERR_PING_PAYLOAD_OVERSIZE;
                    else { payload = true; kind = fin ? WSC_FK_MESSAGE : WSC_FK_FRAG; }
                } else if (op == 8) {
                    if (!(plen == 0 || plen >= 2) || plen > 125) err = WSC_ERR_PROTOCOL_ERROR;
                    else if (plen == 0) kind = WSC_FK_CLOSE;
                    else { payload = true; kind = fin ? WSC_FK_CLOSE : WSC_FK_FRAG; }
                } else if (op == 9) {
                    if (fin != 1) err = WSC_ERR_CTRL_FRAGMENTED;
                    else if (plen > 125) err = WSC_ERR_PING_PAYLOAD_OVERSIZE;   // ctrl.go:130-132
                    else { payload = true; kind = WSC_FK_PING; }
                } else if (op == 10) {
                    if (fin != 1) err = WSC_ERR_CTRL_FRAGMENTED;
                    else if (plen == 0) kind = WSC_FK_PONG_EMPTY;
                    else { payload = true; kind = WSC_FK_PONG; }
                } else {
                    err = WSC_ERR_OPCODE_FAIL;
                }
                bool piece = false;   // the payload is still arriving: stream it (data frames)
                if (payload && !err) {
                    if (plen > a.max_frame_len) err = WSC_ERR_TOO_LARGE;        // Q4
                    else if (avail < hl + plen) {
                        // PING / CLOSE (<= 125 B by the rules above) wait whole; a data frame or a
                        // PONG (no size limit, websocket.go:191-205) streams: websocket_frame.go:16-31
                        if (op == 8 || op == 9) return false;
                        piece = true;
                    }
                }
                if (piece) {
                    take = avail - hl;
                    fr.payload_len = (uint32_t)take;
                    fr.payload_len_hi = (uint8_t)(take >> 32);
                } else {
                    take = plen;
                }
                next = pstart + (payload && !err ? take : 0);
                if (err) {
                    fr.err = (uint8_t)err;
                    status = WSC_SEG_ERROR; close_code = 1002; err_out = err;
                    next = pstart;
                } else if (piece) {
                    // the header is consumed (messageMode set, websocket.go:234-236); the rest of
                    // the payload is carried as state, never as bytes
                    fr.kind = WSC_FK_PIECE;
                    fr.flags |= WSC_FF_UNMASKED;
                    if (op == 10) {
                        region = 1;   // COMPACT: the control region (the payload is discarded)
                    } else {
                        if (mode_h == 1) fr.flags |= WSC_FF_U8_PART;
                        mode = mode_h;
                    }
                    frem = plen - take;
                    flen = plen;
                    fmask = rotr32(mask, 8u * (uint32_t)(take & 3));
                    fhdr = fin << 7 | op;
                    have_span = take > 0;
                } else {
                    fr.kind = (uint8_t)kind;
                    if (payload) fr.flags |= WSC_FF_UNMASKED;
                    const bool text = mode_h == 1;
                    if (kind == WSC_FK_MESSAGE) {                                // frame.go:52-91
                        const bool cmsg = (op == 0 && cont >= 1);
                        if (cmsg) { fr.flags |= WSC_FF_CONT_MSG; cont = 0; }
                        if (text) fr.flags |= cmsg ? WSC_FF_U8_CHAIN : WSC_FF_U8_SELF;
                        mode = 0;                                                // op is 0/1/2
                        msg += 1;
                    } else if (kind == WSC_FK_FRAG) {                            // frame.go:92-99
                        if (text) fr.flags |= WSC_FF_U8_PART;
                        cont += plen;
                        mode = mode_h;
                    } else if (kind == WSC_FK_PING || kind == WSC_FK_PONG) {
                        if (text) fr.flags |= WSC_FF_U8_SELF;                    // Q6
                        msg += 1;                                                // Q5
                        region = 1;
                    } else if (kind == WSC_FK_CLOSE) {                           // :153-183
                        region = 1;
                        if (payload) {
                            if (plen > 2) fr.flags |= WSC_FF_U8_REASON;
                            const uint32_t code = (((uint32_t)w[pstart] ^ (mask & 0xFF)) << 8) |
                                                  ((uint32_t)w[pstart + 1] ^ ((mask >> 8) & 0xFF));
                            if (!close_code_ok(code)) {
                                fr.kind = WSC_FK_ERROR;
                                fr.err = WSC_ERR_PROTOCOL_ERROR;
                                status = WSC_SEG_ERROR; close_code = 1002;
                                err_out = WSC_ERR_PROTOCOL_ERROR;
                            }
                        }
                        if (status == WSC_SEG_OPEN) { status = WSC_SEG_CLOSED; close_code = 1000; }
                    } else if (kind == WSC_FK_PONG_EMPTY) {
                        status = WSC_SEG_CLOSED; close_code = 1000;
                    }
                    have_span = payload && plen > 0;
                }
            }
        }

        finish(fr, take, have_span, region);
        pos = next;
        return status == WSC_SEG_OPEN;
    };

    // Fast path (both passes): a complete, masked FIN BIN frame (0x82) while no fragmented
    // message is open (cont == 0) is always Message{MsgID: msg, Opcode: 2} (websocket.go:142-146,
    // websocket_frame.go:52-91; messageMode 2 -> 0, msgID + 1): its record is written without the
    // general state machine.  So is a FIN TEXT frame (0x81) whose payload is validated chip-wide
    // (above u8_inline_max, one item): Opcode 1, its UTF-8 verdict applied later.  Everything else
    // goes through `step`.
    auto fast = [&](const uint4& hd) -> bool {
        const uint32_t b0 = hd.x & 0xFFu, b1 = (hd.x >> 8) & 0xFFu;
        if ((b0 != 0x82u && b0 != 0x81u) || !(b1 & 0x80u) || cont != 0) return false;
        const bool text = b0 == 0x81u;
        const uint32_t len7 = b1 & 0x7Fu;
        uint64_t plen;
        uint32_t mask, hl;
        if (len7 < 126) {
            plen = len7;
            mask = __builtin_amdgcn_alignbyte(hd.y, hd.x, 2);
            hl = 6;
        } else if (len7 == 126) {
            plen = ((hd.x >> 8) & 0xFF00u) | (hd.x >> 24);
            mask = hd.y;
            hl = 8;
        } else {
            const uint64_t x = (uint64_t)__builtin_amdgcn_alignbyte(hd.y, hd.x, 2) |
                               (uint64_t)__builtin_amdgcn_alignbyte(hd.z, hd.y, 2) << 32;
            plen = __builtin_bswap64(x);
            mask = __builtin_amdgcn_alignbyte(hd.w, hd.z, 2);
            hl = 14;
        }
        if (plen > a.max_frame_len || seg_end - pos < hl + plen) return false;
        // TEXT: only a whole message that is validated chip-wide (one item); small ones are
        // checked inline by `step`
        if (text && (plen <= a.u8_inline_max || plen > U8_PIECE)) return false;
        wsc_frame fr;
        fr.hdr_off = pos;
        fr.payload_len = (uint32_t)plen;
        fr.payload_len_hi = (uint8_t)(plen >> 32);
        fr.mask = mask;
        fr.seg = s;
        fr.msg_id = msg;
        fr.opcode = text ? 1 : 2;
        fr.fin = 1;
        fr.kind = WSC_FK_MESSAGE;
        fr.mode = text ? 1 : 2;
        fr.err = 0;
        fr.hdr_len = (uint8_t)hl;
        fr.flags = text ? (WSC_FF_UNMASKED | WSC_FF_U8_SELF) : WSC_FF_UNMASKED;
        if (text) {
            sflags |= SEGF_UTF8;
            if constexpr (!EMIT) defer(pos + hl, plen, mask, false, false, hl);
        }
        const bool have_span = plen > 0;
        if constexpr (EMIT) emit_frame<COMPACT>(a, e, fr, plen, have_span, 0);
        else record(fr, have_span, 0, plen);
        msg += 1;
        mode = 0;
        nf += 1;
        if (have_span) { ns0 += span_chunks(pos + hl, plen); nb0 += plen; }
        pos += hl + plen;
        return true;
    };

    uint64_t stride = 0;
    bool go = status == WSC_SEG_OPEN;
    if constexpr (!EMIT) {
        // the quad pre-pass walked (and recorded) the segment's leading plain BIN messages: continue
        // after them with the state they leave (websocket_frame.go:84-89: mode 0, msgID + 1 each)
        if (pre && pre->nf) {
            pos = seg_start + pre->pos;
            pend = seg_start + pre->pend;
            msg = pre->msg;
            mode = 0;
            nf = pre->nf;
            ns0 = pre->ns;
            nb0 = pre->nb;
            stride = pre->stride;
        }
    }
    if (go && frem && seg_end > pos) resume();   // (a rest longer than the segment: nothing else)
    go = go && status == WSC_SEG_OPEN && frem == 0;
    while (go) {
        // fewer than 2 bytes left: `step` would stop on them anyway -- no round trip for a header
        // that cannot be there (every segment's walk used to end with one)
        if (seg_end - pos < 2) break;
        // one memory round trip: the next header + SPEC_D-1 speculative ones
        uint4 hc[SPEC_D];
        uint64_t hp[SPEC_D];
#pragma unroll
        for (int k = 0; k < SPEC_D; ++k) {
            hp[k] = pos + (uint64_t)k * stride;
            hc[k] = make_uint4(0, 0, 0, 0);
            if (k == 0 && in && pos == seg_start) hc[k] = in->hdr;
            else if (k == 0 || (stride != 0 && hp[k] + 2 <= seg_end)) hc[k] = hdr_load(w, a.n_bytes, hp[k], a.hdr_nt);
            else hp[k] = ~0ull;
        }
        if (hc_out && pos == seg_start) hc_out[s] = hc[0];
        // consume the round's headers in order from the front of the queue; one copy of `step`
        // in the code (an unrolled consumer made the walk ~20k instructions: instruction-cache bound)
#pragma unroll 1
        for (int k = 0; k < SPEC_D; ++k) {
            if (!go || hp[0] != pos) break;   // speculation ran out or missed: next round trip
            const uint64_t p0 = pos;
            if (!fast(hc[0])) go = step(hc[0]);
            stride = pos - p0;
#pragma unroll
            for (int q = 0; q + 1 < SPEC_D; ++q) {
                hc[q] = hc[q + 1];
                hp[q] = hp[q + 1];
            }
            hp[SPEC_D - 1] = ~0ull;
        }
    }

    if constexpr (!EMIT) dead_fill(pool_next, pool_end);
    SegCount c;
    bool replay = false;
    c.frames = nf; c.spans0 = ns0; c.spans1 = ns1; c.flags = sflags;
    c.bytes0 = nb0; c.bytes1 = nb1;
    if constexpr (!EMIT) {
        // the LDS records replay the segment only if all fit and every offset / length fits 32 bits
        replay = lrec && nf <= cap && seg_end - seg_start <= 0xFFFFFFFFull && !(sflags & SEGF_LONG);
        if (!replay && !PURE) {   // only a re-walking emit pass reads them back
            a.u8info[2 * s] = u8fail;
            a.u8info[2 * s + 1] = u8dfa | pdfa << 8;
        }
        if (u8_n) {
            U8Seg g{};
            g.head = u8_head;
            g.n = u8_ncomp;   // the composite items (single-piece messages are never counted)
            g.done = 0;
            g.pending_end = (u8_pending ? 1u : 0u) | (u8_comp ? 2u : 0u) | (p8_open && frem ? 4u : 0u);
            g.minfail = 0xFFFFFFFFu;
            a.u8seg[s] = g;
            c.flags |= SEGF_U8DEFER;
        }
    }
    WalkEnd we;
    we.pos = pos; we.cont = cont; we.msg = msg; we.mode = mode; we.status = status;
    we.close_code = close_code; we.err = err_out; we.u8dfa = u8dfa; we.pdfa = pdfa;
    we.frem = status == WSC_SEG_OPEN ? frem : 0;
    we.flen = flen; we.fmask = fmask; we.fhdr = fhdr;
    we.last_dend = pend;
    we.replay = replay;
    if (wend) *wend = we;
    if constexpr (EMIT) emit_end<COMPACT>(a, e, we);
    return c;
}

// ---------------------------------------------------------------------------------------------
// Fused walk: count -> block scan -> decoupled look-back across blocks -> emit, one launch.
// Block ids come from a ticket counter in dispatch order, so every block a block waits for has
// already started.  Look-back hand-off (MI355X_MICROARCH.md "Valid forms", row 1): one lane per
// block stores its aggregate / inclusive prefix with agent-scope (sc1, write-through) stores,
// drains them with s_waitcnt vmcnt(0), then publishes the flag with an agent-scope atomic; the
// reader polls the flag and reads the payload with agent-scope atomic RMWs (fetch_add 0), which
// are coherent across XCDs.  Spins are bounded; flags and the ticket are zeroed by k_unmask
// (the next launch on the stream) of every decode, and at context creation.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ SegCount sc_add(const SegCount& x, const SegCount& y) { return SegCountAdd()(x, y); }

__device__ __forceinline__ SegCount sc_shfl_up(const SegCount& v, int d) {
    SegCount o;
    o.frames = __shfl_up(v.frames, d);
    o.spans0 = __shfl_up(v.spans0, d);
    o.spans1 = __shfl_up(v.spans1, d);
    o.flags = __shfl_up(v.flags, d);
    o.bytes0 = __shfl_up(v.bytes0, d);
    o.bytes1 = __shfl_up(v.bytes1, d);
    return o;
}

// Look-back record of a block: 8 words, each (kind << 32 | one 32-bit field of its SegCount), kind
// 1 = the block's aggregate, 2 = its inclusive prefix, 0 = nothing yet (k_unmask re-arms them).
// Every word is one 8-byte agent-scope (sc1, write-through) store by its own lane and tells by
// itself what it holds, so a reader needs no flag: ONE round of eight 8-byte sc1 loads per
// predecessor gets both the status and the value, and a record read half-way through its
// rewrite (aggregate words mixed with inclusive ones, or not all written) reads as not ready
// (MI355X_MICROARCH.md: self-describing granules need no ordering).  Round 5 polled a flag and
// then read the payload with atomic RMWs: two dependent round trips per look-back round.
__device__ __forceinline__ uint32_t sc_word(const SegCount& v, uint32_t k) {
    switch (k) {
    case 0: return v.frames;
    case 1: return v.spans0;
    case 2: return v.spans1;
    case 3: return v.flags;
    case 4: return (uint32_t)v.bytes0;
    case 5: return (uint32_t)(v.bytes0 >> 32);
    case 6: return (uint32_t)v.bytes1;
    default: return (uint32_t)(v.bytes1 >> 32);
    }
}
// lanes 0..7 of the wave each store one word
__device__ __forceinline__ void lb_publish(uint64_t* rec, const SegCount& v, uint32_t kind, uint32_t wl) {
    if (wl < 8) __hip_atomic_store(rec + wl, (uint64_t)kind << 32 | sc_word(v, wl), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one lane reads a whole record: its kind (0 = not ready) and value
__device__ __forceinline__ uint32_t lb_read(const uint64_t* rec, SegCount& v) {
    uint64_t w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = __hip_atomic_load(rec + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t kind = (uint32_t)(w[0] >> 32);
    bool same = true;
#pragma unroll
    for (int k = 1; k < 8; ++k) same = same && (uint32_t)(w[k] >> 32) == kind;
    v.frames = (uint32_t)w[0];
    v.spans0 = (uint32_t)w[1];
    v.spans1 = (uint32_t)w[2];
    v.flags = (uint32_t)w[3];
    v.bytes0 = (uint64_t)(uint32_t)w[4] | (uint64_t)(uint32_t)w[5] << 32;
    v.bytes1 = (uint64_t)(uint32_t)w[6] | (uint64_t)(uint32_t)w[7] << 32;
    return same ? kind : 0u;
}

// ---------------------------------------------------------------------------------------------
// Quad pre-pass of the fused walk (one segment per 4 lanes, every wave of the block).  The serial
// walk spends its time on the header chain: one lane walks its segment's frames one after another,
// each a dependent memory round trip plus the state machine's instructions on one wave per SIMD
// (the configs[2] walk waits 85 % of its cycles).  Most frames are plain complete BIN messages
// (0x82, masked, no fragmented message open: websocket.go:142-146 then websocket_frame.go:52-91 --
// Message{MsgID: msg, Opcode: 2}, messageMode 0, msgID + 1), so a quad speculates: its 16
// candidates (4 per lane) sit at pos + k * stride, stride = the size of the last frame found, all
// loaded in ONE round trip and parsed in parallel; the leading run of candidates that are plain BIN
// messages of exactly that size are real frames -- plus the first one that breaks the stride, if
// it is one.  Their LDS records (the serial walk's format) are written at once, with MsgIDs, span
// ordinals and arena offsets from quad prefix sums.  The run stops at the first frame that is not a
// plain BIN message (or is incomplete, or at the record capacity); the serial walk then continues
// from there with the state the run leaves.  Results never depend on the guess: a candidate is used
// only when the previous real frame ends exactly at it.
// ---------------------------------------------------------------------------------------------
// broadcast lane K of each quad to the quad's 4 lanes (DPP quad_perm: a VALU op, no LDS round trip)
template <int K>
__device__ __forceinline__ uint32_t qb(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K * 0x55, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t qb_dyn(uint32_t v, uint32_t k) {   // k quad-uniform
    const uint32_t v0 = qb<0>(v), v1 = qb<1>(v), v2 = qb<2>(v), v3 = qb<3>(v);
    return k == 0 ? v0 : k == 1 ? v1 : k == 2 ? v2 : v3;
}

template <uint32_t LS>
__device__ __forceinline__ void quad_prefix(const WalkArgs& a, uint32_t s, uint32_t q, uint32_t stride_hint,
                                            uint4* lrec, uint4* lrec2, PreState* out, uint32_t cap) {
    const uint8_t* __restrict__ w = a.wire;
    bool ok = s < a.n_segs;
    uint64_t seg_start = 0, seg_end = 0;
    uint32_t msg = 0;
    if (ok) {
        seg_start = a.seg_off[s];
        seg_end = a.seg_off[s + 1];
        if (a.state_in) {
            const wsc_conn_state st = a.state_in[s];
            ok = st.status == WSC_SEG_OPEN && st.cont_len == 0 && st.frame_rem == 0;
            msg = st.msg_id;
        }
        ok = ok && seg_end - seg_start <= 0xFFFFFFFFull;
    }
    uint64_t pos = seg_start, pend = seg_start;
    // the first round speculates with the stride the previous decode on this context ended with (a
    // hint only: any value is safe); later rounds keep the stride that linked, so a single frame of
    // another size (a 64 KiB frame among 125 B ones) costs one round, not two
    uint32_t stride = stride_hint, nf = 0, ns = 0, nb = 0;
    bool first = true;
    bool go = ok && seg_end - pos >= 2 && cap > 0;
    while (go) {
        // one round trip: candidates 4q .. 4q+3 (candidate 0 is the real next frame)
        uint4 hd[4];
        uint64_t hp[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t idx = 4 * q + j;
            hp[j] = pos + (uint64_t)idx * stride;
            const bool ld = idx == 0 || (stride != 0 && hp[j] + 2 <= seg_end);
            hd[j] = ld ? hdr_load(w, a.n_bytes, hp[j], a.hdr_nt) : make_uint4(0, 0, 0, 0);
            if (!ld) hp[j] = ~0ull;
        }
        uint32_t fbits = 0, lbits = 0;
        uint32_t sz[4], pl[4], hlj[4], mk[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t b0 = hd[j].x & 0xFFu, b1 = (hd[j].x >> 8) & 0xFFu, len7 = b1 & 0x7Fu;
            uint64_t plen;
            uint32_t mask, hl;
            if (len7 < 126) {
                plen = len7;
                mask = __builtin_amdgcn_alignbyte(hd[j].y, hd[j].x, 2);
                hl = 6;
            } else if (len7 == 126) {
                plen = ((hd[j].x >> 8) & 0xFF00u) | (hd[j].x >> 24);
                mask = hd[j].y;
                hl = 8;
            } else {
                const uint64_t x = (uint64_t)__builtin_amdgcn_alignbyte(hd[j].y, hd[j].x, 2) |
                                   (uint64_t)__builtin_amdgcn_alignbyte(hd[j].z, hd[j].y, 2) << 32;
                plen = __builtin_bswap64(x);
                mask = __builtin_amdgcn_alignbyte(hd[j].w, hd[j].z, 2);
                hl = 14;
            }
            // a plain complete BIN message (the serial walk's `fast` path, binary case)
            const bool f = hp[j] != ~0ull && b0 == 0x82u && (b1 & 0x80u) && plen <= a.max_frame_len &&
                           hp[j] + hl + plen <= seg_end;
            sz[j] = f ? hl + (uint32_t)plen : 0u;   // (the segment is < 4 GiB)
            pl[j] = f ? (uint32_t)plen : 0u;
            hlj[j] = hl;
            mk[j] = mask;
            fbits |= (f ? 1u : 0u) << j;
            lbits |= (f && sz[j] == stride ? 1u : 0u) << j;
        }
        const uint32_t F16 = qb<0>(fbits) | qb<1>(fbits) << 4 | qb<2>(fbits) << 8 | qb<3>(fbits) << 12;
        const uint32_t L16 = qb<0>(lbits) | qb<1>(lbits) << 4 | qb<2>(lbits) << 8 | qb<3>(lbits) << 12;
        const uint32_t lead = (uint32_t)__builtin_ctz(~L16 | 0x10000u);   // linked candidates in front
        uint32_t r;
        bool stop;
        if (lead >= 16) {
            r = 16;
            stop = false;
        } else {
            const bool fl = (F16 >> lead) & 1u;   // the candidate at `lead` is real: taken if plain
            r = fl ? lead + 1 : lead;
            stop = !fl;
        }
        if (nf + r > cap) {   // LDS records of this segment: the serial walk counts the rest
            r = cap - nf;
            stop = true;
        }
        if (r == 0) break;
        // exclusive prefix over the taken candidates: spans, payload bytes, last span end
        uint32_t cnt = 0, bytes = 0;
        uint64_t lend = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (4 * q + j < r && pl[j]) { cnt += 1; bytes += pl[j]; lend = hp[j] + sz[j]; }
        const uint32_t lend_lo = (uint32_t)lend, lend_hi = (uint32_t)(lend >> 32);
        const uint32_t c4[4] = {qb<0>(cnt), qb<1>(cnt), qb<2>(cnt), qb<3>(cnt)};
        const uint32_t b4[4] = {qb<0>(bytes), qb<1>(bytes), qb<2>(bytes), qb<3>(bytes)};
        const uint64_t e4[4] = {(uint64_t)qb<0>(lend_hi) << 32 | qb<0>(lend_lo), (uint64_t)qb<1>(lend_hi) << 32 | qb<1>(lend_lo),
                                (uint64_t)qb<2>(lend_hi) << 32 | qb<2>(lend_lo), (uint64_t)qb<3>(lend_hi) << 32 | qb<3>(lend_lo)};
        uint32_t cnt_x = 0, bytes_x = 0;
        uint64_t lend_x = pend, lend_t = pend;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            if (k < q) {
                cnt_x += c4[k];
                bytes_x += b4[k];
                if (e4[k] > lend_x) lend_x = e4[k];
            }
            if (e4[k] > lend_t) lend_t = e4[k];
        }
        const uint32_t cnt_t = c4[0] + c4[1] + c4[2] + c4[3], bytes_t = b4[0] + b4[1] + b4[2] + b4[3];
        // the records, in the serial walk's LDS format (rec_pack / record)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t idx = 4 * q + j;
            if (idx < r) {
                lrec[(nf + idx) * LS] = pre_record(hp[j], pl[j], mk[j], hlj[j], seg_start);
                lrec2[(nf + idx) * LS] = make_uint4(msg + idx, ns + cnt_x, nb + bytes_x, (uint32_t)(lend_x - seg_start));
                if (pl[j]) {
                    cnt_x += 1;
                    bytes_x += pl[j];
                    lend_x = hp[j] + sz[j];
                }
            }
        }
        // the quad's state after the run: the last taken candidate's end and size
        const uint32_t last = r - 1, lj = last & 3;
        const uint32_t lsz = qb_dyn(lj == 0 ? sz[0] : lj == 1 ? sz[1] : lj == 2 ? sz[2] : sz[3], last >> 2);
        pos = pos + (uint64_t)last * stride + lsz;
        // a run that linked keeps its stride (the frame that broke it, taken, is a one-off); one that
        // linked nothing -- a stale hint, or the first frame of another size -- follows that frame
        if (lead == 0) stride = lsz;
        first = false;
        msg += r;
        nf += r;
        ns += cnt_t;
        nb += bytes_t;
        pend = lend_t;
        go = !stop && nf < cap && seg_end - pos >= 2;
    }
    (void)first;
    if (q == 0 && s < a.n_segs) {
        PreState p;
        p.nf = ok ? nf : 0;
        p.ns = ns;
        p.nb = nb;
        p.pos = (uint32_t)(pos - seg_start);
        p.pend = (uint32_t)(pend - seg_start);
        p.msg = msg;
        p.stride = stride;
        p.full = ok && nf > 0 && seg_end - pos < 2;   // nothing left for the serial walk
        *out = p;
    }
}

// LDS of one tile of the walk: NT lanes of which the first WL walk segments (G consecutive
// segments per walking lane), KR frame records per walking lane; every lane emits
template <bool COMPACT, uint32_t KR, uint32_t NT, uint32_t G, uint32_t WL = NT>
struct WalkLds {
    static_assert(WL % 16 == 0 && WL <= NT && WL <= 256, "walking lanes: whole 16-lane rows, owner is a byte");
    SegCount prefix;
    SegCount wave[NT / 64];
    uint32_t wtot[NT / 64];
    uint4 rec[KR * WL];      // [record][lane]: conflict-free 16 B per lane
    uint4 rec2[KR * WL];     // the frame's MsgID / span ordinal / arena offset / previous span end
    uint8_t owner[KR * WL];  // flat replayed frame -> its lane
    uint32_t rpre[WL];       // lane's first flat replayed frame
    uint32_t nbig;           // long spans whose window index the wave writes
    uint4 big[64];
    // per segment, [segment of the lane][lane]: start, global frame / span (/ arena) bases, counts,
    // consumed bytes + terminal status, wire end of its last span, replayed from LDS or not
    uint64_t sstart[G * WL], ldend[G * WL];
    uint32_t fbase[G * WL], sbase[G * WL], nf[G * WL], ns[G * WL];
    uint32_t cons[G * WL], endst[G * WL];
    uint64_t abase[COMPACT ? G * WL : 1], ob0[COMPACT ? G * WL : 1];
    uint8_t rep[G * WL], r0[G * WL];   // (r0: the segment's first record in the lane's list)
    PreState pre[(G == 1 && NT == 4 * WL) ? WL : 1];   // quad pre-pass results (one quad per segment)
};

// Count phase of a tile: each lane walks its G segments (first one s0; segments from seg_lim on
// are not the tile's), keeping up to KR frame records in LDS; writes the connections' carried
// state.  Returns the lane's total (lanes from WL on walk nothing).
template <bool COMPACT, uint32_t KR, uint32_t NT, uint32_t G, uint32_t WL>
__device__ __forceinline__ SegCount tile_count(const WalkArgs& a, WalkLds<COMPACT, KR, NT, G, WL>& L, uint32_t s0,
                                               uint32_t seg_lim, uint32_t lane, uint32_t& nrec, bool pre = false,
                                               const SegIn* in = nullptr) {
    const SegCount zero = {};
    SegCount tot = zero;
    nrec = 0;
    if (lane >= WL) return tot;
    for (uint32_t j = 0; j < G; ++j) {
        const uint32_t s = s0 + j;
        const uint32_t q = j * WL + lane;
        if (s >= seg_lim) {
            L.nf[q] = L.ns[q] = 0;
            L.rep[q] = 0;
            L.sstart[q] = ~0ull;
            continue;
        }
        WalkEnd we;
        const uint32_t cap = KR - nrec;
        const PreState* ps = pre && j == 0 ? L.pre + (lane < WL ? lane : 0) : nullptr;
        const SegIn* sin = j == 0 ? in : nullptr;
        const uint64_t ss = sin ? sin->start : a.seg_off[s];
        SegCount c;
        if (ps && ps->full && ps->nf) {
            // the quad pre-pass walked the whole segment (plain BIN messages from a connection with
            // no fragmented message or frame open): its end state, without a serial walk -- what
            // walk_segment would return after those frames (mode 0, msgID advanced, no text)
            const wsc_conn_state st0 = a.state_in ? a.state_in[s] : wsc_conn_state{};
            c = zero;
            c.frames = ps->nf;
            c.spans0 = ps->ns;
            c.bytes0 = ps->nb;
            we = pre_end(*ps, ss, st0.status);   // (nf <= cap and the segment is < 4 GiB)
        } else {
            c = walk_segment<false, COMPACT, WL>(a, s, zero, zero, L.rec + nrec * WL + lane, &we,
                                                 L.rec2 + nrec * WL + lane, cap, j, ps, sin);
        }
        const bool rep = we.replay;
        L.r0[q] = (uint8_t)nrec;
        if (rep) nrec += c.frames;
        L.rep[q] = rep ? 1 : 0;
        L.sstart[q] = ss;
        L.ldend[q] = we.last_dend;
        L.nf[q] = c.frames;
        L.ns[q] = c.spans0 + c.spans1;
        L.cons[q] = (uint32_t)(we.pos - ss);
        L.endst[q] = we.status | we.err << 4 | we.close_code << 8;
        L.fbase[q] = c.flags;   // (the flags until the bases are known)
        if constexpr (COMPACT) {
            L.abase[q] = c.bytes0 + c.bytes1;
            L.ob0[q] = c.bytes0;
        }
        a.state_out[s] = end_state(we);   // the connection's carried state
        tot = sc_add(tot, c);
    }
    return tot;
}

// Block-wide exclusive scan of the lanes' totals (64-lane shuffles, then across the waves); also
// the block's total.  Ends with a __syncthreads.
template <uint32_t NT, typename LDS>
__device__ __forceinline__ SegCount tile_scan(const SegCount& tot, LDS& L, uint32_t wl, uint32_t wave, SegCount& btot) {
    const SegCount zero = {};
    SegCount inc = tot;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const SegCount o = sc_shfl_up(inc, d);
        if (wl >= (uint32_t)d) inc = sc_add(o, inc);
    }
    SegCount excl = sc_shfl_up(inc, 1);
    if (wl == 0) excl = zero;
    if (wl == 63) L.wave[wave] = inc;
    __syncthreads();
    btot = zero;
#pragma unroll
    for (uint32_t w = 0; w < NT / 64; ++w) {
        if (w < wave) excl = sc_add(excl, L.wave[w]);
        btot = sc_add(btot, L.wave[w]);
    }
    return excl;
}

// Decoupled look-back by one wave (64 predecessors examined per round): publishes block bid's
// total, returns the sum of every earlier block's total.  Records: lb_publish / lb_read above.
__device__ __forceinline__ SegCount block_lookback(const WalkArgs& a, uint32_t bid, const SegCount& btot, uint32_t wl) {
    const SegCount zero = {};
    uint64_t* rec = a.lb_rec;      // [block][8]
    lb_publish(rec + 8ull * bid, btot, bid == 0 ? 2u : 1u, wl);
    SegCount prefix = zero;
    int64_t j0 = (int64_t)bid - 1;
    uint32_t spins = 0;
    while (j0 >= 0) {
        const int64_t j = j0 - (int64_t)wl;
        SegCount v = zero;
        const uint32_t f = j >= 0 ? lb_read(rec + 8ull * j, v) : 2u;   // before block 0: an inclusive prefix of zero
        const uint64_t m2 = __ballot(f == 2);
        const uint64_t m0 = __ballot(f == 0);
        const uint32_t first2 = m2 ? (uint32_t)__builtin_ctzll(m2) : 64u;
        const uint64_t need = first2 >= 63 ? ~0ull : ((2ull << first2) - 1);   // wls 0..first2
        if (m0 & need) {   // a predecessor in range has not published yet: poll again
            if (++spins > (1u << 22)) {   // bounded: never hang the device
                if (wl == 0) __hip_atomic_fetch_or(a.lb_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        if (!(wl <= first2 && j >= 0)) v = zero;   // lanes past the first inclusive prefix
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            SegCount o;
            o.frames = __shfl_xor(v.frames, d);
            o.spans0 = __shfl_xor(v.spans0, d);
            o.spans1 = __shfl_xor(v.spans1, d);
            o.flags = __shfl_xor(v.flags, d);
            o.bytes0 = __shfl_xor(v.bytes0, d);
            o.bytes1 = __shfl_xor(v.bytes1, d);
            v = sc_add(v, o);
        }
        prefix = sc_add(prefix, v);
        if (first2 < 64) break;
        j0 -= 64;
    }
    if (bid != 0) lb_publish(rec + 8ull * bid, sc_add(prefix, btot), 2u, wl);
    return prefix;
}

// Emit phase of a tile, once the lane's first output position `lb` is known (the tile's prefix +
// the lane's exclusive scan): per segment bases, then every frame held in LDS emitted
// cooperatively in flat order (consecutive records, spans and arena offsets in memory, so each
// store instruction covers contiguous bytes), then the per segment results; segments whose frames
// did not fit re-walk their (cache-warm) headers to emit.  Walking lane o's first segment is
// seg0 + o * G; lanes from WL on only take part in the cooperative emit.
template <bool COMPACT, uint32_t KR, uint32_t NT, uint32_t G, uint32_t WL>
__device__ __forceinline__ void tile_emit(const WalkArgs& a, WalkLds<COMPACT, KR, NT, G, WL>& L, const SegCount& lb,
                                          uint32_t nrec, uint32_t seg0, uint32_t seg_lim, uint32_t lane,
                                          uint32_t col = ~0u) {
    constexpr uint32_t NW = NT / 64;
    const uint32_t wl = lane & 63, wave = lane >> 6;
    if (col == ~0u) col = lane;   // the walking lane's column (its segments, LDS records); physical lane by default
    const uint32_t s0 = seg0 + col * G;
    const bool walker = col < WL;
    const SegCount zero = {};
    // ---- per segment bases ----
    if (walker) {
        uint32_t fb = lb.frames, sb = lb.spans0 + lb.spans1;
        uint64_t ab = lb.bytes0 + lb.bytes1;
        for (uint32_t j = 0; j < G; ++j) {
            const uint32_t q = j * WL + col;
            const uint32_t s = s0 + j;
            const uint32_t fl = L.fbase[q];
            if (s < seg_lim && (fl & SEGF_U8DEFER)) {
                a.u8seg[s].sbase = sb;
                a.u8seg[s].nspans = L.ns[q];
                a.u8seg[s].fbase = fb;
            }
            L.fbase[q] = fb;
            L.sbase[q] = sb;
            fb += L.nf[q];
            sb += L.ns[q];
            if constexpr (COMPACT) {
                const uint64_t n = L.abase[q];
                L.abase[q] = ab;
                ab += n;
            }
        }
    }
    // ---- flat order of the frames held in LDS ----
    uint32_t rv = nrec;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(rv, d);
        if (wl >= (uint32_t)d) rv += o;
    }
    if (wl == 63) L.wtot[wave] = rv;
    if (lane == 0) L.nbig = 0;
    __syncthreads();
    uint32_t rpre = rv - nrec, F = 0;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) {
        if (w < wave) rpre += L.wtot[w];
        F += L.wtot[w];
    }
    if (walker) L.rpre[col] = rpre;
    for (uint32_t k = 0; k < nrec; ++k) L.owner[rpre + k] = (uint8_t)col;
    __syncthreads();
    // ---- cooperative emit ----
    const uint32_t W = 1u << a.win_shift;
    for (uint32_t f = lane; f < F; f += NT) {
        const uint32_t o = L.owner[f];
        const uint32_t k = f - L.rpre[o];
        const uint4 r = L.rec[k * WL + o];
        const uint4 q = L.rec2[k * WL + o];
        const uint32_t j = r.w >> 28;
        const uint32_t qi = j * WL + o;
        const uint64_t ss = L.sstart[qi];
        const uint32_t hl = (r.w >> 14) & 15, fl = (r.w >> 18) & 0xFF, region = (r.w >> 26) & 1;
        const bool have_span = (r.w >> 27) & 1;
        const uint64_t hdr_off = ss + r.x;
        uint64_t dst = ~0ull;
        if constexpr (COMPACT)
            if (fl & WSC_FF_UNMASKED) dst = L.abase[qi] + (region ? L.ob0[qi] : 0ull) + q.z;
        const uint32_t fidx = L.fbase[qi] + (k - L.r0[qi]);   // the segment's first frame + ordinal
        if (fidx < a.frames_cap) {
            const uint4 r0 = make_uint4((uint32_t)hdr_off, (uint32_t)(hdr_off >> 32), r.y, r.z);
            const uint4 r1 = make_uint4(seg0 + o * G + j, q.x,
                                        (r.w & 0xF) | ((r.w >> 4) & 1) << 8 | ((r.w >> 5) & 15) << 16 |
                                            ((r.w >> 9) & 3) << 24,
                                        ((r.w >> 11) & 7) | hl << 8 | fl << 16);
            reinterpret_cast<uint4*>(a.frames + fidx)[0] = r0;
            reinterpret_cast<uint4*>(a.frames + fidx)[1] = r1;
            if constexpr (COMPACT) a.frame_dst[fidx] = dst;
        }
        if (have_span) {
            const uint32_t idx = L.sbase[qi] + q.y;
            Span sp;
            sp.src = hdr_off + hl;
            sp.len = r.y;
            sp.dst = COMPACT ? dst : sp.src;
            sp.key = rotr32(r.z, 8u * ((uint32_t)(0u - (uint32_t)sp.src) & 3u));
            if (idx < a.spans_cap) a.spans[idx] = sp;
            // windows starting in [previous span end, this span end) look this span up first
            uint64_t t = (ss + q.w + W - 1) >> a.win_shift;
            const uint64_t t_end = ((sp.src + r.y - 1) >> a.win_shift) + 1;
            if (t_end > t + 64) {   // a long span: its windows are written by the whole wave below
                const uint32_t jb = atomicAdd(&L.nbig, 1u);
                if (jb < 64) {
                    L.big[jb] = make_uint4((uint32_t)t, (uint32_t)(t >> 32), (uint32_t)(t_end - t), idx);
                    t = t_end;
                }
            }
            for (; t < t_end && (t & 3); ++t) a.tile_first[t] = idx;
            const uint4 q4 = make_uint4(idx, idx, idx, idx);
            for (; t + 4 <= t_end; t += 4) *reinterpret_cast<uint4*>(a.tile_first + t) = q4;
            for (; t < t_end; ++t) a.tile_first[t] = idx;
        }
    }
    __syncthreads();
    {
        const uint32_t nbig = L.nbig < 64 ? L.nbig : 64;
        for (uint32_t jb = wave; jb < nbig; jb += NW) {   // one wave per long span
            const uint64_t tb = L.big[jb].x | (uint64_t)L.big[jb].y << 32;
            const uint32_t nw = L.big[jb].z, idx = L.big[jb].w;
            for (uint32_t i = wl; i < nw; i += 64) a.tile_first[tb + i] = idx;
        }
    }
    // ---- per segment results; segments not held in LDS re-walk their (cache-warm) headers ----
    for (uint32_t j = 0; j < G && walker; ++j) {
        const uint32_t s = s0 + j;
        if (s >= seg_lim) break;
        const uint32_t q = j * WL + col;
        const uint64_t se = a.seg_off[s + 1];
        if (L.rep[q]) {
            const uint64_t Wd = W;   // windows that start after the last span, up to the segment end
            const uint32_t nx = L.sbase[q] + L.ns[q];
            for (uint64_t x = (L.ldend[q] + Wd - 1) & ~(Wd - 1); x < se; x += Wd) a.tile_first[x >> a.win_shift] = nx;
            wsc_seg_result r;
            r.consumed = L.cons[q];
            r.frame_begin = L.fbase[q];
            r.frame_count = L.nf[q];
            r.status = L.endst[q] & 0xF;
            r.close_code = L.endst[q] >> 8;
            r.err = (L.endst[q] >> 4) & 0xF;
            r.pad = 0;
            a.seg_out[s] = r;
        } else {
            SegCount base = zero, own = zero;
            base.frames = L.fbase[q];
            base.spans0 = L.sbase[q];
            own.frames = L.nf[q];
            if constexpr (COMPACT) {
                base.bytes0 = L.abase[q];
                own.bytes0 = L.ob0[q];
            }
            walk_segment<true, COMPACT, NT>(a, s, base, own, nullptr, nullptr);
        }
    }
}

// The batch summary, by the block holding the last segments: totals `tt` of the whole batch.
template <bool COMPACT>
__device__ __forceinline__ void write_summary(const WalkArgs& a, const SegCount& tt) {
    wsc_summary sm;
    sm.data_bytes = COMPACT ? tt.bytes0 : 0;
    sm.ctrl_bytes = COMPACT ? tt.bytes1 : 0;
    sm.n_frames = tt.frames;
    // spans past the capacity were never written: the unmask must not read them (an overflowed
    // batch unmasks the spans that fit; n_spans = spans unmasked)
    sm.n_spans = tt.spans0 + tt.spans1 < a.spans_cap ? tt.spans0 + tt.spans1 : a.spans_cap;
    sm.overflow = (tt.frames > a.frames_cap || tt.spans0 + tt.spans1 > a.spans_cap) ? 1u : 0u;
    if (__hip_atomic_load(a.lb_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) sm.overflow |= 2u;
    sm.pad = 0;
    *a.summary = sm;
    if (sm.overflow) __hip_atomic_fetch_or(a.sticky, sm.overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The fused walk kernel: NT lanes (64 or 256) per block, the first WL of them walk G consecutive
// segments each, KR frame records per walking lane in LDS.  The host picks the geometry so that
// the blocks fill the CUs once (the count phase wants every CU; the look-back wants few blocks).
// WL < NT (64 walking lanes in a 256-lane block): one wave per CU walks -- the chain of headers of
// a segment is serial whatever the wave count -- and all four emit, so the emit's stores issue
// from every SIMD (configs[2]: 64 segments per CU, the emit was 10 us on one wave).  Phases: count (each lane walks its
// segments; records in LDS) -> block scan -> decoupled look-back -> cooperative emit.  Block ids
// come from a ticket counter in dispatch order, so every block a block waits for has already
// started.  Flags and the ticket are zeroed by k_unmask (the next launch on the stream) of every
// decode, and at context creation.
// SPREAD (> 0): the WL walking columns are spread SPREAD per wave over WL / SPREAD waves, so several
// SIMDs issue the header chains (same blocks, same look-back as SPREAD = 0).
// A walk block's position in the look-back order: a ticket in start order, so every block a block
// waits on has started (the hardware workgroup index, without the ticket atomic, measured slower:
// profiles/r04_walk_hw_order_ab.log).  The look-back's bounded spin backs it.
__device__ __forceinline__ uint32_t walk_block_id(const WalkArgs& a) {
    return __hip_atomic_fetch_add(a.lb_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool COMPACT, uint32_t KR, uint32_t NT, uint32_t G, uint32_t WL, uint32_t SPREAD>
__global__ __launch_bounds__(NT) void k_walk_fused(WalkArgs a) {
    static_assert(SPREAD == 0 || (WL % SPREAD == 0 && WL / SPREAD <= NT / 64 && SPREAD <= 64), "spread geometry");
    __shared__ uint32_t sh_bid;
    __shared__ WalkLds<COMPACT, KR, NT, G, WL> L;
    const uint32_t lane = threadIdx.x, wl = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __builtin_amdgcn_s_setprio(3);   // a latency-bound chain beside streaming unmask waves (neutral, round 5)
    if (lane == 0) sh_bid = walk_block_id(a);
    __syncthreads();
    const uint32_t bid = sh_bid;
    const uint32_t n_blocks = (a.n_segs + WL * G - 1) / (WL * G);
    uint64_t t0 = 0, t1 = 0, t2 = 0;
    if (a.dbg && lane == 0) t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t nrec;
    // quad pre-pass (one segment per 4 lanes, all waves): the leading plain BIN messages of each
    // segment, recorded in LDS; the walking lane continues after them
    // Only where the block has a quad per walking lane (one walking wave in four: modes 65, 16).
    // With more walking lanes than quads (modes 64, 256) the quads would take the segments NT / 4
    // at a time, one pass after another: measured slower there (the pipelined configs[2] walk on
    // 16 CUs: 0.0618 -> 0.0648 ms per batch) or neutral (configs[1] 16 frames/segment).
    // (The pass loop below also serves PASSES > 1; a pass finding no plain BIN message at all --
    // fragmented or text traffic -- skips the rest.)
    constexpr bool PRE = G == 1 && SPREAD == 0 && NT == 4 * WL;
    if constexpr (PRE) {
        constexpr uint32_t NQ = NT / 4, PASSES = WL / NQ;
        __shared__ uint32_t sh_found;
        if (lane == 0) sh_found = 0;
        if (lane < WL) {   // (segments no pass reaches -- skipped passes -- keep these)
            L.pre[lane].nf = 0;
            L.pre[lane].full = false;
        }
        __syncthreads();
        if (a.quad_pre) {
            const uint32_t hint = a.stride_hint ? *a.stride_hint : 0u;
            for (uint32_t g = 0; g < PASSES; ++g) {
                const uint32_t qc = g * NQ + (lane >> 2);
                quad_prefix<WL>(a, bid * WL + qc, lane & 3u, hint, L.rec + qc, L.rec2 + qc, L.pre + qc, KR);
                if (g + 1 == PASSES) break;
                if ((lane & 3u) == 0 && L.pre[qc].nf) sh_found = 1;   // (benign race: any writer sets 1)
                __syncthreads();
                if (g == 0 && sh_found == 0) break;
            }
        }
        __syncthreads();
        if (a.dbg && lane == 0) a.dbg[8 * bid + 4] = __builtin_amdgcn_s_memrealtime();   // pre-pass done
        // the next decode's first speculation (a hint: any value is safe)
        if (bid == 0 && lane == 0 && a.stride_hint && L.pre[0].nf) *a.stride_hint = L.pre[0].stride;
    }
    // walking column: in lane order, so the block scan over physical lanes stays in segment order
    const uint32_t col = SPREAD == 0 ? lane : (wl < SPREAD && wave < WL / (SPREAD ? SPREAD : 1)) ? wave * SPREAD + wl : WL + lane;
    const SegCount tot = tile_count<COMPACT, KR, NT, G>(a, L, (bid * WL + col) * G, a.n_segs, col, nrec, PRE);
    SegCount btot;
    const SegCount excl = tile_scan<NT>(tot, L, wl, wave, btot);
    if (wave == 0) {
        if (a.dbg && wl == 0) t1 = __builtin_amdgcn_s_memrealtime();
        const SegCount prefix = block_lookback(a, bid, btot, wl);
        if (wl == 0) L.prefix = prefix;
    }
    __syncthreads();
    if (a.dbg && lane == 0) t2 = __builtin_amdgcn_s_memrealtime();
    tile_emit<COMPACT, KR, NT, G>(a, L, sc_add(L.prefix, excl), nrec, bid * WL * G, a.n_segs, lane, col);
    if (a.dbg) {   // diagnostic timestamps (100 MHz s_memrealtime), written only to the dbg buffer
        __syncthreads();
        if (lane == 0) {
            a.dbg[8 * bid + 0] = t0;
            a.dbg[8 * bid + 1] = t1;
            a.dbg[8 * bid + 2] = t2;
            a.dbg[8 * bid + 3] = __builtin_amdgcn_s_memrealtime();
        }
    }
    if (bid == n_blocks - 1 && lane == 0) write_summary<COMPACT>(a, sc_add(L.prefix, btot));
}

// A segment that is exactly ONE complete plain masked FIN BIN frame of a connection with nothing
// open (status OPEN, no fragmented message, no streamed frame): websocket.go:142-146 then
// websocket_frame.go:52-91 -- Message{MsgID, Opcode 2}, messageMode 0, msgID + 1.  walk_segment's
// `fast` path for it counts {1 frame, 1 span, plen bytes} and emits what emit_simple writes; the
// tiled walk (one connection read per segment, the commonest shape at 1 M segments) takes it
// without the state machine in both passes.  (plen > 0: a span; the segment < 4 GiB.)
struct SimpleSeg {
    uint32_t plen, mask, hl;
};
__device__ __forceinline__ bool simple_hdr(const WalkArgs& a, uint64_t start, uint64_t end, const uint4& hd,
                                           SimpleSeg& o) {
    const uint32_t b0 = hd.x & 0xFFu, b1 = (hd.x >> 8) & 0xFFu;
    if (b0 != 0x82u || !(b1 & 0x80u)) return false;
    const uint32_t len7 = b1 & 0x7Fu;
    uint64_t plen;
    if (len7 < 126) {
        plen = len7;
        o.mask = __builtin_amdgcn_alignbyte(hd.y, hd.x, 2);
        o.hl = 6;
    } else if (len7 == 126) {
        plen = ((hd.x >> 8) & 0xFF00u) | (hd.x >> 24);
        o.mask = hd.y;
        o.hl = 8;
    } else {
        const uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(hd.y, hd.x, 2) |
                           (uint64_t)__builtin_amdgcn_alignbyte(hd.z, hd.y, 2) << 32;
        plen = __builtin_bswap64(v);
        o.mask = __builtin_amdgcn_alignbyte(hd.w, hd.z, 2);
        o.hl = 14;
    }
    if (plen == 0 || plen > 0xFFFFFFFFull || plen > a.max_frame_len) return false;
    o.plen = (uint32_t)plen;
    return end - start == (uint64_t)o.hl + plen;
}
__device__ __forceinline__ bool simple_state(uint32_t status, uint64_t cont_len, uint64_t frame_rem) {
    return status == WSC_SEG_OPEN && cont_len == 0 && frame_rem == 0;
}
__device__ __forceinline__ bool simple_seg(const WalkArgs& a, const SegIn& x, SimpleSeg& o) {
    return simple_state(x.st.status, x.st.cont_len, x.st.frame_rem) && simple_hdr(a, x.start, x.end, x.hdr, o);
}

// The outputs walk_segment<EMIT> writes for a simple segment s (frame fi, span si): its record, span,
// window-index entries (windows starting inside the segment look the span up), result and carried
// state -- consecutive lanes hold consecutive segments, so every store is coalesced.
__device__ __forceinline__ void emit_simple(const WalkArgs& a, uint32_t s, const SegIn& x, const SimpleSeg& g,
                                            uint32_t fi, uint32_t si) {
    const uint32_t msg = x.st.msg_id;
    if (fi < a.frames_cap) {
        const uint4 r0 = make_uint4((uint32_t)x.start, (uint32_t)(x.start >> 32), g.plen, g.mask);
        const uint4 r1 = make_uint4(s, msg, 2u | 1u << 8 | (uint32_t)WSC_FK_MESSAGE << 16 | 2u << 24,
                                    (uint32_t)WSC_ERR_NONE | g.hl << 8 | (uint32_t)WSC_FF_UNMASKED << 16);
        reinterpret_cast<uint4*>(a.frames + fi)[0] = r0;
        reinterpret_cast<uint4*>(a.frames + fi)[1] = r1;
    }
    const uint64_t src = x.start + g.hl;
    if (si < a.spans_cap) {
        Span sp;
        sp.src = src;
        sp.dst = src;
        sp.len = g.plen;
        sp.key = rotr32(g.mask, 8u * ((uint32_t)(0u - (uint32_t)src) & 3u));
        a.spans[si] = sp;
    }
    const uint64_t W = 1ull << a.win_shift;
    for (uint64_t w = (x.start + W - 1) >> a.win_shift; (w << a.win_shift) < x.end; ++w) a.tile_first[w] = si;
    wsc_seg_result r;
    r.consumed = x.end - x.start;
    r.frame_begin = fi;
    r.frame_count = 1;
    r.status = WSC_SEG_OPEN;
    r.close_code = 0;
    r.err = 0;
    r.pad = 0;
    a.seg_out[s] = r;
    wsc_conn_state o{};
    o.msg_id = msg + 1;
    a.state_out[s] = o;
}

// Tiled walk for batches of many (short) segments (more than 256 per CU: one connection read per
// segment, e.g. configs[1] with one frame per segment).  A persistent grid whose blocks are all
// resident; block b (by ticket) owns the contiguous segments [b * per, (b + 1) * per) and walks
// them in tiles of NT lanes, one segment per lane:
//   phase 1  count every tile with a PURE walk (no side effects: no records, items or state) into
//            the block's total;
//   look-back  the block's prefix (every block is running, so no block waits on one not started);
//   phase 2  per tile: the count walk again with LDS records (headers now cache-warm), tile scan
//            on top of the running prefix, cooperative emit from LDS -- or, for a tile whose
//            segments are each one complete plain BIN frame (simple_seg), each lane's outputs
//            written straight from its cached header (emit_simple).
// One launch and no per-segment counts in HBM (round 2's three-launch walk wrote and re-read 32 B of
// counts per segment and re-walked every header in its emit pass).
template <bool COMPACT, uint32_t KR, uint32_t NT>
__global__ __launch_bounds__(NT) void k_walk_tiled(WalkArgs a, uint32_t per_block) {
    __shared__ uint32_t sh_bid;
    __shared__ WalkLds<COMPACT, KR, NT, 1> L;
    const uint32_t lane = threadIdx.x, wl = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __builtin_amdgcn_s_setprio(3);   // a latency-bound chain beside streaming unmask waves (neutral, round 5)
    if (lane == 0) sh_bid = walk_block_id(a);
    __syncthreads();
    const uint32_t bid = sh_bid;
    const uint32_t sb = bid * per_block < a.n_segs ? bid * per_block : a.n_segs;
    const uint32_t se = a.n_segs - sb < per_block ? a.n_segs : sb + per_block;
    const SegCount zero = {};
    uint64_t t0 = 0, t1 = 0, t2 = 0;   // diagnostic stamps (WSC_WALK_DEBUG_STAMPS)
    if (a.dbg && lane == 0) t0 = __builtin_amdgcn_s_memrealtime();
    // Inputs are pipelined across tiles: while tile t is walked, tile t+1's first headers and
    // tile t+2's bounds and carried states are already in flight (phase 1); tile t+1's bounds,
    // states and cached headers (phase 2) -- so a tile costs no dependent round trip of its own.
    auto bounds = [&](uint32_t t, SegIn& x) {
        const uint32_t s = t + lane;
        x.st = wsc_conn_state{};
        if (t < se && s < se) {
            x.start = a.seg_off[s];
            x.end = a.seg_off[s + 1];
            if (a.state_in) x.st = a.state_in[s];
        } else {
            x.start = x.end = 0;
        }
    };
    auto first_hdr = [&](SegIn& x) {
        x.hdr = x.end - x.start >= 2 ? hdr_load(a.wire, a.n_bytes, x.start, a.hdr_nt) : make_uint4(0, 0, 0, 0);
    };
    // ---- phase 1: the block's total ----
    // (four tiles per step, every lane's inputs for all four in flight together, measured the same:
    // 34.5-37.3 vs 35.6-39.2 us of count at 1 M one-frame segments -- the header lines, one per
    // segment, are what this phase streams; profiles/r06/stamps_*.log)
    SegCount tot = zero;
    {
        SegIn x0, x1, x2;
        bounds(sb, x0);
        bounds(sb + NT, x1);
        first_hdr(x0);
        for (uint32_t t = sb; t < se; t += NT) {
            if (t + NT < se) first_hdr(x1);
            bounds(t + 2 * NT, x2);
            if (t + lane < se) {
                SimpleSeg g;
                if (!COMPACT && simple_seg(a, x0, g)) {   // what walk_segment's count returns for it
                    tot.frames += 1;
                    tot.spans0 += 1;
                    tot.bytes0 += g.plen;
                    if (a.hdr_cache) a.hdr_cache[t + lane] = x0.hdr;
                } else {
                    tot = sc_add(tot, walk_segment<false, COMPACT, NT, 4, true>(a, t + lane, zero, zero, nullptr, nullptr,
                                                                                nullptr, 0, 0, nullptr, &x0, a.hdr_cache));
                }
            }
            x0 = x1;
            x1 = x2;
        }
    }
    SegCount btot;
    (void)tile_scan<NT>(tot, L, wl, wave, btot);
    if (a.dbg && lane == 0) t1 = __builtin_amdgcn_s_memrealtime();
    if (wave == 0) {
        const SegCount prefix = block_lookback(a, bid, btot, wl);
        if (wl == 0) L.prefix = prefix;
    }
    __syncthreads();
    if (a.dbg && lane == 0) t2 = __builtin_amdgcn_s_memrealtime();
    const SegCount block_prefix = L.prefix;
    // ---- phase 2: tiles in order, each on top of the running prefix ----
    SegCount run = block_prefix;
    auto cached = [&](uint32_t t, SegIn& x) {   // the header cache phase 1 wrote (coalesced)
        bounds(t, x);
        const uint32_t s = t + lane;
        x.hdr = (t < se && s < se && a.hdr_cache) ? a.hdr_cache[s] : make_uint4(0, 0, 0, 0);
        if (!a.hdr_cache) first_hdr(x);
    };
    SegIn y0, y1;
    cached(sb, y0);
    for (uint32_t t = sb; t < se; t += NT) {
        cached(t + NT, y1);
        if constexpr (!COMPACT) {
            // a tile of simple segments only (one complete plain BIN frame each): frame and span
            // ordinals are the lane's, so each lane writes its outputs straight from the cached
            // header -- no second walk, no LDS records, no cooperative emit
            const bool mine = t + lane < se;
            SimpleSeg g{};
            const bool simple = !mine || simple_seg(a, y0, g);
            if (__syncthreads_and(simple)) {
                const uint32_t n = se - t < NT ? se - t : NT;
                uint64_t b = mine ? g.plen : 0u;
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) {
                    const uint32_t lo = __shfl_xor((uint32_t)b, d), hi = __shfl_xor((uint32_t)(b >> 32), d);
                    b += (uint64_t)hi << 32 | lo;
                }
                if (wl == 0) L.wave[wave].bytes0 = b;
                if (mine) emit_simple(a, t + lane, y0, g, run.frames + lane, run.spans0 + run.spans1 + lane);
                __syncthreads();
                uint64_t bsum = 0;
#pragma unroll
                for (uint32_t w = 0; w < NT / 64; ++w) bsum += L.wave[w].bytes0;
                run.frames += n;
                run.spans0 += n;
                run.bytes0 += bsum;
                y0 = y1;
                __syncthreads();   // (L.wave is reused by the next tile)
                continue;
            }
        }
        uint32_t nrec;   // (lanes past the block's last segment count nothing)
        const SegCount c = tile_count<COMPACT, KR, NT, 1>(a, L, t + lane, se, lane, nrec, false, &y0);
        y0 = y1;
        SegCount ttot;
        const SegCount excl = tile_scan<NT>(c, L, wl, wave, ttot);
        tile_emit<COMPACT, KR, NT, 1>(a, L, sc_add(run, excl), nrec, t, se, lane);
        run = sc_add(run, ttot);
        __syncthreads();   // (the tile's LDS is reused by the next tile)
    }
    // phase 2 emitted at the offsets phase 1 published: both passes must have counted the same
    // frames, spans and bytes, or records and summary disagree -- flag it as an internal error
    // (look-back timeout bit: the batch's results are invalid; sticky for wsc_error_flags)
    if (lane == 0) {
        const SegCount want = sc_add(block_prefix, btot);
        if (run.frames != want.frames || run.spans0 != want.spans0 || run.spans1 != want.spans1 ||
            run.bytes0 != want.bytes0 || run.bytes1 != want.bytes1) {
            __hip_atomic_fetch_or(a.lb_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_or(a.sticky, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (a.dbg) {
            a.dbg[8 * bid + 0] = t0;
            a.dbg[8 * bid + 1] = t1;
            a.dbg[8 * bid + 2] = t2;
            a.dbg[8 * bid + 3] = __builtin_amdgcn_s_memrealtime();
        }
    }
    if (se == a.n_segs && sb < se && lane == 0) write_summary<COMPACT>(a, sc_add(block_prefix, btot));
}

// 4 waves per SIMD (128 VGPRs).  Launched after the unmask on the same stream.  (Run instead as
// extra workgroups of the unmask launch, waiting on an unmask-done counter, it measured no faster
// on binary batches and far slower on text: profiles/r04_u8_merge_ab.log, DESIGN.md "Round 4".)
template <uint32_t NCH, uint32_t WPB>
#ifndef WSC_CHECK_WPE   // waves per SIMD k_u8_check is built for (A/B: tools/build_variant.sh)
#define WSC_CHECK_WPE 4
#endif
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(WSC_CHECK_WPE))) void k_u8_check(U8Args a) {
    __shared__ U8Lds T;
    __shared__ uint4 stage[WPB][U8_STAGE];
    u8_check_run<NCH, WPB>(a, T, stage, blockIdx.x, gridDim.x);
    // staged pipeline: the decode's last kernel tells the host its scratch is free
    if (a.fin_host) {
        __syncthreads();
        if (threadIdx.x == 0) fin_signal(a.fin_ctr, a.fin_host, a.fin_seq);
    }
}

template __global__ void k_u8_check<4, 4>(U8Args);

// explicit instantiations used by the host code (every one reached by test_fuzz_walk_geometries):
// 16 frame records per lane (4 in mode 257), one segment per walking lane, blocks of 64 or 256
// lanes; batches of more segments use the tiled walk
template __global__ void k_walk_fused<false, 16, 64, 1, 64, 0>(WalkArgs);
template __global__ void k_walk_fused<false, 16, 64, 1, 16, 0>(WalkArgs);
template __global__ void k_walk_fused<true, 16, 64, 1, 16, 0>(WalkArgs);
template __global__ void k_walk_fused<false, 16, 64, 1, 32, 0>(WalkArgs);
template __global__ void k_walk_fused<true, 16, 64, 1, 32, 0>(WalkArgs);
template __global__ void k_walk_fused<true, 16, 64, 1, 64, 0>(WalkArgs);
template __global__ void k_walk_fused<false, 16, 256, 1, 256, 0>(WalkArgs);
template __global__ void k_walk_fused<true, 16, 256, 1, 256, 0>(WalkArgs);
template __global__ void k_walk_fused<false, 4, 256, 1, 256, 0>(WalkArgs);
template __global__ void k_walk_fused<true, 4, 256, 1, 256, 0>(WalkArgs);
template __global__ void k_walk_fused<false, 16, 256, 1, 64, 0>(WalkArgs);
template __global__ void k_walk_fused<true, 16, 256, 1, 64, 0>(WalkArgs);
template __global__ void k_walk_fused<false, 16, 256, 1, 64, 16>(WalkArgs);
template __global__ void k_walk_fused<true, 16, 256, 1, 64, 16>(WalkArgs);
template __global__ void k_walk_tiled<false, 4, 256>(WalkArgs, uint32_t);
template __global__ void k_walk_tiled<true, 4, 256>(WalkArgs, uint32_t);

// ---------------------------------------------------------------------------------------------
// wsc_kcopy: device <-> pinned host by a kernel that reads or writes host memory over PCIe (no
// copy engine, so the enqueue never holds the host thread).  Grid-stride over 16-byte chunks, 4
// per lane in flight (a PCIe read round trip is ~1-2 us: 256 blocks x 256 lanes x 64 B keeps ~4 MB
// outstanding); non-temporal reads, default stores (a device destination is read next).
// ---------------------------------------------------------------------------------------------
// Any alignment: the head up to dst's first 16-byte boundary and the tail go byte by byte; the
// body stores aligned 16-byte chunks, loading them aligned (nt) when src shares dst's alignment
// and with unaligned 16-byte loads otherwise.
template <bool SRC_ALIGNED>
__device__ __forceinline__ void kcopy_body(u32x4* __restrict__ d4, const uint8_t* __restrict__ s, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    auto ld = [&](uint64_t k) -> u32x4 {
        if constexpr (SRC_ALIGNED) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s) + k);
        const u32x4u_ld t = __builtin_nontemporal_load(reinterpret_cast<const u32x4u_ld*>(s + 16 * k));
        return u32x4{t.x, t.y, t.z, t.w};
    };
    for (; i + 3 * stride < n16; i += 4 * stride) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = ld(i + k * stride);
#pragma unroll
        for (int k = 0; k < 4; ++k) d4[i + k * stride] = v[k];
    }
    for (; i < n16; i += stride) d4[i] = ld(i);
}

__global__ __launch_bounds__(256) void k_kcopy(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t bytes) {
    uint64_t head = (16u - (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u;
    if (head > bytes) head = bytes;
    const uint64_t n16 = (bytes - head) >> 4;
    const uint64_t tail0 = head + (n16 << 4);
    if (blockIdx.x == 0 && threadIdx.x < 16) {
        if (threadIdx.x < head) dst[threadIdx.x] = src[threadIdx.x];
        if (tail0 + threadIdx.x < bytes) dst[tail0 + threadIdx.x] = src[tail0 + threadIdx.x];
    }
    u32x4* d4 = reinterpret_cast<u32x4*>(dst + head);
    if ((reinterpret_cast<uintptr_t>(src + head) & 15u) == 0) kcopy_body<true>(d4, src + head, n16);
    else kcopy_body<false>(d4, src + head, n16);
}

}  // namespace wsc
