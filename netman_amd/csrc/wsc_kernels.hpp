// wsc_kernels.hpp -- device-side types shared by the gfx950 kernels and the host launch code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/wscodec.h"

namespace wsc {

// Per-segment counts produced by the header walk; the exclusive scan of these gives each
// segment its slice of every output array.  In-place mode uses only frames/spans0/flags.
struct SegCount {
    uint32_t frames;   // frame records
    uint32_t spans0;   // payload spans (in-place: all; COMPACT: data region)
    uint32_t spans1;   // COMPACT: control-region spans
    uint32_t flags;    // SEGF_*
    uint64_t bytes0;   // COMPACT: data-region bytes
    uint64_t bytes1;   // COMPACT: control-region bytes
};

struct SegCountAdd {
    __host__ __device__ SegCount operator()(const SegCount& a, const SegCount& b) const {
        SegCount r;
        r.frames = a.frames + b.frames;
        r.spans0 = a.spans0 + b.spans0;
        r.spans1 = a.spans1 + b.spans1;
        r.flags = a.flags | b.flags;
        r.bytes0 = a.bytes0 + b.bytes0;
        r.bytes1 = a.bytes1 + b.bytes1;
        return r;
    }
};

// SEGF_LONG: a record's length needs more than 32 bits (the LDS replay keeps 32): emit by re-walking
enum : uint32_t { SEGF_UTF8 = 1u, SEGF_U8DEFER = 2u, SEGF_LONG = 4u };

// ---- chip-wide UTF-8 (k_u8_check) ------------------------------------------------------------
// The walk validates text payloads of at most u8_inline_max bytes itself (serial DFA per lane);
// larger ones -- and every later frame of a text chain that has a deferred part -- become items of
// at most U8_PIECE bytes (one per frame below 1 GiB), validated chip-wide: the unmask folds the
// maps of the windows inside them, k_u8_check the partial windows at their ends (after the unmask).
constexpr uint32_t U8_PIECE = 1u << 30;
// close reasons are SELF items; a streamed PONG's piece under TEXT mode (Q6) is a PONG item (the
// PONG continues in the next batch: its end state is carried) or PONG_END (its verdict), entry state
// known at the walk (0 at its header, else the carried frame_utf8)
enum : uint8_t { U8K_SELF = 0, U8K_PART = 1, U8K_CHAIN = 2, U8K_PONG = 3, U8K_PONG_END = 4 };
constexpr uint32_t U8_DEAD = 0xFFFFFFFFu;   // U8Item.seg of an unused walk-pool slot
struct U8Item {
    uint64_t src;       // wire offset of the first (masked) byte
    uint32_t len;
    uint32_t mask;      // mask word, phase 0 at src
    uint32_t seg;
    uint32_t ordinal;   // frame ordinal within the segment
    uint32_t next;      // next item of the same segment (0xFFFFFFFF = last)
    uint8_t kind;       // U8K_*
    uint8_t s_in;       // DFA state entering a chain frame, 0xFF = the previous chain item's result
    uint8_t first, last;   // first / last piece of its frame
};
static_assert(sizeof(U8Item) == 32, "U8Item layout");
struct U8Seg {          // per segment with deferred items (written by the walk)
    uint32_t head, n, done;
    uint32_t pending_end;  // bit 0: a text chain with a deferred part is still open; bit 1: composite items;
                           // bit 2: a deferred PONG piece is still open (its state -> frame_utf8)
    uint32_t sbase, nspans, fbase;         // the segment's span and frame ranges (emit pass)
    uint32_t minfail;      // first failing single-piece SELF frame (ordinal), 0xFFFFFFFF = none
};

// One contiguous run of masked payload bytes to XOR: source in the wire, destination either the
// same bytes (in place) or the arena (COMPACT).  `key` is the mask word rotated so that it XORs
// 4-byte-aligned destination dwords directly: key = rotr(mask, 8 * ((-dst) & 3)).
// spans carry u32 lengths: a payload of 4 GiB or more (64-bit length, websocket.go:291-299) is
// cut into spans at the ABSOLUTE wire offsets that are multiples of SPAN_CHUNK (2 GiB) -- window
// boundaries, so no unmask window ever holds a cut (every window inside a text payload stays a
// one-span fast-path window whose UTF-8 map the unmask folds); everything shorter is one span
constexpr uint64_t SPAN_CHUNK = 1ull << 31;
__host__ __device__ __forceinline__ uint32_t span_chunks(uint64_t src, uint64_t plen) {
    return plen <= 0xFFFFFFFFull ? 1u : (uint32_t)(((src + plen - 1) >> 31) - (src >> 31) + 1);
}

struct Span {
    uint64_t src;
    uint64_t dst;
    uint32_t len;
    uint32_t key;
};
static_assert(sizeof(Span) == 24, "span layout");

struct WalkArgs {
    const uint8_t* wire;
    uint64_t n_bytes;
    const uint64_t* seg_off;
    uint32_t n_segs;
    uint32_t frames_cap;
    const wsc_conn_state* state_in;
    uint64_t max_frame_len;
    wsc_frame* frames;
    Span* spans;
    uint32_t spans_cap;
    uint32_t win_shift;          // log2(unmask window bytes)
    uint32_t* tile_first;        // per wire window: first span (stream order) whose wire end > window start
    uint64_t* frame_dst;         // COMPACT
    wsc_conn_state* state_out;
    wsc_seg_result* seg_out;
    wsc_summary* summary;
    uint32_t* lb_ticket;         // look-back: dynamic block id counter
    uint64_t* lb_rec;            // per block: its look-back record, 8 self-tagged words (block_lookback)
    uint32_t* lb_err;            // bounded-spin timeout
    uint64_t* dbg;               // optional per-block timestamps (WSC_WALK_DEBUG_STAMPS)
    uint32_t* u8info;            // per segment: {first utf8-failing frame ordinal, DFA state}
    U8Item* u8items;             // deferred UTF-8 items
    uint32_t u8items_cap;
    uint32_t* u8count;           // item counter, one per decode parity (re-armed by the next decode's k_unmask)
    U8Seg* u8seg;
    uint32_t u8_inline_max;      // text payloads up to this many bytes are validated in the walk
    uint32_t* sticky;            // context error bits, never re-armed by a kernel (wsc_error_flags)
    uint32_t* u8host;            // host-visible word set when any UTF-8 item is deferred (cleared by the host)
    uint32_t* win_flag;          // per unmask window: 1 = inside a deferred text item (k_unmask folds its map)
    uint32_t compact;            // WSC_F_COMPACT (the kernels are also templated on it)
    uint32_t quad_pre;           // fused walk with one walking wave per 4: the quad pre-pass (WSC_WALK_NO_QUAD_PRE: off)
    uint4* hdr_cache;            // tiled walk: per segment, the 16 bytes at its first frame (null: off)
    uint32_t* stride_hint;       // quad pre-pass: the stride the last decode ended with (first speculation)
    uint32_t hdr_nt;             // non-temporal header loads (hdr_load): COMPACT batches (and WSC_WALK_HDR_NT)
};

// k_u8_check runs AFTER the unmask: the unmask has already folded every text window that lies
// inside an item (win_map), so the check reads only the items' partial windows at their ends --
// in place from the unmasked wire (mask 0), COMPACT from the still-masked wire -- composes, and
// applies the verdicts (segment by segment, as their last items finish).  Frames after a failing
// one were unmasked too: their spans are XORed again (re-masked), so the output equals what the
// reference leaves (it never reads them).
struct U8Args {
    const uint8_t* wire;
    uint64_t n_bytes;
    const uint64_t* seg_off;
    const U8Item* items;
    const uint32_t* count;       // item count (this decode's parity)
    uint32_t items_cap;
    uint64_t* maps;              // per item: DFA transition map (9 x 4 bits)
    U8Seg* seg;
    wsc_frame* frames;
    Span* spans;
    wsc_seg_result* seg_out;
    wsc_conn_state* state_out;
    wsc_summary* summary;
    const uint64_t* win_map;     // per unmask window: the map the unmask folded
    uint32_t win_shift;
    uint32_t unmasked;           // 1: the wire is already unmasked (in place): items are read with mask 0
    uint8_t* out;                // where the spans' bytes went: the wire (in place) or the arena (COMPACT)
    uint32_t n_segs;
    uint32_t* fin_ctr;           // staged pipeline: finished-workgroup counters (fin_signal)
    uint32_t* fin_host;          // ... the last workgroup writes fin_seq here
    uint32_t fin_seq;
};

// The unmask's side of the text windows (k_unmask): flag / map per window, and the item count
// (zero = nothing deferred: the LDS tables are not even built).
struct U8Win {
    uint32_t* flag;
    uint64_t* map;
    const uint32_t* count;
    uint32_t* rearm;             // the next decode's item counter (zeroed by the unmask: always launched)
    uint32_t xcd_run;            // blocks per XCD run: consecutive logical blocks (windows) on one XCD
                                 // (0 / 1: the hardware's round-robin deal), see unmask_all
    uint64_t* lb_rec;            // the walk's look-back records, re-armed (zeroed) by this launch
};


// ---- encode (wsc_encode.hip) ----------------------------------------------------------------
constexpr uint32_t ENC_WIN_SHIFT = 12;                 // 4 KiB output windows
constexpr uint32_t ENC_WIN = 1u << ENC_WIN_SHIFT;
constexpr uint32_t ENC_IPT = 16;                       // encode scan: consecutive messages per thread

struct EncArgs {
    const wsc_out_msg* msgs;
    uint32_t n_msgs;
    uint64_t* out_off;           // n_msgs + 1
    uint32_t* tile;              // per output window: the frame its first byte belongs to
    uint64_t tile_entries;
    uint32_t* lb_ticket;
    uint64_t* lb_rec;            // per scan block: its self-tagged look-back word
    uint32_t* lb_err;
    uint32_t* sticky;            // context error bits (bit2: encode look-back timeout)
};

struct EncCopyArgs {
    const wsc_out_msg* msgs;
    uint32_t n_msgs;
    const uint64_t* out_off;
    const uint8_t* src;
    uint64_t src_bytes;
    uint8_t* out;
    uint64_t out_cap;
    const uint32_t* tile;
    uint64_t tile_entries;
    uint32_t* lb_state;          // the scan's look-back state, re-armed by this launch
    uint64_t* lb_rec;            // ... and its records
    uint32_t n_lb;
    uint32_t xcd_run;            // blocks per XCD run (xcd_run_block)
    uint32_t hoist;              // load the window's frames before the inside-one-payload test (small messages)
};

}  // namespace wsc
