// wsc_api.cpp -- host side of libwscodec: context, launch sequence, host-staged path, timing.
// Compiled by hipcc together with wsc_kernels.hip (gfx950 only; no CPU fallback anywhere: a
// missing device is an error, WSC_E_NODEVICE).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>

#include "wsc_kernels.hpp"

namespace wsc {
template <bool COMPACT, uint32_t KR, uint32_t NT, uint32_t G, uint32_t WL, uint32_t SPREAD> __global__ void k_walk_fused(WalkArgs);
template <bool COMPACT, uint32_t KR, uint32_t NT> __global__ void k_walk_tiled(WalkArgs, uint32_t);
template <uint32_t NCH, uint32_t WPB> __global__ void k_u8_check(U8Args);
template <bool COMPACT, int P, int NT, int MINW, bool U8>
__global__ void k_unmask(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*,
                         const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template <uint32_t IPT> __global__ void k_encode_scan(EncArgs);
__global__ void k_kcopy(uint8_t*, const uint8_t*, uint64_t);
template <int NT> __global__ void k_encode_copy(EncCopyArgs);
}  // namespace wsc

using namespace wsc;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
}  // namespace

namespace wsc {
// wsc_last_error() text for the session layer (wsc_session.cpp), same thread-local slot
int set_last_error(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace wsc

namespace {
#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return fail(WSC_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

uint32_t ilog2(uint32_t x) {
    uint32_t r = 0;
    while ((1u << (r + 1)) <= x) ++r;
    return r;
}
}  // namespace

struct wsc_ctx {
    int device = 0;
    int n_cu = 256;
    hipStream_t stream = nullptr;
    hipEvent_t ev_walked = nullptr;   // wsc_decode_split: walk done (unmask stream waits on it)
    hipEvent_t ev_done = nullptr;     // wsc_decode_split: unmask done (the next walk on this ctx waits)
    // host-visible words (pinned, coherent): [0] the walk deferred UTF-8 items, [1] sequence number
    // of the last staged unmask that has finished (written by its last workgroup)
    uint32_t* hflag = nullptr;
    uint32_t* fin_ctr = nullptr;      // staged unmask: finished-workgroup counters (two-level, self re-arming)
    uint32_t fin_seq = 0;             // sequence number of the last staged unmask enqueued
    bool fin_pending = false;         // a staged unmask was enqueued without ev_done
    hipStream_t fin_stream = nullptr; // ... on this stream
    bool walk_waited = false;         // wsc_walk_wait saw the last walk complete
    // Measured-and-rejected variants are not built into this library (tools/build_variant.sh builds
    // them for A/B runs); nothing here reads the environment.  The fixed choices, with their A/Bs:
    //  - k_u8_check: 4 independent byte chains per 64-byte lane chunk, 256-lane workgroups, 4 per CU
    //    (1 KiB TEXT 0.241 -> 0.238 ms vs 2 chains; 1,024-lane workgroups slower on text, round 5)
    //  - in-place unmask windows through buffer ops, sc0 nt sc1 stores (headline 2,890-2,898 ->
    //    2,911-2,918 GiB/s, profiles/r02_unmask_policy.log); 4 KiB windows (r01_tune_*)
    //  - walk look-back order by ticket (hardware order measured slower, r04_walk_hw_order_ab.log);
    //    walk waves at raised issue priority (neutral, round 5)
    wsc_config cfg{};
    uint32_t pieces = 8;          // 16 B pieces per lane -> window = pieces KiB
    uint32_t* sticky = nullptr;      // error bits of every decode/encode (wsc_error_flags), never re-armed
    uint32_t* lb_state = nullptr;    // [0] ticket, [1] spin-timeout flag, [2] UTF-8 item count, [3..] per-block flags
    uint32_t* u8info = nullptr;      // per segment {utf8-failing frame ordinal, DFA state}
    uint64_t* lb_rec = nullptr;      // per walk block: its look-back record (8 words)
    uint64_t* dbg = nullptr;         // WSC_WALK_DEBUG_STAMPS: per-block walk timestamps
    Span* spans = nullptr;
    uint32_t* tile = nullptr;
    // chip-wide UTF-8 (k_u8_check): deferred items, their maps, per-segment lists
    U8Item* u8items = nullptr;
    uint64_t* u8maps = nullptr;
    uint32_t u8items_cap = 0;
    U8Seg* u8seg = nullptr;
    uint32_t* win_flag = nullptr;       // per unmask window: inside a deferred text item (walk sets, unmask clears)
    uint64_t* win_map = nullptr;        // per unmask window: the DFA map the unmask folded
    uint32_t* u8ctr = nullptr;          // UTF-8 item counters, one per decode parity ([0], [32]): a decode's walk
                                        // allocates from its own, its unmask zeroes the other (the next decode's)
    uint32_t u8par = 0;                 // parity of the decode the last walk belongs to
    bool u8_dirty = false;              // a walk was launched whose unmask (which zeroes the next decode's item
                                        // counter) was not: the next walk zeroes its counter itself
    uint32_t u8_inline_max = 256;       // wsc_config.u8_inline_max
    bool hdr_nt_all = false;            // WSC_WALK_HDR_NT: non-temporal header loads in place too (COMPACT always)
    bool quad_pre = true;               // !WSC_WALK_NO_QUAD_PRE
    static constexpr uint32_t xcd_run = 8;       // unmask blocks per XCD run (1 = the hardware deal; one run per
                                                 // XCD over the whole grid measured slower: 0.347 -> 0.359 ms)
    static constexpr uint32_t enc_xcd_run = 1;   // the same for the encode copy (8 measured 0.381 -> 0.383-0.399
                                                 // ms at 64 KiB, no change at 1 KiB: off)
    int walk_mode = 0;                  // wsc_config.walk_mode: 16, 32, 64, 65, 66, 256, 257 or 3 pins the geometry; 0 = auto
    uint32_t walk_used = 0;             // geometry (64 / 256 / 3) and block count of the last walk launched:
    uint32_t walk_blocks = 0;           // the staged unmask re-arms exactly that walk's look-back flags
    uint32_t max_walk_blocks = 0;       // look-back state allocated for this many walk blocks
    uint4* hdr_cache = nullptr;         // tiled walk: per segment, its first 16 header bytes (WSC_WALK_NO_HDR_CACHE: off)
    uint32_t* stride_hint = nullptr;    // quad pre-pass: the frame stride the last decode ended with
    uint64_t tile_entries = 0;
    // host-staged path buffers (lazily allocated)
    uint8_t* d_wire = nullptr;
    uint8_t* d_arena = nullptr;
    uint64_t* d_seg_off = nullptr;
    wsc_conn_state* d_state_in = nullptr;
    wsc_conn_state* d_state_out = nullptr;
    wsc_seg_result* d_seg_out = nullptr;
    wsc_frame* d_frames = nullptr;
    uint64_t* d_frame_dst = nullptr;
    wsc_summary* d_summary = nullptr;
    // encode scratch: look-back state [ticket, timeout, flags...], aggregates, window index
    uint32_t* enc_lb_state = nullptr;
    uint64_t* enc_lb_rec = nullptr;   // per scan block: its look-back word
    uint32_t enc_blocks = 0;
    uint32_t* enc_tile = nullptr;
    uint64_t enc_cap = 0;             // largest out_cap: max_batch_bytes + 16 * max_frames
    uint64_t enc_tile_entries = 0;
    // host-staged encode buffers (lazily allocated)
    wsc_out_msg* d_enc_msgs = nullptr;
    uint8_t* d_enc_src = nullptr;
    uint8_t* d_enc_out = nullptr;
    uint64_t* d_enc_off = nullptr;
};

extern "C" {

// walk geometry (see launch): 64 = fused walk with 64-lane blocks, 256 = fused with 256-lane
// blocks, 3 = the tiled walk
// CUs of the streams made by wsc_stream_create with a CU mask (any context of the process may
// launch on them): the walk's geometry must fit the CUs it actually runs on -- a fused walk whose
// blocks cannot all be resident serialises on its look-back (a 65 k-segment walk on 16 CUs ran
// longer than the 4 GiB unmask beside it)
static std::mutex g_stream_mu;
static std::unordered_map<hipStream_t, uint32_t> g_stream_cus;
static uint32_t stream_cus(const wsc_ctx* c, hipStream_t s) {
    if (s) {
        std::lock_guard<std::mutex> lk(g_stream_mu);
        auto it = g_stream_cus.find(s);
        if (it != g_stream_cus.end()) return it->second;
    }
    return (uint32_t)c->n_cu;
}
static uint32_t walk_mode(const wsc_ctx* c, uint32_t n_segs, uint32_t cus) {
    if (c->walk_mode) return (uint32_t)c->walk_mode;
    // a CU-masked walk stream whose CUs hold every segment in 4 resident 64-lane blocks per CU:
    // 64-lane blocks (headline pipeline, 16 CUs: 2,941 vs 2,842 GiB/s with 256-lane blocks).
    // Larger batches keep the whole-chip choice: measured, a fused walk whose blocks are not all
    // resident still beat the (since removed) three-launch walk there (configs[1] on 32 CUs: 0.435 vs 0.497 ms)
    if (cus < (uint32_t)c->n_cu && n_segs <= 256u * cus) return 64;
    const uint32_t all = (uint32_t)c->n_cu;
    // up to one wave of segments per CU: one walking wave per CU, four emitting (mode 65)
    if (n_segs <= 64u * all) return 65;
    if (n_segs <= 256u * all) return 256;
    return 3;
}

// The staged pipeline's unmask records no event (a marker between two unmasks costs ~6 us of
// idle chip): its last workgroup writes the sequence number to hflag[1] instead, and the next
// walk on this context waits for it here, on the host.  A stream that drains without the word
// arriving means the unmask failed.
static int fin_wait(wsc_ctx* c) {
    if (!c->fin_pending) return WSC_OK;
    // no HIP call while the unmask is expected to finish: hipStreamQuery puts a marker packet on
    // the stream (measured: a 5.6 us gap between consecutive unmasks); only a wait that has lasted
    // 100 ms asks the stream whether it is still busy
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (uint32_t spin = 1;; ++spin) {
        if (__atomic_load_n(&c->hflag[1], __ATOMIC_ACQUIRE) == c->fin_seq) break;
        if ((spin & 4095) == 0 && clk::now() - t0 > std::chrono::milliseconds(100)) {
            const hipError_t q = hipStreamQuery(c->fin_stream);
            if (q == hipErrorNotReady) continue;
            if (__atomic_load_n(&c->hflag[1], __ATOMIC_ACQUIRE) == c->fin_seq) break;
            c->fin_pending = false;
            return fail(WSC_E_DEVICE, std::string("staged unmask did not finish: ") +
                                          (q == hipSuccess ? "stream drained" : hipGetErrorString(q)));
        }
        __builtin_ia32_pause();
    }
    c->fin_pending = false;
    return WSC_OK;
}

int wsc_abi_version(void) { return WSC_ABI_VERSION; }
const char* wsc_last_error(void) { return g_err.c_str(); }

int wsc_config_default(wsc_config* cfg) {
    if (!cfg) return fail(WSC_E_INVAL, "cfg is NULL");
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->max_batch_bytes = 64ull << 20;
    cfg->max_segs = 1u << 16;
    cfg->max_frames = 1u << 20;
    cfg->max_frame_len = 0xFFFFFFFFFFull;   // 2^40 - 1: the record width (Q4)
    cfg->unmask_window = 4096;       // tools/tune_unmask.py, profiles/r01_tune_*.log
    cfg->unmask_waves_per_cu = 0;    // 0: one window per wave (grid = windows)
    cfg->unmask_nt = 3 | 1 << 2;     // in place: non-temporal loads and stores; COMPACT (bits 2-3): NT loads,
                                     // default-policy stores.  The arena is written at byte offsets, so each
                                     // 1 KiB store instruction starts and ends inside a line; NT stores sent
                                     // those partial lines to HBM separately: configs[4] wrote 2,570 MB for
                                     // 2,419 MB of payload, default stores 2,426 MB, decode time unchanged
                                     // (0.999 vs 1.001 ms back to back, profiles/r04_compact_store_policy.log)
    cfg->walk_mode = 0;
    cfg->u8_inline_max = 256;
    cfg->walk_flags = 0;
    return WSC_OK;
}
static constexpr uint32_t UNMASK_NT_DEFAULT = 3 | 1 << 2;

static int alloc_host_path(wsc_ctx* c) {
    if (c->d_wire) return WSC_OK;
    const wsc_config& g = c->cfg;
    HIP_TRY(hipMalloc(&c->d_wire, g.max_batch_bytes + 64));
    HIP_TRY(hipMalloc(&c->d_arena, g.max_batch_bytes + 64));
    HIP_TRY(hipMalloc(&c->d_seg_off, (g.max_segs + 1) * sizeof(uint64_t)));
    HIP_TRY(hipMalloc(&c->d_state_in, g.max_segs * sizeof(wsc_conn_state)));
    HIP_TRY(hipMalloc(&c->d_state_out, g.max_segs * sizeof(wsc_conn_state)));
    HIP_TRY(hipMalloc(&c->d_seg_out, g.max_segs * sizeof(wsc_seg_result)));
    HIP_TRY(hipMalloc(&c->d_frames, (uint64_t)g.max_frames * sizeof(wsc_frame)));
    HIP_TRY(hipMalloc(&c->d_frame_dst, (uint64_t)g.max_frames * sizeof(uint64_t)));
    HIP_TRY(hipMalloc(&c->d_summary, sizeof(wsc_summary)));
    return WSC_OK;
}

int wsc_create(int device, const wsc_config* cfg_in, wsc_ctx** out) {
    if (!out) return fail(WSC_E_INVAL, "out is NULL");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(WSC_E_NODEVICE, "no HIP device visible");
    if (device < 0 || device >= ndev) return fail(WSC_E_INVAL, "device index out of range");
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(WSC_E_NODEVICE, std::string("libwscodec is built for gfx950, device is ") + prop.gcnArchName);
    wsc_config cfg;
    if (cfg_in) cfg = *cfg_in; else wsc_config_default(&cfg);
    if (cfg.max_segs == 0 || cfg.max_frames == 0 || cfg.max_batch_bytes == 0)
        return fail(WSC_E_INVAL, "zero capacity in config");
    if (cfg.max_frame_len > 0xFFFFFFFFFFull) return fail(WSC_E_INVAL, "max_frame_len > 2^40-1");
    // only the measured defaults are built (8 KiB windows and the other cache policies: A/B builds)
    const uint32_t win = cfg.unmask_window ? cfg.unmask_window : 4096;
    if (win != 4096) return fail(WSC_E_INVAL, "unmask_window must be 4096 (or 0)");
    cfg.unmask_window = win;
    if (cfg.unmask_nt == 0) cfg.unmask_nt = UNMASK_NT_DEFAULT;
    if (cfg.unmask_nt != UNMASK_NT_DEFAULT) return fail(WSC_E_INVAL, "unmask_nt must be the default (or 0)");
    const uint32_t wm = cfg.walk_mode;
    if (!(wm == 0 || wm == 16 || wm == 32 || wm == 64 || wm == 65 || wm == 66 || wm == 256 || wm == 257 || wm == 3))
        return fail(WSC_E_INVAL, "walk_mode must be 0, 16, 32, 64, 65, 66, 256, 257 or 3");
    if (cfg.walk_flags & ~(uint32_t)(WSC_WALK_NO_QUAD_PRE | WSC_WALK_NO_HDR_CACHE | WSC_WALK_HDR_NT | WSC_WALK_DEBUG_STAMPS))
        return fail(WSC_E_INVAL, "unknown walk_flags bits");

    HIP_TRY(hipSetDevice(device));
    wsc_ctx* c = new wsc_ctx();
    c->device = device;
    c->n_cu = prop.multiProcessorCount;
    c->cfg = cfg;
    c->pieces = win / 1024;
    int rc = WSC_OK;
    auto chk = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && rc == WSC_OK) rc = fail(WSC_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
    };
    chk(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "hipStreamCreate");
    // the split pipeline's events join streams of this device only: no system-scope fence at the
    // record (which writes back and invalidates caches; measured ~13 us between one batch's unmask
    // and the next -- as long as the walk the split was meant to hide).  Kernel ends still release
    // at device scope, which is what the other stream's kernels need.
    const unsigned ev_flags = hipEventDisableTiming | hipEventDisableSystemFence;
    chk(hipEventCreateWithFlags(&c->ev_walked, ev_flags), "hipEventCreate");
    chk(hipEventCreateWithFlags(&c->ev_done, ev_flags), "hipEventCreate");
    chk(hipHostMalloc(&c->hflag, 64, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc hflag");
    chk(hipMalloc(&c->fin_ctr, 257 * 32 * sizeof(uint32_t)), "hipMalloc fin_ctr");   // k_unmask FIN_GROUPS/STRIDE
    if (rc == WSC_OK) {
        std::memset(c->hflag, 0, 64);
        chk(hipMemsetAsync(c->fin_ctr, 0, 257 * 32 * sizeof(uint32_t), c->stream), "hipMemset fin_ctr");
    }
    chk(hipMalloc(&c->sticky, sizeof(uint32_t)), "hipMalloc sticky");
    chk(hipMalloc(&c->stride_hint, sizeof(uint32_t)), "hipMalloc stride_hint");
    if (rc == WSC_OK) chk(hipMemsetAsync(c->stride_hint, 0, sizeof(uint32_t), c->stream), "hipMemset stride_hint");
    if (!(cfg.walk_flags & WSC_WALK_NO_HDR_CACHE))
        chk(hipMalloc(&c->hdr_cache, (uint64_t)cfg.max_segs * sizeof(uint4)), "hipMalloc hdr_cache");
    if (rc == WSC_OK) chk(hipMemsetAsync(c->sticky, 0, sizeof(uint32_t), c->stream), "hipMemset sticky");
    // the most walk blocks (64 segments per block; 16 per block for up to 64 segments per CU); the
    // look-back flags, aggregates and prefixes are indexed by block
    const uint64_t max_blocks = std::max<uint64_t>((cfg.max_segs + 63) / 64,
                                                   (std::min<uint64_t>(cfg.max_segs, 64ull * (uint64_t)c->n_cu) + 15) / 16) + 1;
    c->max_walk_blocks = (uint32_t)max_blocks;
    chk(hipMalloc(&c->lb_state, (max_blocks + 3) * sizeof(uint32_t)), "hipMalloc lb_state");
    chk(hipMalloc(&c->u8info, (uint64_t)cfg.max_segs * 2 * sizeof(uint32_t)), "hipMalloc u8info");
    chk(hipMalloc(&c->lb_rec, max_blocks * 8 * sizeof(uint64_t)), "hipMalloc lb_rec");
    if (cfg.walk_flags & WSC_WALK_DEBUG_STAMPS)
        chk(hipMalloc(&c->dbg, max_blocks * 8 * sizeof(uint64_t)), "hipMalloc dbg");
    if (rc == WSC_OK) {
        chk(hipMemsetAsync(c->lb_state, 0, (max_blocks + 3) * sizeof(uint32_t), c->stream), "hipMemset lb_state");
        chk(hipMemsetAsync(c->lb_rec, 0, max_blocks * 8 * sizeof(uint64_t), c->stream), "hipMemset lb_rec");
        chk(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    }
    chk(hipMalloc(&c->spans, (uint64_t)cfg.max_frames * sizeof(Span)), "hipMalloc spans");
    c->tile_entries = cfg.max_batch_bytes / 1024 + 2;
    chk(hipMalloc(&c->tile, c->tile_entries * sizeof(uint32_t)), "hipMalloc tile");
    // a frame is one item up to U8_PIECE (1 GiB), longer ones one per U8_PIECE-aligned boundary
    // inside their payload more, so frames + bytes / U8_PIECE + 1 bounds the total
    // (+ up to 3 unused pool slots per segment and per > 1 GiB frame: the walk's item pools)
    c->u8items_cap = cfg.max_frames + 4 * cfg.max_segs + 4 * (uint32_t)(cfg.max_batch_bytes / U8_PIECE) + 64;
    chk(hipMalloc(&c->u8items, (uint64_t)c->u8items_cap * sizeof(U8Item)), "hipMalloc u8items");
    chk(hipMalloc(&c->u8maps, (uint64_t)c->u8items_cap * sizeof(uint64_t)), "hipMalloc u8maps");
    chk(hipMalloc(&c->u8seg, (uint64_t)cfg.max_segs * sizeof(U8Seg)), "hipMalloc u8seg");
    chk(hipMalloc(&c->win_flag, c->tile_entries * sizeof(uint32_t)), "hipMalloc win_flag");
    chk(hipMalloc(&c->win_map, c->tile_entries * sizeof(uint64_t)), "hipMalloc win_map");
    chk(hipMalloc(&c->u8ctr, 64 * sizeof(uint32_t)), "hipMalloc u8ctr");
    if (rc == WSC_OK) {
        chk(hipMemsetAsync(c->win_flag, 0, c->tile_entries * sizeof(uint32_t), c->stream), "hipMemset win_flag");
        chk(hipMemsetAsync(c->u8ctr, 0, 64 * sizeof(uint32_t), c->stream), "hipMemset u8ctr");
        chk(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    }
    c->quad_pre = !(cfg.walk_flags & WSC_WALK_NO_QUAD_PRE);
    c->hdr_nt_all = (cfg.walk_flags & WSC_WALK_HDR_NT) != 0;
    c->walk_mode = (int)cfg.walk_mode;
    c->u8_inline_max = cfg.u8_inline_max;
    if (c->u8_inline_max >= 4096) c->u8_inline_max = 4095;   // a payload holding a whole window is deferred
    c->enc_blocks = (cfg.max_frames + 255) / 256 + 1;
    c->enc_cap = cfg.max_batch_bytes + 16ull * cfg.max_frames;
    c->enc_tile_entries = c->enc_cap / ENC_WIN + 2;
    chk(hipMalloc(&c->enc_lb_state, (c->enc_blocks + 2) * sizeof(uint32_t)), "hipMalloc enc_lb_state");
    chk(hipMalloc(&c->enc_lb_rec, (c->enc_blocks + 2) * sizeof(uint64_t)), "hipMalloc enc_lb_rec");
    chk(hipMalloc(&c->enc_tile, c->enc_tile_entries * sizeof(uint32_t)), "hipMalloc enc_tile");
    if (rc == WSC_OK) {
        chk(hipMemsetAsync(c->enc_lb_state, 0, (c->enc_blocks + 2) * sizeof(uint32_t), c->stream), "hipMemset enc_lb_state");
        chk(hipMemsetAsync(c->enc_lb_rec, 0, (c->enc_blocks + 2) * sizeof(uint64_t), c->stream), "hipMemset enc_lb_rec");
        chk(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    }
    if (rc != WSC_OK) {
        wsc_destroy(c);
        return rc;
    }
    *out = c;
    return WSC_OK;
}

int wsc_destroy(wsc_ctx* c) {
    if (!c) return WSC_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    (void)fin_wait(c);
    void* ptrs[] = {c->fin_ctr, c->dbg, c->sticky, c->hdr_cache, c->stride_hint, c->lb_state, c->u8info, c->lb_rec, c->spans, c->tile, c->d_wire, c->d_arena,
                    c->d_seg_off, c->d_state_in, c->d_state_out, c->d_seg_out, c->d_frames,
                    c->d_frame_dst, c->d_summary, c->enc_lb_state, c->enc_lb_rec, c->enc_tile,
                    c->d_enc_msgs, c->d_enc_src, c->d_enc_out, c->d_enc_off, c->u8items, c->u8maps, c->u8seg,
                    c->win_flag, c->win_map, c->u8ctr};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->ev_walked) (void)hipEventDestroy(c->ev_walked);
    if (c->ev_done) (void)hipEventDestroy(c->ev_done);
    if (c->hflag) (void)hipHostFree(c->hflag);
    delete c;
    return WSC_OK;
}

int wsc_dev_alloc(wsc_ctx* c, uint64_t bytes, void** out) {
    if (!c || !out) return fail(WSC_E_INVAL, "NULL argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMalloc(out, bytes ? bytes : 16));
    return WSC_OK;
}
int wsc_dev_free(wsc_ctx* c, void* p) {
    if (!c) return fail(WSC_E_INVAL, "NULL ctx");
    HIP_TRY(hipSetDevice(c->device));
    if (p) HIP_TRY(hipFree(p));
    return WSC_OK;
}
int wsc_host_alloc(uint64_t bytes, void** out) {
    if (!out) return fail(WSC_E_INVAL, "NULL out");
    HIP_TRY(hipHostMalloc(out, bytes ? bytes : 16, hipHostMallocDefault));
    return WSC_OK;
}
int wsc_host_free(void* p) {
    if (p) HIP_TRY(hipHostFree(p));
    return WSC_OK;
}

// the address a kernel uses for p: device memory as is, pinned host memory through its device
// mapping; nullptr for memory the device cannot reach (pageable host memory would fault the GPU)
static const void* device_view(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) return p;
    if (a.type == hipMemoryTypeHost) {   // (offset from the reported host address: interior pointers)
        if (!a.devicePointer) return p;
        if (!a.hostPointer) return a.devicePointer;
        return static_cast<const uint8_t*>(a.devicePointer) + (static_cast<const uint8_t*>(p) - static_cast<const uint8_t*>(a.hostPointer));
    }
    return nullptr;
}

int wsc_kcopy(wsc_ctx* c, void* dst, const void* src, uint64_t bytes, void* hip_stream) {
    if (!c || ((!dst || !src) && bytes)) return fail(WSC_E_INVAL, "NULL argument");
    if (bytes == 0) return WSC_OK;
    HIP_TRY(hipSetDevice(c->device));
    const void* dv = device_view(dst);
    const void* sv = device_view(src);
    if (!dv || !sv) return fail(WSC_E_INVAL, "wsc_kcopy: dst and src must be device memory or pinned host memory");
    dst = const_cast<void*>(dv);
    src = sv;
    const uint64_t chunks = (bytes + 15) >> 4;
    uint64_t blocks = (chunks + 4 * 256 - 1) / (4 * 256);
    if (blocks > (uint64_t)c->n_cu) blocks = (uint64_t)c->n_cu;   // one block per CU: reads in flight, not occupancy
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_kcopy, dim3((uint32_t)blocks), dim3(256), 0, static_cast<hipStream_t>(hip_stream),
                       static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), bytes);
    HIP_TRY(hipGetLastError());
    return WSC_OK;
}

// The launch sequence.  `ev` (optional, 6 pairs) brackets each stage for wsc_profile.  With
// sw != st (wsc_decode_split) the walk runs on sw and the UTF-8 check + unmask on st, joined by
// the context's events; otherwise everything runs in order on st.
// phase: 0 = the whole decode; 1 = only the walk (split: on sw, recording ev_walked); 2 = only the
// UTF-8 check + unmask (split: on st, joined to the walk only if it has not completed yet).
static int launch(wsc_ctx* c, const wsc_batch* b, hipStream_t st, hipEvent_t* ev, hipStream_t sw = nullptr,
                  bool split = false, int phase = 0) {
    const bool compact = (b->flags & WSC_F_COMPACT) != 0;
    const uint32_t n = b->n_segs;
    if (n == 0) return fail(WSC_E_INVAL, "n_segs == 0");
    if (n > c->cfg.max_segs) return fail(WSC_E_CAPACITY, "n_segs > max_segs");
    if (b->n_bytes > c->cfg.max_batch_bytes) return fail(WSC_E_CAPACITY, "n_bytes > max_batch_bytes");
    if (!b->wire || !b->seg_off || !b->state_out || !b->seg_out || !b->frames || !b->summary)
        return fail(WSC_E_INVAL, "NULL batch pointer");
    if (reinterpret_cast<uintptr_t>(b->wire) & 15) return fail(WSC_E_INVAL, "wire must be 16-byte aligned");
    if (compact && (!b->arena || !b->frame_dst)) return fail(WSC_E_INVAL, "COMPACT needs arena + frame_dst");
    if (compact && (reinterpret_cast<uintptr_t>(b->arena) & 15)) return fail(WSC_E_INVAL, "arena must be 16-byte aligned");

    WalkArgs wa{};
    wa.wire = b->wire;
    wa.n_bytes = b->n_bytes;
    wa.seg_off = b->seg_off;
    wa.n_segs = n;
    wa.frames_cap = b->frames_cap;
    wa.state_in = b->state_in;
    wa.max_frame_len = c->cfg.max_frame_len;
    wa.lb_ticket = c->lb_state;
    wa.u8info = c->u8info;
    wa.lb_rec = c->lb_rec;
    wa.lb_err = c->lb_state + 1;
    wa.dbg = c->dbg;
    wa.frames = b->frames;
    wa.spans = c->spans;
    wa.spans_cap = c->cfg.max_frames;
    wa.win_shift = ilog2(c->pieces * 1024);
    wa.tile_first = c->tile;
    wa.frame_dst = b->frame_dst;
    wa.state_out = b->state_out;
    wa.seg_out = b->seg_out;
    wa.summary = b->summary;
    wa.u8items = c->u8items;
    wa.u8items_cap = c->u8items_cap;
    // a new decode uses the other item counter (zeroed by the last decode's unmask); committed to
    // the context only once every check below has passed (round-3 ADVICE medium)
    const uint32_t par = phase != 2 ? c->u8par ^ 1u : c->u8par;
    wa.u8count = c->u8ctr + 32 * par;
    wa.u8seg = c->u8seg;
    wa.u8_inline_max = c->u8_inline_max;
    wa.sticky = c->sticky;
    wa.u8host = c->hflag;
    wa.win_flag = c->win_flag;
    wa.compact = compact ? 1u : 0u;
    wa.quad_pre = c->quad_pre ? 1u : 0u;
    wa.hdr_cache = c->hdr_cache;
    wa.stride_hint = c->stride_hint;
    wa.hdr_nt = (compact || c->hdr_nt_all) ? 1u : 0u;

    // walk geometry: the fused walk with blocks that fill the CUs once (64 lanes for up to 64
    // segments per CU, else 256), or -- for more segments than the chip holds lanes at once -- the
    // tiled walk (a persistent grid of contiguous segment ranges)
    // (phase 2 -- the staged unmask -- re-arms the look-back state of the walk phase 1 launched,
    // whose geometry followed ITS stream's CUs: recomputing it here from another stream could pick
    // fewer flags and leave stale inclusive prefixes for the next walk)
    const uint32_t mode = phase == 2 && c->walk_used ? c->walk_used : walk_mode(c, n, stream_cus(c, split ? sw : st));
    const uint32_t wnt = (mode == 64 || mode == 16 || mode == 32) ? 64u : 256u;
    const uint32_t spb = (mode == 65 || mode == 66) ? 64u : (mode == 16 || mode == 32) ? mode : wnt;   // segments per walk block
    const dim3 wblk(wnt), wgrid((n + spb - 1) / spb);
    if (phase != 2 && wgrid.x + 1 > c->max_walk_blocks)   // never index look-back state past its allocation
        return fail(WSC_E_INTERNAL, "walk geometry needs more look-back blocks than allocated");
    uint32_t rearm = 0;   // (after the launch below: the tiled walk sets walk_blocks)
    auto rec = [&](int i) {
        if (ev) (void)hipEventRecord(ev[i], st);
    };
    rec(0);
    // split: the walk reuses this context's scratch, so it waits for the context's previous unmask
    // (an event never recorded is a no-op wait)
    const hipStream_t ws = split ? sw : st;
    if (phase != 2) {
    if (const int r = fin_wait(c)) return r;
    // from here the decode's state is the context's: geometry, item-counter parity
    c->walk_used = mode;
    c->walk_blocks = wgrid.x;
    c->u8par = par;
    const bool stale = c->u8_dirty;   // the previous decode's unmask never launched: this counter is stale
    c->u8_dirty = true;
    __atomic_store_n(&c->hflag[0], 0u, __ATOMIC_RELEASE);
    c->walk_waited = false;
    if (split) HIP_TRY(hipStreamWaitEvent(ws, c->ev_done, 0));
    if (stale) {   // ... and its look-back ticket / flags were not re-armed either
        HIP_TRY(hipMemsetAsync(c->u8ctr + 32 * par, 0, sizeof(uint32_t), ws));
        HIP_TRY(hipMemsetAsync(c->lb_state, 0, (c->max_walk_blocks + 3) * sizeof(uint32_t), ws));
        HIP_TRY(hipMemsetAsync(c->lb_rec, 0, (uint64_t)c->max_walk_blocks * 8 * sizeof(uint64_t), ws));
    }
    // fused: 16 frame records per lane in LDS (segments with more frames re-walk their headers)
    if (mode == 3) {
        // tiled: a persistent grid (2 blocks per CU of the walk's stream), contiguous segment ranges
        const uint32_t nb = std::max<uint32_t>(1u, std::min<uint32_t>(2u * stream_cus(c, ws), (n + 255) / 256));
        const uint32_t per = ((n + nb - 1) / nb + 255) / 256 * 256;
        const uint32_t used = (n + per - 1) / per;
        c->walk_blocks = used;
        if (compact) hipLaunchKernelGGL((k_walk_tiled<true, 4, 256>), dim3(used), dim3(256), 0, ws, wa, per);
        else hipLaunchKernelGGL((k_walk_tiled<false, 4, 256>), dim3(used), dim3(256), 0, ws, wa, per);
    } else if (compact) {
        if (mode == 65) hipLaunchKernelGGL((k_walk_fused<true, 16, 256, 1, 64, 0>), wgrid, wblk, 0, ws, wa);
        else if (mode == 66) hipLaunchKernelGGL((k_walk_fused<true, 16, 256, 1, 64, 16>), wgrid, wblk, 0, ws, wa);
        else if (mode == 16) hipLaunchKernelGGL((k_walk_fused<true, 16, 64, 1, 16, 0>), wgrid, wblk, 0, ws, wa);
        else if (mode == 32) hipLaunchKernelGGL((k_walk_fused<true, 16, 64, 1, 32, 0>), wgrid, wblk, 0, ws, wa);
        else if (wnt == 64) hipLaunchKernelGGL((k_walk_fused<true, 16, 64, 1, 64, 0>), wgrid, wblk, 0, ws, wa);
        else if (mode == 257) hipLaunchKernelGGL((k_walk_fused<true, 4, 256, 1, 256, 0>), wgrid, wblk, 0, ws, wa);
        else hipLaunchKernelGGL((k_walk_fused<true, 16, 256, 1, 256, 0>), wgrid, wblk, 0, ws, wa);
    } else {
        if (mode == 65) hipLaunchKernelGGL((k_walk_fused<false, 16, 256, 1, 64, 0>), wgrid, wblk, 0, ws, wa);
        else if (mode == 66) hipLaunchKernelGGL((k_walk_fused<false, 16, 256, 1, 64, 16>), wgrid, wblk, 0, ws, wa);
        else if (mode == 16) hipLaunchKernelGGL((k_walk_fused<false, 16, 64, 1, 16, 0>), wgrid, wblk, 0, ws, wa);
        else if (mode == 32) hipLaunchKernelGGL((k_walk_fused<false, 16, 64, 1, 32, 0>), wgrid, wblk, 0, ws, wa);
        else if (wnt == 64) hipLaunchKernelGGL((k_walk_fused<false, 16, 64, 1, 64, 0>), wgrid, wblk, 0, ws, wa);
        else if (mode == 257) hipLaunchKernelGGL((k_walk_fused<false, 4, 256, 1, 256, 0>), wgrid, wblk, 0, ws, wa);
        else hipLaunchKernelGGL((k_walk_fused<false, 16, 256, 1, 256, 0>), wgrid, wblk, 0, ws, wa);
    }
    HIP_TRY(hipGetLastError());
    if (split) HIP_TRY(hipEventRecord(c->ev_walked, ws));
    }   // phase != 2
    if (phase == 1) return WSC_OK;
    // look-back flags the walk used: ticket, timeout, flags
    rearm = c->walk_blocks + 1;
    // a stream wait is a barrier packet between this unmask and the previous one on st: skipped
    // when the host already knows the walk has finished (the staged pipeline waits for it)
    const bool walked = split && (c->walk_waited || hipEventQuery(c->ev_walked) == hipSuccess);
    c->walk_waited = false;
    if (split && !walked) HIP_TRY(hipStreamWaitEvent(st, c->ev_walked, 0));
    rec(1);
    // deferred UTF-8 (large text) runs after the unmask (which folds the text windows it unmasks):
    // both the fold and the check are skipped when the walk has completed and its host-visible
    // flag says it deferred nothing -- the check would still be a launch between two unmasks
    const bool need_u8 = !(walked && __atomic_load_n(&c->hflag[0], __ATOMIC_ACQUIRE) == 0);
    const bool signal = phase == 2;   // staged: the decode's last kernel signals the host, no ev_done

    uint8_t* udst = compact ? b->arena : b->wire;
    const uint64_t wb = (uint64_t)c->pieces * 1024;
    const uint64_t n_win = (b->n_bytes + wb - 1) / wb;
    // one wire window per wave (both modes read the wire window by window, wsc_unmask.inl)
    uint64_t waves = c->cfg.unmask_waves_per_cu ? (uint64_t)c->n_cu * c->cfg.unmask_waves_per_cu : n_win;
    if (waves > n_win) waves = n_win;
    if (waves == 0) waves = 1;
    const dim3 ublk(256), ugrid((uint32_t)((waves + 3) / 4));
    using UK = void (*)(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*,
                        const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
    // [U8 fold][compact]: 4 KiB windows; in place through buffer ops with nt loads and sc0 nt sc1
    // stores (NT = 307), COMPACT with nt loads and default-policy stores (NT = 1)
    static const UK table[2][2] = {{k_unmask<false, 4, 307, 1, false>, k_unmask<true, 4, 1, 1, false>},
                                   {k_unmask<false, 4, 307, 1, true>, k_unmask<true, 4, 1, 1, true>}};
    const int ui = need_u8 ? 1 : 0;
    const UK kern = table[ui][compact ? 1 : 0];
    const bool sig_unmask = signal && !need_u8;
    U8Win uw{};
    uw.rearm = c->u8ctr + 32 * (c->u8par ^ 1u);
    uw.xcd_run = c->xcd_run;
    uw.lb_rec = c->lb_rec;
    if (need_u8) {
        uw.flag = c->win_flag;
        uw.map = c->win_map;
        uw.count = c->u8ctr + 32 * c->u8par;
    }
    hipLaunchKernelGGL(kern, ugrid, ublk, 0, st, udst, (const uint8_t*)b->wire, b->n_bytes, b->n_bytes,
                       (const Span*)c->spans, (const uint32_t*)c->tile, (const wsc_summary*)b->summary,
                       c->lb_state, rearm,   // re-arms ticket, timeout, flags
                       sig_unmask ? c->fin_ctr : nullptr, sig_unmask ? c->hflag + 1 : nullptr, c->fin_seq + 1, uw);
    HIP_TRY(hipGetLastError());
    c->u8_dirty = false;   // the next decode's counter is zeroed by this unmask
    rec(2);
    if (need_u8) {
        U8Args ua{};
        ua.wire = b->wire;
        ua.n_bytes = b->n_bytes;
        ua.seg_off = b->seg_off;
        ua.items = c->u8items;
        ua.count = c->u8ctr + 32 * c->u8par;
        ua.items_cap = c->u8items_cap;
        ua.maps = c->u8maps;
        ua.seg = c->u8seg;
        ua.frames = b->frames;
        ua.spans = c->spans;
        ua.seg_out = b->seg_out;
        ua.state_out = b->state_out;
        ua.summary = b->summary;
        ua.win_map = c->win_map;
        ua.win_shift = ilog2(c->pieces * 1024);
        ua.unmasked = compact ? 0u : 1u;
        ua.out = udst;
        ua.n_segs = n;
        ua.fin_ctr = c->fin_ctr;
        ua.fin_host = signal ? c->hflag + 1 : nullptr;
        ua.fin_seq = c->fin_seq + 1;
        const dim3 ug((uint32_t)c->n_cu * 4);   // resident: 4 waves/SIMD (128 VGPRs; 3 waves/SIMD without
        // the large path's spills measured slower: 64 KiB TEXT check 79 -> 95 us)
        hipLaunchKernelGGL((k_u8_check<4, 4>), ug, dim3(256), 0, st, ua);
        HIP_TRY(hipGetLastError());
    }
    rec(3);
    rec(4);
    if (signal) {
        ++c->fin_seq;
        c->fin_pending = true;
        c->fin_stream = st;
    } else if (split) {
        HIP_TRY(hipEventRecord(c->ev_done, st));
    }
    rec(5);
    return WSC_OK;
}

int wsc_decode(wsc_ctx* c, const wsc_batch* b, void* hip_stream) {
    if (!c || !b) return fail(WSC_E_INVAL, "NULL argument");
    HIP_TRY(hipSetDevice(c->device));
    // like every HIP API: NULL is the default (null) stream
    return launch(c, b, static_cast<hipStream_t>(hip_stream), nullptr);
}

int wsc_decode_split(wsc_ctx* c, const wsc_batch* b, void* walk_stream, void* unmask_stream) {
    if (!c || !b) return fail(WSC_E_INVAL, "NULL argument");
    if (walk_stream == unmask_stream) return fail(WSC_E_INVAL, "walk_stream == unmask_stream: use wsc_decode");
    HIP_TRY(hipSetDevice(c->device));
    return launch(c, b, static_cast<hipStream_t>(unmask_stream), nullptr, static_cast<hipStream_t>(walk_stream), true);
}

int wsc_decode_walk(wsc_ctx* c, const wsc_batch* b, void* walk_stream) {
    if (!c || !b) return fail(WSC_E_INVAL, "NULL argument");
    HIP_TRY(hipSetDevice(c->device));
    return launch(c, b, nullptr, nullptr, static_cast<hipStream_t>(walk_stream), true, 1);
}

int wsc_decode_finish(wsc_ctx* c, const wsc_batch* b, void* unmask_stream) {
    if (!c || !b) return fail(WSC_E_INVAL, "NULL argument");
    HIP_TRY(hipSetDevice(c->device));
    return launch(c, b, static_cast<hipStream_t>(unmask_stream), nullptr, nullptr, true, 2);
}

int wsc_walk_wait(wsc_ctx* c) {
    if (!c) return fail(WSC_E_INVAL, "NULL ctx");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipEventSynchronize(c->ev_walked));
    c->walk_waited = true;
    return WSC_OK;
}

int wsc_stream_create(wsc_ctx* c, const uint32_t* cu_mask, uint32_t mask_words, void** out) {
    if (!c || !out) return fail(WSC_E_INVAL, "NULL argument");
    *out = nullptr;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = nullptr;
    if (cu_mask && mask_words) {
        HIP_TRY(hipExtStreamCreateWithCUMask(&s, mask_words, cu_mask));
        uint32_t cus = 0;
        for (uint32_t w = 0; w < mask_words; ++w) cus += (uint32_t)__builtin_popcount(cu_mask[w]);
        if (cus > (uint32_t)c->n_cu) cus = (uint32_t)c->n_cu;
        std::lock_guard<std::mutex> lk(g_stream_mu);
        g_stream_cus[s] = cus ? cus : 1u;
    } else {
        HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
    *out = s;
    return WSC_OK;
}

int wsc_stream_create_ex(wsc_ctx* c, const uint32_t* cu_mask, uint32_t mask_words, int priority, void** out) {
    if (!c || !out) return fail(WSC_E_INVAL, "NULL argument");
    if (priority == 0) return wsc_stream_create(c, cu_mask, mask_words, out);
    if (cu_mask && mask_words) return fail(WSC_E_INVAL, "a CU-masked stream has the default priority");
    *out = nullptr;
    HIP_TRY(hipSetDevice(c->device));
    int least = 0, greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority > 0 ? greatest : least));
    *out = s;
    return WSC_OK;
}

int wsc_stream_destroy(wsc_ctx* c, void* stream) {
    if (!c) return fail(WSC_E_INVAL, "NULL ctx");
    HIP_TRY(hipSetDevice(c->device));
    if (stream) {
        {
            std::lock_guard<std::mutex> lk(g_stream_mu);
            g_stream_cus.erase(static_cast<hipStream_t>(stream));
        }
        HIP_TRY(hipStreamDestroy(static_cast<hipStream_t>(stream)));
    }
    return WSC_OK;
}

int wsc_sync(wsc_ctx* c, void* hip_stream) {
    if (!c) return fail(WSC_E_INVAL, "NULL ctx");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(hip_stream)));
    return WSC_OK;
}

int wsc_decode_host(wsc_ctx* c, uint8_t* wire, uint64_t n_bytes, const uint64_t* seg_off,
                    uint32_t n_segs, uint32_t flags, const wsc_conn_state* state_in,
                    wsc_conn_state* state_out, wsc_seg_result* seg_out, wsc_frame* frames,
                    uint32_t frames_cap, uint8_t* arena, uint64_t* frame_dst, wsc_summary* summary) {
    if (!c || !wire || !seg_off || !state_out || !seg_out || !frames || !summary)
        return fail(WSC_E_INVAL, "NULL argument");
    const bool compact = (flags & WSC_F_COMPACT) != 0;
    if (compact && (!arena || !frame_dst)) return fail(WSC_E_INVAL, "COMPACT needs arena + frame_dst");
    if (n_segs == 0 || n_segs > c->cfg.max_segs) return fail(WSC_E_CAPACITY, "n_segs out of range");
    if (n_bytes > c->cfg.max_batch_bytes) return fail(WSC_E_CAPACITY, "n_bytes > max_batch_bytes");
    HIP_TRY(hipSetDevice(c->device));
    int rc = alloc_host_path(c);
    if (rc) return rc;
    const uint32_t cap = frames_cap < c->cfg.max_frames ? frames_cap : c->cfg.max_frames;
    hipStream_t st = c->stream;
    HIP_TRY(hipMemcpyAsync(c->d_wire, wire, n_bytes, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(c->d_seg_off, seg_off, (n_segs + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    if (state_in)
        HIP_TRY(hipMemcpyAsync(c->d_state_in, state_in, n_segs * sizeof(wsc_conn_state), hipMemcpyHostToDevice, st));
    wsc_batch b{};
    b.wire = c->d_wire;
    b.n_bytes = n_bytes;
    b.seg_off = c->d_seg_off;
    b.n_segs = n_segs;
    b.flags = flags;
    b.state_in = state_in ? c->d_state_in : nullptr;
    b.state_out = c->d_state_out;
    b.seg_out = c->d_seg_out;
    b.frames = c->d_frames;
    b.frames_cap = cap;
    b.arena = compact ? c->d_arena : nullptr;
    b.frame_dst = compact ? c->d_frame_dst : nullptr;
    b.summary = c->d_summary;
    rc = launch(c, &b, st, nullptr);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(summary, c->d_summary, sizeof(wsc_summary), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const uint32_t nf = summary->n_frames < cap ? summary->n_frames : cap;
    HIP_TRY(hipMemcpyAsync(state_out, c->d_state_out, n_segs * sizeof(wsc_conn_state), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(seg_out, c->d_seg_out, n_segs * sizeof(wsc_seg_result), hipMemcpyDeviceToHost, st));
    if (nf) HIP_TRY(hipMemcpyAsync(frames, c->d_frames, (uint64_t)nf * sizeof(wsc_frame), hipMemcpyDeviceToHost, st));
    if (compact) {
        const uint64_t ab = summary->data_bytes + summary->ctrl_bytes;
        if (ab) HIP_TRY(hipMemcpyAsync(arena, c->d_arena, ab, hipMemcpyDeviceToHost, st));
        if (nf) HIP_TRY(hipMemcpyAsync(frame_dst, c->d_frame_dst, (uint64_t)nf * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    } else if (n_bytes) {
        HIP_TRY(hipMemcpyAsync(wire, c->d_wire, n_bytes, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    return wsc_summary_status(summary);
}

int wsc_summary_status(const wsc_summary* summary) {
    if (!summary) return fail(WSC_E_INVAL, "NULL summary");
    if (summary->overflow & 2u) return fail(WSC_E_INTERNAL, "device look-back timeout: batch results are invalid");
    if (summary->overflow & 1u) return fail(WSC_E_CAPACITY, "frame capacity exceeded: records beyond frames_cap dropped");
    return WSC_OK;
}

int wsc_error_flags(wsc_ctx* c, uint32_t* flags, int clear) {
    if (!c || !flags) return fail(WSC_E_INVAL, "NULL argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(flags, c->sticky, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (clear) HIP_TRY(hipMemset(c->sticky, 0, sizeof(uint32_t)));
    return WSC_OK;
}

// ---- encode ---------------------------------------------------------------------------------
// messages per scan thread: the smallest of 1 / 4 / ENC_IPT that keeps the scan within 256 blocks
// (one per CU)
static uint32_t enc_scan_ipt(uint32_t n) {
    if (n <= 256u * 256u) return 1;
    if (n <= 256u * 256u * 4u) return 4;
    return ENC_IPT;
}

static int launch_encode(wsc_ctx* c, const wsc_out_msg* msgs, uint32_t n, const uint8_t* src, uint64_t src_bytes,
                         uint8_t* out, uint64_t out_cap, uint64_t* out_off, hipStream_t st) {
    if (!msgs || !out || !out_off || (!src && src_bytes)) return fail(WSC_E_INVAL, "NULL encode pointer");
    if (n > c->cfg.max_frames) return fail(WSC_E_CAPACITY, "n_msgs > max_frames");
    if (out_cap > c->enc_cap) return fail(WSC_E_CAPACITY, "out_cap > max_batch_bytes + 16 * max_frames");
    if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(out)) & 15)
        return fail(WSC_E_INVAL, "src and out must be 16-byte aligned");
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(out_off, 0, sizeof(uint64_t), st));
        return WSC_OK;
    }
    EncArgs ea{};
    ea.msgs = msgs;
    ea.n_msgs = n;
    ea.out_off = out_off;
    ea.tile = c->enc_tile;
    ea.tile_entries = c->enc_tile_entries;
    ea.lb_ticket = c->enc_lb_state;
    ea.lb_err = c->enc_lb_state + 1;
    ea.lb_rec = c->enc_lb_rec;
    ea.sticky = c->sticky;
    const uint32_t ipt = enc_scan_ipt(n);
    const uint32_t sblocks = (n + 256 * ipt - 1) / (256 * ipt);
    if (ipt == 1) hipLaunchKernelGGL(k_encode_scan<1>, dim3(sblocks), dim3(256), 0, st, ea);
    else if (ipt == 4) hipLaunchKernelGGL(k_encode_scan<4>, dim3(sblocks), dim3(256), 0, st, ea);
    else hipLaunchKernelGGL(k_encode_scan<16>, dim3(sblocks), dim3(256), 0, st, ea);
    HIP_TRY(hipGetLastError());
    EncCopyArgs ca{};
    ca.msgs = msgs;
    ca.n_msgs = n;
    ca.out_off = out_off;
    ca.src = src;
    ca.src_bytes = src_bytes;
    ca.out = out;
    ca.out_cap = out_cap;
    ca.tile = c->enc_tile;
    ca.tile_entries = c->enc_tile_entries;
    ca.lb_state = c->enc_lb_state;
    ca.lb_rec = c->enc_lb_rec;
    ca.n_lb = sblocks + 2;
    ca.xcd_run = c->enc_xcd_run;
    // small messages (src bytes per message < two windows): most windows hold frame edges
    ca.hoist = src_bytes < (uint64_t)n * 2 * ENC_WIN ? 1u : 0u;
    uint64_t wins = (out_cap + ENC_WIN - 1) / ENC_WIN;   // the grid covers out_cap; waves past the total exit
    if (wins > c->enc_tile_entries) wins = c->enc_tile_entries;
    if (wins == 0) wins = 1;
    const dim3 cgrid((uint32_t)((wins + 3) / 4));
    hipLaunchKernelGGL(k_encode_copy<3>, cgrid, dim3(256), 0, st, ca);   // nt loads and stores
    HIP_TRY(hipGetLastError());
    return WSC_OK;
}

int wsc_encode(wsc_ctx* c, const wsc_out_msg* msgs, uint32_t n_msgs, const uint8_t* src, uint64_t src_bytes,
               uint8_t* out, uint64_t out_cap, uint64_t* out_off, void* hip_stream) {
    if (!c) return fail(WSC_E_INVAL, "NULL ctx");
    HIP_TRY(hipSetDevice(c->device));
    return launch_encode(c, msgs, n_msgs, src, src_bytes, out, out_cap, out_off, static_cast<hipStream_t>(hip_stream));
}

int wsc_encode_host(wsc_ctx* c, const wsc_out_msg* msgs, uint32_t n_msgs, const uint8_t* src, uint64_t src_bytes,
                    uint8_t* out, uint64_t out_cap, uint64_t* out_off) {
    if (!c || !msgs || !out || !out_off || (!src && src_bytes)) return fail(WSC_E_INVAL, "NULL argument");
    if (n_msgs > c->cfg.max_frames) return fail(WSC_E_CAPACITY, "n_msgs > max_frames");
    if (src_bytes > c->cfg.max_batch_bytes) return fail(WSC_E_CAPACITY, "src_bytes > max_batch_bytes");
    HIP_TRY(hipSetDevice(c->device));
    if (!c->d_enc_msgs) {
        HIP_TRY(hipMalloc(&c->d_enc_msgs, (uint64_t)c->cfg.max_frames * sizeof(wsc_out_msg)));
        HIP_TRY(hipMalloc(&c->d_enc_src, c->cfg.max_batch_bytes + 64));
        HIP_TRY(hipMalloc(&c->d_enc_out, c->enc_cap + 64));
        HIP_TRY(hipMalloc(&c->d_enc_off, ((uint64_t)c->cfg.max_frames + 1) * sizeof(uint64_t)));
    }
    const uint64_t cap = out_cap < c->enc_cap ? out_cap : c->enc_cap;
    hipStream_t st = c->stream;
    if (n_msgs) HIP_TRY(hipMemcpyAsync(c->d_enc_msgs, msgs, (uint64_t)n_msgs * sizeof(wsc_out_msg), hipMemcpyHostToDevice, st));
    if (src_bytes) HIP_TRY(hipMemcpyAsync(c->d_enc_src, src, src_bytes, hipMemcpyHostToDevice, st));
    int rc = launch_encode(c, c->d_enc_msgs, n_msgs, c->d_enc_src, src_bytes, c->d_enc_out, cap, c->d_enc_off, st);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out_off, c->d_enc_off, ((uint64_t)n_msgs + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const uint64_t total = out_off[n_msgs];
    if (total == ~0ull) return fail(WSC_E_INTERNAL, "device look-back timeout in the encode scan: output invalid");
    if (total > out_cap) return fail(WSC_E_CAPACITY, "encoded frames exceed out_cap");
    if (total) HIP_TRY(hipMemcpyAsync(out, c->d_enc_out, total, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return WSC_OK;
}

int wsc_profile(wsc_ctx* c, const wsc_batch* b, int iters, double* out_ms) {
    if (!c || !b || !out_ms || iters <= 0) return fail(WSC_E_INVAL, "bad argument");
    HIP_TRY(hipSetDevice(c->device));
    hipEvent_t ev[6];
    for (auto& e : ev) HIP_TRY(hipEventCreate(&e));
    double acc[6] = {0, 0, 0, 0, 0, 0};
    int rc = WSC_OK;
    for (int it = 0; it < iters && rc == WSC_OK; ++it) {
        rc = launch(c, b, c->stream, ev);
        if (rc) break;
        if (hipStreamSynchronize(c->stream) != hipSuccess) { rc = fail(WSC_E_DEVICE, "sync"); break; }
        for (int k = 0; k < 5; ++k) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, ev[k], ev[k + 1]);
            acc[k] += ms;
        }
        float tot = 0;
        (void)hipEventElapsedTime(&tot, ev[0], ev[5]);
        acc[5] += tot;
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    for (int k = 0; k < 6; ++k) out_ms[k] = acc[k] / iters;
    return rc;
}

int wsc_debug_stamps(wsc_ctx* c, uint64_t* out, uint32_t max_blocks) {
    if (!c || !out) return fail(WSC_E_INVAL, "NULL argument");
    if (!c->dbg) return fail(WSC_E_STATE, "context created without WSC_WALK_DEBUG_STAMPS");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    if (max_blocks > c->max_walk_blocks) max_blocks = c->max_walk_blocks;
    HIP_TRY(hipMemcpy(out, c->dbg, (uint64_t)max_blocks * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return WSC_OK;
}

int wsc_walk_info(wsc_ctx* c, uint32_t* mode, uint32_t* blocks) {
    if (!c || !mode || !blocks) return fail(WSC_E_INVAL, "NULL argument");
    *mode = c->walk_used;
    *blocks = c->walk_blocks;
    return WSC_OK;
}

}  // extern "C"
