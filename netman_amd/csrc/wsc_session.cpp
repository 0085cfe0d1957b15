// wsc_session.cpp -- C++ host side above the ABI: the per-connection DecodePacket() mirror.
//
// In netman every poller goroutine calls conn.DecodePacket() once per readiness event
// (eventloop/epoll.go:105) and gets back at most one (IMessage, error) (server/websocket.go:82-212).
// Here a poller instead reads each ready connection ONCE, straight into pinned staging
// (wsc_session_reserve + recv + wsc_session_commit, or wsc_session_feed), runs ONE batched device
// decode over all of them (wsc_session_submit / wsc_session_complete, or wsc_session_decode =
// both), and then drains each connection's results one at a time with wsc_session_next(), which
// returns exactly what the reference's DecodePacket + epoll.go:104-140 would have produced:
//   WSC_EV_MESSAGE  (Message, nil)          -> IWebsocketHandler.Message   (routermgr.go:101)
//   WSC_EV_PONG     pong() echo             -> push(encode(0x8A, payload)) (websocket_ctrl.go:128-153)
//   WSC_EV_CLOSE    CloseCode(code)         -> epoll.go:106-129 mapping of the sentinel
//   WSC_EV_STALL    unmasked frame (Q3)     -> nothing more is delivered
//   WSC_EV_NONE     (nil, syscall.EAGAIN)
//
// Data path (per poller round): socket -> pinned staging (the one host copy, done by recv) -> H2D
// (a kernel reading the staging over PCIe, wsc_kcopy: a hipMemcpyAsync held the poller thread for
// the copy) -> header walk + unmask (HBM) -> D2H into a pinned result buffer -> messages handed
// out as views into it, valid until the next complete (a server can send replies straight from
// them).  Two staging sets, each with its own device context and HIP stream, so round r+1's
// H2D + kernels run while the poller sends round r's replies (submit/complete).  A connection's
// undecoded tail (an incomplete frame) is kept on the host (Conn::carry) and placed in front of
// its next bytes.
//
// Capacity is handled per connection, never per session (one connection cannot stall the others):
//   * payloads stream: a data frame whose header is in a batch is unmasked piece by piece as its
//     bytes arrive (WSC_FK_PIECE records, the connection's device state carries the rest of the
//     frame, never its bytes); the pieces collect in Conn::rbuf -- nextFrame's rBuffer,
//     websocket_frame.go:16-31 -- and the message is delivered when its last piece decodes, so a
//     frame of any size up to max_frame_len passes through batches of any size;
//   * a connection whose bytes do not fit the batch is decoded from a prefix (it always leads a
//     batch then) and the rest follows in the next batch;
//   * a batch whose frame records exceed max_frames is re-decoded in halves (one connection: a
//     prefix ending at a frame boundary the device reported).
// Device failure policy (the reference drops a poller's connections when epoll_wait
// fails, eventloop/epoll.go:41-49): the connections of the failed batch get WSC_EV_CLOSE with
// close_code 1011 and err WSC_ERR_DEVICE, keep their carried bytes (wsc_session_state), and
// decode nothing more; the other connections are untouched; the call returns the error.  There
// is no CPU fallback.
// Threading: wsc_session_remove may be called from ANY thread at any time (netman's handler and
// heartbeat goroutines call Close() -> remove(), websocket_ctrl.go:73-96); it only queues the
// handle, and the poller thread applies queued removals at its next session call.  Every other
// function belongs to the one poller thread that owns the session.
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/wscodec.h"

namespace wsc {
int set_last_error(int code, const std::string& msg);   // wsc_api.cpp: the wsc_last_error() text
}

namespace {

constexpr uint32_t SLOT_BITS = 22;                  // handle = slot | generation << 22
constexpr uint32_t SLOT_MASK = (1u << SLOT_BITS) - 1;
constexpr uint32_t GEN_MASK = (1u << (32 - SLOT_BITS)) - 1;
constexpr uint32_t DEAD_SEG = 0xFFFFFFFFu;          // staging region of no connection (decodes nothing)
constexpr uint64_t MIN_RESERVE = 64 << 10;          // staging room worth handing to recv()

struct Event {
    wsc_event ev;
    std::vector<uint8_t> data;     // owned copy (fragmented messages, materialised views)
    const uint8_t* view = nullptr; // zero-copy: points into a staging set's pinned result buffer
    uint64_t view_len = 0;
    int set = -1;                  // staging set of the view
};

struct Conn {
    bool live = false;
    uint32_t gen = 0;
    wsc_conn_state st{};
    std::vector<uint8_t> carry;   // undecoded tail of earlier reads (starts at a frame header), masked
    std::vector<uint8_t> spill;   // bytes fed while they did not fit the staging being filled
    std::vector<uint8_t> cont;    // continueBuffer (unmasked fragments so far)
    std::vector<uint8_t> rbuf;    // rBuffer: the unmasked pieces of the frame still arriving
    std::deque<Event> pending;
    Event current;                // storage for the event last returned by next()
    uint64_t fill_epoch = ~0ull;  // == session fill_epoch while placed in the staging being filled
    uint32_t seg = 0;             // its segment there
    uint64_t reserved = 0;        // bytes handed out by the last reserve (0 = none)
    bool reserved_spill = false;
    bool failed = false;          // its batch hit a device error (WSC_ERR_DEVICE)
    bool in_flight = false;       // has a segment in the submitted batch: new bytes wait in the
                                  // spill until complete() has set the carry they must follow
    bool eof = false;             // the peer closed (a read returned 0): once every byte read before it
                                  // is decoded, the last event is Close() (baseconnect.go:100-103,
                                  // epoll.go:108-110)
};

struct Stage {                    // one staging set: pinned host buffers, device buffers, context
    wsc_ctx* ctx = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev = nullptr;      // WSC_SESSION_BLOCKING_WAIT: a blocking-sync event complete() sleeps on
    hipEvent_t done_ev = nullptr; // recorded after the launch's last operation: wsc_session_ready
    uint32_t frames_pre = 0;      // frame records already copied back with the launch (launch_stage)
    uint8_t* h_wire = nullptr;    // masked bytes as read (input)
    uint8_t* h_res = nullptr;     // results: unmasked wire (in place) or the arena (COMPACT)
    uint64_t* h_seg_off = nullptr;
    wsc_conn_state* h_state_in = nullptr;
    wsc_conn_state* h_state_out = nullptr;
    wsc_seg_result* h_seg_out = nullptr;
    wsc_frame* h_frames = nullptr;
    uint64_t* h_frame_dst = nullptr;
    wsc_summary* h_summary = nullptr;
    void* d_wire = nullptr;
    void* d_arena = nullptr;
    void* d_seg_off = nullptr;
    void* d_state_in = nullptr;
    void* d_state_out = nullptr;
    void* d_seg_out = nullptr;
    void* d_frames = nullptr;
    void* d_frame_dst = nullptr;
    void* d_summary = nullptr;
    // the batch being filled / in flight
    uint64_t bytes = 0;
    std::vector<uint32_t> seg_conn;   // handle per segment (DEAD_SEG: a region nobody owns)
    std::vector<uint64_t> seg_start;
    std::vector<uint64_t> seg_len;
    std::vector<uint8_t> done;        // segment harvested (complete)
    bool in_flight = false;
    int launch_rc = WSC_OK;
    std::vector<uint32_t> view_conns; // slots holding zero-copy views into h_res
};

uint32_t close_code_for(uint32_t err) {   // eventloop/epoll.go:106-129
    return err == WSC_ERR_MUST_UTF8 ? 1007u : 1002u;
}

void push_close(Conn& c, uint32_t code, uint32_t err) {
    Event e;
    std::memset(&e.ev, 0, sizeof(e.ev));
    e.ev.type = WSC_EV_CLOSE;
    e.ev.close_code = code;
    e.ev.err = err;
    c.pending.push_back(std::move(e));
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct wsc_session {
    wsc_config cfg{};
    uint32_t flags = 0;
    int device = 0;
    std::vector<Conn> conns;
    std::vector<uint32_t> free_slots;
    std::atomic<uint32_t> n_slots{0};
    Stage st[2];
    int fill = 0;                 // staging set being filled
    uint64_t fill_epoch = 1;
    // removals queued by any thread, applied by the poller thread
    std::mutex rm_mu;
    std::vector<uint32_t> rm_q;
    std::atomic<uint32_t> rm_pending{0};
    // test hook (wsc_session_inject_fault): the fault_at-th device batch fails as a device error would
    uint64_t fault_at = 0, n_submits = 0;
    // WSC_SESSION_TIMING: seconds per phase, printed at destroy
    bool timing = false;
    int kcopy = 1;                // staging copies by wsc_kcopy: 1 the wire's H2D (default), 2 all
                                  // (WSC_SESSION_KCOPY_ALL), 0 none (WSC_SESSION_COPY_ENGINE).  At 2 the small copies
                                  // queue as kernels behind other pollers' decodes on the shared
                                  // compute queues (profiles/r05/ab11_echo_*: 4 pollers, 512 KiB
                                  // reads 4.24 -> 3.02 GiB/s), so they stay on the copy engines
    std::vector<std::vector<uint8_t>> retired;   // owned event bytes handed out this round (wsc_session_next)
    double t_pack = 0, t_launch = 0, t_device = 0, t_harvest = 0;
    double t_lh2d = 0, t_ldec = 0;   // parts of t_launch: the H2D enqueues, the decode's launches
    uint64_t n_batches = 0, n_bytes = 0;
    // wsc_session_stats: bytes read, sent to the device, of those sent again (carried), batches,
    // streamed payload bytes collected into messages
    uint64_t st_read = 0, st_h2d = 0, st_resent = 0, st_batches = 0, st_pieces = 0;
    uint64_t max_message = 0;     // wsc_session_set_max_message: 0 = no cap (the reference has none, Q4)
    uint32_t frames_hint = 0;     // records of the last batch (+1/8): how many the next launch copies back up front
};

namespace {

Conn* lookup(wsc_session* s, uint32_t h) {
    const uint32_t slot = h & SLOT_MASK;
    if (slot >= s->conns.size()) return nullptr;
    Conn& c = s->conns[slot];
    if (!c.live || c.gen != (h >> SLOT_BITS)) return nullptr;
    return &c;
}

void kill_conn(wsc_session* s, uint32_t slot) {
    Conn& c = s->conns[slot];
    const uint32_t gen = c.gen;
    Stage& f = s->st[s->fill];
    if (c.fill_epoch == s->fill_epoch && c.seg < f.seg_conn.size()) f.seg_conn[c.seg] = DEAD_SEG;
    c = Conn();
    c.gen = gen;   // the next open() of this slot bumps it
    s->free_slots.push_back(slot);
}

// websocket_ctrl.go:73-96 remove(): applied on the poller thread
void apply_removes(wsc_session* s) {
    if (!s->rm_pending.load(std::memory_order_acquire)) return;
    std::vector<uint32_t> q;
    {
        std::lock_guard<std::mutex> g(s->rm_mu);
        q.swap(s->rm_q);
        s->rm_pending.store(0, std::memory_order_relaxed);
    }
    for (uint32_t h : q)
        if (lookup(s, h)) kill_conn(s, h & SLOT_MASK);
}

void materialize_views(wsc_session* s, int set) {
    Stage& g = s->st[set];
    for (uint32_t slot : g.view_conns) {
        if (slot >= s->conns.size()) continue;
        for (Event& e : s->conns[slot].pending)
            if (e.view && e.set == set) {
                e.data.assign(e.view, e.view + e.view_len);
                e.view = nullptr;
                e.set = -1;
            }
    }
    g.view_conns.clear();
}

// place connection c (its carry first) in the staging being filled, with room for `extra` more
// bytes; false if the staging cannot host it now
bool place(wsc_session* s, Conn& c, uint32_t handle, uint64_t extra) {
    Stage& f = s->st[s->fill];
    const wsc_config& g = s->cfg;
    if (c.fill_epoch == s->fill_epoch) return true;
    const uint64_t need = c.carry.size() + c.spill.size() + extra;
    if (f.bytes + need > g.max_batch_bytes && f.bytes > 0) return false;
    if (f.seg_conn.size() + 2 > g.max_segs) return false;   // keep one slot for a dead region
    if (need > g.max_batch_bytes) {
        // only a batch's first connection may exceed it: it is decoded from a prefix (below)
        if (f.bytes > 0) return false;
    }
    uint64_t n = c.carry.size() + c.spill.size();
    if (n > g.max_batch_bytes) n = g.max_batch_bytes;   // prefix (carry first, at most one frame)
    c.seg = (uint32_t)f.seg_conn.size();
    f.seg_conn.push_back(handle);
    f.seg_start.push_back(f.bytes);
    uint64_t k = 0;
    const uint64_t kc = c.carry.size() < n ? c.carry.size() : n;
    if (kc) std::memcpy(f.h_wire + f.bytes, c.carry.data(), kc);
    s->st_resent += kc;   // an incomplete header / control frame goes over PCIe again
    k = kc;
    if (k < n) {
        const uint64_t ks = n - k;
        std::memcpy(f.h_wire + f.bytes + k, c.spill.data(), ks);
        k += ks;
    }
    // what was copied leaves carry/spill (a prefix leaves the rest behind, in order)
    if (kc) c.carry.erase(c.carry.begin(), c.carry.begin() + (long)kc);
    if (k > kc) c.spill.erase(c.spill.begin(), c.spill.begin() + (long)(k - kc));
    if (!c.carry.empty()) {   // prefix cut inside the carry: keep order carry -> spill
        c.spill.insert(c.spill.begin(), c.carry.begin(), c.carry.end());
        c.carry.clear();
    }
    f.seg_len.push_back(n);
    f.bytes += n;
    c.fill_epoch = s->fill_epoch;
    return true;
}

// turn one segment's frame records into the DecodePacket results the reference would return
void harvest(wsc_session* s, int set, Conn& c, uint32_t slot, const uint8_t* in_seg, const uint8_t* res_base,
             uint64_t seg_len, const wsc_seg_result& r, const wsc_conn_state& so,
             const wsc_frame* frames, const uint64_t* frame_dst, uint64_t arena_base) {
    const bool compact = (s->flags & WSC_F_COMPACT) != 0;
    bool views = false;
    // wsc_session_set_max_message: a message (or the fragments / pieces of one) past the cap closes
    // the connection with 1009 instead of buffering it (off by default: the reference buffers any size)
    bool capped = false;
    auto over = [&](uint64_t more) {
        if (!s->max_message || c.cont.size() + c.rbuf.size() + more <= s->max_message) return false;
        push_close(c, 1009, WSC_ERR_MSG_TOO_BIG);
        capped = true;
        return true;
    };
    for (uint32_t i = r.frame_begin; i < r.frame_begin + r.frame_count && !capped; ++i) {
        const wsc_frame& f = frames[i];
        const uint64_t flen = f.payload_len | (uint64_t)f.payload_len_hi << 32;   // 40-bit length
        const uint8_t* p = compact ? res_base + arena_base + frame_dst[i] : res_base + f.hdr_off + f.hdr_len;
        Event e;
        std::memset(&e.ev, 0, sizeof(e.ev));
        switch (f.kind) {
        case WSC_FK_PIECE:                                    // websocket_frame.go:16-31 (rBuffer)
            if (f.opcode == 10) continue;                     // a PONG's bytes: discarded when complete
            if (over(flen)) continue;
            c.rbuf.insert(c.rbuf.end(), p, p + flen);
            s->st_pieces += flen;
            continue;
        case WSC_FK_FRAG:                                     // websocket_frame.go:95-98
            if (over(flen)) continue;
            if (!c.rbuf.empty()) {                            // a streamed fragment's earlier pieces
                c.cont.insert(c.cont.end(), c.rbuf.begin(), c.rbuf.end());
                c.rbuf.clear();
            }
            c.cont.insert(c.cont.end(), p, p + flen);
            continue;
        case WSC_FK_MESSAGE:                                  // websocket_frame.go:62-91
            if (over(flen)) continue;
            if (f.flags & WSC_FF_CONT_MSG) {
                e.data.swap(c.cont);
                e.data.insert(e.data.end(), c.rbuf.begin(), c.rbuf.end());
                c.rbuf.clear();
                e.data.insert(e.data.end(), p, p + flen);
            } else if (!c.rbuf.empty()) {                     // a streamed message: rBuffer || last piece
                e.data.swap(c.rbuf);
                e.data.insert(e.data.end(), p, p + flen);
            } else {
                e.view = p;
                e.view_len = flen;
                e.set = set;
                views = true;
            }
            e.ev.type = WSC_EV_MESSAGE;
            e.ev.msg_id = f.msg_id;
            e.ev.opcode = f.mode;
            break;
        case WSC_FK_PING:                                     // websocket_ctrl.go:128-153
            e.view = p;
            e.view_len = flen;
            e.set = set;
            views = true;
            e.ev.type = WSC_EV_PONG;
            break;
        case WSC_FK_PONG:
            continue;
        case WSC_FK_CLOSE: case WSC_FK_PONG_EMPTY:           // Close() -> CloseCode(1000, "")
            e.ev.type = WSC_EV_CLOSE;
            e.ev.close_code = 1000;
            break;
        case WSC_FK_ERROR:
            e.ev.type = WSC_EV_CLOSE;
            e.ev.close_code = close_code_for(f.err);
            e.ev.err = f.err;
            break;
        case WSC_FK_STALL:
            e.ev.type = WSC_EV_STALL;
            break;
        default:
            continue;
        }
        c.pending.push_back(std::move(e));
    }
    if (views) s->st[set].view_conns.push_back(slot);
    c.st = so;
    // no-progress guard: a whole batch of this connection's bytes decoded nothing (only a header or a
    // PING / CLOSE frame longer than max_batch_bytes can do that): re-sending it would never end
    const bool stuck = r.status == WSC_SEG_OPEN && r.consumed == 0 && r.frame_count == 0 &&
                       seg_len >= s->cfg.max_batch_bytes;
    if (stuck) push_close(c, 1009, WSC_ERR_NO_PROGRESS);
    if (capped || stuck) c.st.status = WSC_SEG_ERROR;
    if (c.st.status == WSC_SEG_OPEN) {   // the undecoded tail (still masked) goes in front of the next bytes
        c.carry.assign(in_seg + r.consumed, in_seg + seg_len);   // (placing a segment emptied the carry)
    } else {
        c.carry.clear();
        c.spill.clear();
        c.cont.clear();
        c.rbuf.clear();
    }
}

// EOF (wsc_session_eof): once nothing of the connection is left to decode -- no bytes in a batch
// being filled or in flight, none waiting in its spill -- its last event is Close() with code 1000
// (epoll.go:108-110), after every event its earlier bytes produced; an incomplete frame left in
// its carry is dropped, as the reference's next read returns io.EOF inside nextFrame or the header
void maybe_eof(wsc_session* s, Conn& c) {
    if (!c.eof || !c.live || c.failed || c.st.status != WSC_SEG_OPEN) return;
    if (c.in_flight || c.fill_epoch == s->fill_epoch || !c.spill.empty()) return;
    push_close(c, 1000, 0);
    c.st.status = WSC_SEG_CLOSED;
    c.carry.clear();
    c.cont.clear();
    c.rbuf.clear();
}

void fail_conn(wsc_session* s, Conn& c) {
    (void)s;
    c.failed = true;
    Event e;
    std::memset(&e.ev, 0, sizeof(e.ev));
    e.ev.type = WSC_EV_CLOSE;
    e.ev.close_code = 1011;   // RFC 6455 §7.4.1 internal error
    e.ev.err = WSC_ERR_DEVICE;
    c.pending.push_back(std::move(e));
    c.st.status = WSC_SEG_ERROR;
}

// Synchronous decode of segments [a, b) of a completed-with-overflow staging set, re-read from the
// masked input into the result buffer; halves until every part's records fit.
int decode_range(wsc_session* s, int set, uint32_t a, uint32_t b, uint64_t prefix_limit);

int decode_sync_part(wsc_session* s, int set, uint32_t a, uint32_t b, uint64_t prefix_limit) {
    Stage& g = s->st[set];
    const bool compact = (s->flags & WSC_F_COMPACT) != 0;
    const uint64_t base = g.seg_start[a];
    const uint32_t n = b - a;
    std::vector<uint64_t> off(n + 1);
    std::vector<wsc_conn_state> sin(n);
    for (uint32_t q = 0; q < n; ++q) {
        off[q] = g.seg_start[a + q] - base;
        sin[q] = g.h_state_in[a + q];
    }
    uint64_t end = g.seg_start[b - 1] + g.seg_len[b - 1] - base;
    if (prefix_limit && n == 1 && prefix_limit < end) end = prefix_limit;
    off[n] = end;
    uint8_t* res = g.h_res + base;
    if (!compact) std::memcpy(res, g.h_wire + base, end);
    std::vector<wsc_conn_state> sout(n);
    std::vector<wsc_seg_result> sres(n);
    std::vector<wsc_frame> fr(s->cfg.max_frames);
    std::vector<uint64_t> fd(compact ? s->cfg.max_frames : 0);
    wsc_summary sm{};
    // COMPACT: this part's arena lands at the same offset of the result buffer (arena <= wire bytes)
    std::vector<uint8_t> wire_copy;
    uint8_t* wire = res;
    if (compact) {
        wire_copy.assign(g.h_wire + base, g.h_wire + base + end);
        wire = wire_copy.data();
    }
    s->st_h2d += end;   // (a re-decode sends the part again)
    const int rc = wsc_decode_host(g.ctx, wire, end, off.data(), n, s->flags, sin.data(), sout.data(), sres.data(),
                                   fr.data(), s->cfg.max_frames, compact ? res : nullptr,
                                   compact ? fd.data() : nullptr, &sm);
    if (rc == WSC_E_CAPACITY && (sm.overflow & 1u)) {
        if (n > 1) {
            const uint32_t mid = a + n / 2;
            const int r1 = decode_range(s, set, a, mid, 0);
            if (r1) return r1;
            return decode_range(s, set, mid, b, 0);
        }
        // one connection: decode the prefix that ends where its last reported frame begins
        const uint64_t cut = fr[s->cfg.max_frames - 1].hdr_off;
        if (cut == 0 || (prefix_limit && cut >= prefix_limit)) return WSC_E_CAPACITY;
        return decode_range(s, set, a, b, cut);
    }
    if (rc) return rc;
    for (uint32_t q = 0; q < n; ++q) {
        const uint32_t h = g.seg_conn[a + q];
        if (h == DEAD_SEG) continue;
        Conn* c = lookup(s, h);
        if (!c) continue;
        const uint64_t seg_len = (q + 1 < n ? off[q + 1] : end) - off[q];
        harvest(s, set, *c, h & SLOT_MASK, g.h_wire + base + off[q], res, seg_len, sres[q], sout[q],
                fr.data(), compact ? fd.data() : nullptr, 0);
        g.done[a + q] = 1;
        if (n == 1 && end < g.seg_len[a]) {   // a prefix: the rest is decoded by the caller's next batch
            std::vector<uint8_t> tail(g.h_wire + base + end, g.h_wire + base + g.seg_len[a]);
            if (c->st.status == WSC_SEG_OPEN) c->spill.insert(c->spill.begin(), tail.begin(), tail.end());
        }
        maybe_eof(s, *c);
    }
    // views handed out above point into res (in place) / the arena copy region: both in h_res
    return WSC_OK;
}

int decode_range(wsc_session* s, int set, uint32_t a, uint32_t b, uint64_t prefix_limit) {
    return decode_sync_part(s, set, a, b, prefix_limit);
}

// a failed HIP call of the session: WSC_E_DEVICE with wsc_last_error() naming the call and the
// runtime's error text (never a stale message of an earlier error)
int hip_fail(const char* what, hipError_t e) {
    return wsc::set_last_error(WSC_E_DEVICE, std::string("wsc_session: ") + what + ": " + hipGetErrorString(e));
}

// one staging copy on the stage's stream: by a kernel (wsc_kcopy) at s->kcopy >= level, else by
// the copy engine.  A hipMemcpyAsync to or from pinned memory held the poller thread for about the
// copy (the session's launch took 6.6 ms per 20 MB round at 8 pollers, profiles/r05/ab9_timing_P8.log)
int stage_copy(const wsc_session* s, const Stage& g, void* dst, const void* src, uint64_t bytes, hipMemcpyKind kind,
               int level) {
    if (bytes == 0) return WSC_OK;
    if (s->kcopy >= level) return wsc_kcopy(g.ctx, dst, src, bytes, g.stream);
    const hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, g.stream);
    return e == hipSuccess ? WSC_OK : hip_fail("hipMemcpyAsync", e);
}

int launch_stage(wsc_session* s, Stage& g) {
    const bool compact = (s->flags & WSC_F_COMPACT) != 0;
    const uint32_t n = (uint32_t)g.seg_conn.size();
    hipStream_t st = g.stream;
    s->st_h2d += g.bytes;
    s->st_batches += 1;
#define HT(x) do { const hipError_t e_ = (x); if (e_ != hipSuccess) return hip_fail(#x, e_); } while (0)
    const double t0 = s->timing ? now_s() : 0;
#define CP(d, s_, n_, k, lvl) do { if (const int r_ = stage_copy(s, g, d, s_, n_, k, lvl)) return r_; } while (0)
    CP(g.d_wire, g.h_wire, g.bytes, hipMemcpyHostToDevice, 1);
    CP(g.d_seg_off, g.h_seg_off, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, 2);
    CP(g.d_state_in, g.h_state_in, n * sizeof(wsc_conn_state), hipMemcpyHostToDevice, 2);
    const double ta = s->timing ? now_s() : 0;
    if (s->timing) s->t_lh2d += ta - t0;
    wsc_batch b{};
    b.wire = (uint8_t*)g.d_wire;
    b.n_bytes = g.bytes;
    b.seg_off = (const uint64_t*)g.d_seg_off;
    b.n_segs = n;
    b.flags = s->flags;
    b.state_in = (const wsc_conn_state*)g.d_state_in;
    b.state_out = (wsc_conn_state*)g.d_state_out;
    b.seg_out = (wsc_seg_result*)g.d_seg_out;
    b.frames = (wsc_frame*)g.d_frames;
    b.frames_cap = s->cfg.max_frames;
    b.arena = compact ? (uint8_t*)g.d_arena : nullptr;
    b.frame_dst = compact ? (uint64_t*)g.d_frame_dst : nullptr;
    b.summary = (wsc_summary*)g.d_summary;
    const int rc = wsc_decode(g.ctx, &b, st);
    if (rc) return rc;
    if (s->timing) {
        const double tb = now_s();
        s->t_ldec += tb - ta;
    }
    CP(g.h_summary, g.d_summary, sizeof(wsc_summary), hipMemcpyDeviceToHost, 2);
    CP(g.h_state_out, g.d_state_out, n * sizeof(wsc_conn_state), hipMemcpyDeviceToHost, 2);
    CP(g.h_seg_out, g.d_seg_out, n * sizeof(wsc_seg_result), hipMemcpyDeviceToHost, 2);
    // in place the unmasked wire is the batch's whole input range, known now: its D2H goes out with
    // the launch instead of after complete()'s first wait, so it overlaps the host's work on the
    // previous round (views into h_res of this set were materialised by the complete() before)
    if (!compact) CP(g.h_res, g.d_wire, g.bytes, hipMemcpyDeviceToHost, 2);
    // ... and, in place, as many frame records as the last batch had (+1/8): when this batch has no
    // more, complete() needs no second copy and no second wait (the records cost 32 B each)
    g.frames_pre = 0;
    if (!compact && s->frames_hint) {
        g.frames_pre = s->frames_hint < s->cfg.max_frames ? s->frames_hint : s->cfg.max_frames;
        CP(g.h_frames, g.d_frames, (uint64_t)g.frames_pre * sizeof(wsc_frame), hipMemcpyDeviceToHost, 2);
    }
    HT(hipEventRecord(g.done_ev, st));
#undef CP
#undef HT
    return WSC_OK;
}

// wait for everything enqueued on the stage's stream so far
hipError_t stage_wait(const wsc_session* s, Stage& g) {
    if (!(s->flags & WSC_SESSION_BLOCKING_WAIT)) return hipStreamSynchronize(g.stream);
    const hipError_t e = hipEventRecord(g.ev, g.stream);
    return e != hipSuccess ? e : hipEventSynchronize(g.ev);
}

void reset_stage(Stage& g) {
    g.bytes = 0;
    g.seg_conn.clear();
    g.seg_start.clear();
    g.seg_len.clear();
    g.in_flight = false;
    g.launch_rc = WSC_OK;
}

}  // namespace

extern "C" {

int wsc_session_destroy(wsc_session* s);

int wsc_session_create(int device, const wsc_config* cfg, uint32_t flags, wsc_session** out) {
    if (!out) return WSC_E_INVAL;
    *out = nullptr;
    wsc_session* s = new wsc_session();
    if (cfg) s->cfg = *cfg; else wsc_config_default(&s->cfg);
    wsc_config& g = s->cfg;
    if (g.max_frames < 2 || g.max_segs < 2 || g.max_batch_bytes < 64) { delete s; return WSC_E_INVAL; }
    // (no clamp of max_frame_len to the batch: payloads stream across batches)
    if (flags & ~(uint32_t)(WSC_F_COMPACT | WSC_SESSION_BLOCKING_WAIT | WSC_SESSION_TIMING | WSC_SESSION_COPY_ENGINE |
                            WSC_SESSION_KCOPY_ALL)) { delete s; return WSC_E_INVAL; }
    if ((flags & WSC_SESSION_COPY_ENGINE) && (flags & WSC_SESSION_KCOPY_ALL)) { delete s; return WSC_E_INVAL; }
    s->flags = flags & (WSC_F_COMPACT | WSC_SESSION_BLOCKING_WAIT);
    s->timing = (flags & WSC_SESSION_TIMING) != 0;
    s->kcopy = (flags & WSC_SESSION_COPY_ENGINE) ? 0 : (flags & WSC_SESSION_KCOPY_ALL) ? 2 : 1;
    s->device = device;
    int rc = WSC_OK;
    for (Stage& t : s->st) {
        if (rc == WSC_OK) rc = wsc_create(device, &g, &t.ctx);
        if (rc) break;
        if (const hipError_t e = hipSetDevice(device); e != hipSuccess) { rc = hip_fail("hipSetDevice", e); break; }
        if (const hipError_t e = hipStreamCreateWithFlags(&t.stream, hipStreamNonBlocking); e != hipSuccess) {
            rc = hip_fail("hipStreamCreateWithFlags", e);
            break;
        }
        if (const hipError_t e = hipEventCreateWithFlags(&t.done_ev, hipEventDisableTiming); e != hipSuccess) {
            rc = hip_fail("hipEventCreateWithFlags", e);
            break;
        }
        if (s->flags & WSC_SESSION_BLOCKING_WAIT)
            if (const hipError_t e = hipEventCreateWithFlags(&t.ev, hipEventBlockingSync | hipEventDisableTiming); e != hipSuccess) {
                rc = hip_fail("hipEventCreateWithFlags", e);
                break;
            }
        auto H = [&](uint64_t bytes) -> void* {
            void* p = nullptr;
            if (rc == WSC_OK) rc = wsc_host_alloc(bytes, &p);
            return p;
        };
        auto D = [&](uint64_t bytes) -> void* {
            void* p = nullptr;
            if (rc == WSC_OK) rc = wsc_dev_alloc(t.ctx, bytes, &p);
            return p;
        };
        t.h_wire = (uint8_t*)H(g.max_batch_bytes + 64);
        t.h_res = (uint8_t*)H(g.max_batch_bytes + 64);
        t.h_seg_off = (uint64_t*)H((g.max_segs + 1) * sizeof(uint64_t));
        t.h_state_in = (wsc_conn_state*)H(g.max_segs * sizeof(wsc_conn_state));
        t.h_state_out = (wsc_conn_state*)H(g.max_segs * sizeof(wsc_conn_state));
        t.h_seg_out = (wsc_seg_result*)H(g.max_segs * sizeof(wsc_seg_result));
        t.h_frames = (wsc_frame*)H((uint64_t)g.max_frames * sizeof(wsc_frame));
        t.h_frame_dst = (uint64_t*)H((uint64_t)g.max_frames * sizeof(uint64_t));
        t.h_summary = (wsc_summary*)H(sizeof(wsc_summary));
        t.d_wire = D(g.max_batch_bytes + 64);
        t.d_arena = D(g.max_batch_bytes + 64);
        t.d_seg_off = D((g.max_segs + 1) * sizeof(uint64_t));
        t.d_state_in = D(g.max_segs * sizeof(wsc_conn_state));
        t.d_state_out = D(g.max_segs * sizeof(wsc_conn_state));
        t.d_seg_out = D(g.max_segs * sizeof(wsc_seg_result));
        t.d_frames = D((uint64_t)g.max_frames * sizeof(wsc_frame));
        t.d_frame_dst = D((uint64_t)g.max_frames * sizeof(uint64_t));
        t.d_summary = D(sizeof(wsc_summary));
    }
    if (rc) { wsc_session_destroy(s); return rc; }
    *out = s;
    return WSC_OK;
}

int wsc_session_destroy(wsc_session* s) {
    if (!s) return WSC_OK;
    if (s->timing)
        fprintf(stderr, "wsc_session: %llu batches, %llu bytes: pack %.4f s, launch (enqueue) %.4f s (H2D %.4f, decode %.4f), device wait (H2D+kernels+D2H) %.4f s, harvest %.4f s\n",
                (unsigned long long)s->n_batches, (unsigned long long)s->n_bytes, s->t_pack, s->t_launch, s->t_lh2d, s->t_ldec, s->t_device, s->t_harvest);
    for (Stage& t : s->st) {
        if (t.stream) (void)hipStreamSynchronize(t.stream);
        void* hs[] = {t.h_wire, t.h_res, t.h_seg_off, t.h_state_in, t.h_state_out, t.h_seg_out, t.h_frames,
                      t.h_frame_dst, t.h_summary};
        for (void* p : hs)
            if (p) wsc_host_free(p);
        if (t.ctx) {
            void* ds[] = {t.d_wire, t.d_arena, t.d_seg_off, t.d_state_in, t.d_state_out, t.d_seg_out, t.d_frames,
                          t.d_frame_dst, t.d_summary};
            for (void* p : ds)
                if (p) wsc_dev_free(t.ctx, p);
        }
        if (t.ev) (void)hipEventDestroy(t.ev);
        if (t.done_ev) (void)hipEventDestroy(t.done_ev);
        if (t.stream) (void)hipStreamDestroy(t.stream);
        if (t.ctx) wsc_destroy(t.ctx);
    }
    delete s;
    return WSC_OK;
}

int wsc_session_open(wsc_session* s, uint32_t* conn_out) {   // newWebsocketProtocol, websocket.go:59-79
    if (!s || !conn_out) return WSC_E_INVAL;
    apply_removes(s);
    uint32_t slot;
    if (!s->free_slots.empty()) {
        slot = s->free_slots.back();
        s->free_slots.pop_back();
    } else {
        if (s->conns.size() > SLOT_MASK) return WSC_E_CAPACITY;
        slot = (uint32_t)s->conns.size();
        s->conns.emplace_back();
        s->n_slots.store((uint32_t)s->conns.size(), std::memory_order_release);
    }
    Conn& c = s->conns[slot];
    const uint32_t gen = (c.gen + 1) & GEN_MASK;
    c = Conn();
    c.gen = gen;
    c.live = true;
    *conn_out = slot | gen << SLOT_BITS;
    return WSC_OK;
}

// remove() (websocket_ctrl.go:73-96): safe from any thread; applied by the poller thread
int wsc_session_remove(wsc_session* s, uint32_t conn) {
    if (!s) return WSC_E_INVAL;
    if ((conn & SLOT_MASK) >= s->n_slots.load(std::memory_order_acquire)) return WSC_E_STATE;
    std::lock_guard<std::mutex> g(s->rm_mu);
    s->rm_q.push_back(conn);
    s->rm_pending.store(1, std::memory_order_release);
    return WSC_OK;
}

int wsc_session_reserve(wsc_session* s, uint32_t conn, uint64_t max_bytes, uint8_t** ptr, uint64_t* avail) {
    if (!s || !ptr || !avail) return WSC_E_INVAL;
    apply_removes(s);
    Conn* c = lookup(s, conn);
    if (!c) return WSC_E_STATE;
    *ptr = nullptr;
    *avail = 0;
    c->reserved = 0;
    if (c->st.status != WSC_SEG_OPEN || c->failed || c->eof || max_bytes == 0) return WSC_OK;   // closed: nothing to read into
    Stage& f = s->st[s->fill];
    const uint64_t cap = s->cfg.max_batch_bytes;
    // straight into the staging being filled, right behind the connection's segment there (its
    // carried bytes first); bytes already waiting in its spill keep the order, so they go first
    if (c->spill.empty() && !c->in_flight) {
        if (c->fill_epoch == s->fill_epoch && c->seg + 1 != f.seg_conn.size()) {
            // read twice in one round and no longer the last segment: the old region becomes a dead
            // segment and the bytes move to the end
            const uint64_t a = f.seg_start[c->seg], n = f.seg_len[c->seg];
            c->carry.assign(f.h_wire + a, f.h_wire + a + n);
            f.seg_conn[c->seg] = DEAD_SEG;
            c->fill_epoch = ~0ull;
        }
        if (place(s, *c, conn, 0)) {
            const uint64_t room = cap > f.bytes ? cap - f.bytes : 0;
            const uint64_t k = room < max_bytes ? room : max_bytes;
            if (k >= max_bytes || k >= MIN_RESERVE) {
                *ptr = f.h_wire + f.bytes;
                *avail = k;
                c->reserved = k;
                c->reserved_spill = false;
                return WSC_OK;
            }
        }
    }
    // otherwise into the connection's spill (decoded in a later batch)
    const uint64_t at = c->spill.size();
    c->spill.resize(at + max_bytes);
    *ptr = c->spill.data() + at;
    *avail = max_bytes;
    c->reserved = max_bytes;
    c->reserved_spill = true;
    return WSC_OK;
}

int wsc_session_commit(wsc_session* s, uint32_t conn, uint64_t n) {
    if (!s) return WSC_E_INVAL;
    Conn* c = lookup(s, conn);
    if (!c) return WSC_E_STATE;
    if (n > c->reserved) return WSC_E_INVAL;
    // a staging reservation belongs to the staging set being filled when it was made: if a submit
    // switched sets since (a misuse: commit must come first), c->seg indexes the other set's vectors
    // -- nothing is read into the batch; an empty commit (wsc_session_eof's) just drops it (round-5
    // ADVICE)
    if (c->reserved && !c->reserved_spill && c->fill_epoch != s->fill_epoch) {
        c->reserved = 0;
        return n == 0 ? WSC_OK : WSC_E_STATE;
    }
    s->st_read += n;
    if (c->reserved_spill) {
        c->spill.resize(c->spill.size() - (c->reserved - n));
    } else if (c->reserved) {
        Stage& f = s->st[s->fill];
        f.seg_len[c->seg] += n;
        f.bytes += n;
    }
    c->reserved = 0;
    if (c->eof) maybe_eof(s, *c);   // nothing left of it to decode: Close() is due now
    return WSC_OK;
}

int wsc_session_feed(wsc_session* s, uint32_t conn, const uint8_t* bytes, uint64_t n) {
    if (!s) return WSC_E_INVAL;
    if (n && !bytes) return WSC_E_INVAL;
    while (n) {
        uint8_t* p = nullptr;
        uint64_t k = 0;
        int rc = wsc_session_reserve(s, conn, n, &p, &k);
        if (rc) return rc;
        if (!p) return WSC_OK;   // closed / stalled: bytes are ignored
        if (k > n) k = n;
        std::memcpy(p, bytes, k);
        rc = wsc_session_commit(s, conn, k);
        if (rc) return rc;
        bytes += k;
        n -= k;
    }
    Conn* c = lookup(s, conn);
    return c ? WSC_OK : WSC_E_STATE;
}

// Launch the staging being filled (async: H2D, walk + unmask, small D2H on its stream) and switch
// filling to the other set.  Connections whose bytes wait in their spill are packed first.
int wsc_session_submit(wsc_session* s) {
    if (!s) return WSC_E_INVAL;
    apply_removes(s);
    if (s->st[0].in_flight || s->st[1].in_flight) return WSC_E_STATE;   // complete() first
    const double t0 = s->timing ? now_s() : 0;
    Stage& f = s->st[s->fill];
    for (uint32_t slot = 0; slot < s->conns.size(); ++slot) {   // spilled bytes ride in this batch if they fit
        Conn& c = s->conns[slot];
        // a reservation still open (a misuse: commit comes first) reads nothing into this batch: it
        // is dropped, so a spill region held open is not packed as data and a later commit(0) --
        // wsc_session_eof's -- finds nothing to shrink (round-5 ADVICE)
        if (c.reserved) {
            if (c.reserved_spill) c.spill.resize(c.spill.size() - c.reserved);
            c.reserved = 0;
        }
        if (!c.live || c.failed || c.st.status != WSC_SEG_OPEN || c.spill.empty()) continue;
        if (c.fill_epoch == s->fill_epoch) {
            if (c.seg + 1 != f.seg_conn.size()) continue;   // not last: next batch
            const uint64_t room = s->cfg.max_batch_bytes - f.bytes;
            const uint64_t k = c.spill.size() < room ? c.spill.size() : room;
            std::memcpy(f.h_wire + f.bytes, c.spill.data(), k);
            c.spill.erase(c.spill.begin(), c.spill.begin() + (long)k);
            f.seg_len[c.seg] += k;
            f.bytes += k;
        } else {
            place(s, c, slot | c.gen << SLOT_BITS, 0);
        }
    }
    const uint32_t n = (uint32_t)f.seg_conn.size();
    if (n == 0) return WSC_OK;
    for (uint32_t q = 0; q < n; ++q) {
        s->st[s->fill].h_seg_off[q] = f.seg_start[q];
        Conn* c = f.seg_conn[q] == DEAD_SEG ? nullptr : lookup(s, f.seg_conn[q]);
        wsc_conn_state st{};
        if (c) st = c->st;
        else st.status = WSC_SEG_CLOSED;   // a dead region: the walk decodes nothing there
        f.h_state_in[q] = st;
    }
    f.h_seg_off[n] = f.bytes;
    for (uint32_t q = 0; q < n; ++q)
        if (Conn* c = f.seg_conn[q] == DEAD_SEG ? nullptr : lookup(s, f.seg_conn[q])) c->in_flight = true;
    const double t1 = s->timing ? now_s() : 0;
    s->n_submits += 1;
    if (s->fault_at && s->n_submits == s->fault_at)   // test hook: as a failed launch would
        f.launch_rc = wsc::set_last_error(WSC_E_DEVICE, "wsc_session: injected device failure (wsc_session_inject_fault)");
    else
        f.launch_rc = launch_stage(s, f);
    const double t2 = s->timing ? now_s() : 0;
    f.in_flight = true;
    s->fill ^= 1;
    s->fill_epoch += 1;
    Stage& nf = s->st[s->fill];
    reset_stage(nf);
    if (s->timing) {
        s->t_pack += t1 - t0;
        s->t_launch += t2 - t1;
        s->n_batches += 1;
        s->n_bytes += f.bytes;
    }
    return WSC_OK;
}

// Wait for the batch in flight and turn its records into events.  Event data handed out by the
// previous complete() is materialised (copied) or dropped here: it stays valid until this call.
int wsc_session_complete(wsc_session* s) {
    if (!s) return WSC_E_INVAL;
    apply_removes(s);
    s->retired.clear();   // event data handed out before this call is no longer valid
    const int set = s->st[0].in_flight ? 0 : (s->st[1].in_flight ? 1 : -1);
    if (set < 0) return WSC_OK;
    Stage& g = s->st[set];
    const bool compact = (s->flags & WSC_F_COMPACT) != 0;
    const double t0 = s->timing ? now_s() : 0;
    int rc = g.launch_rc;
    if (rc == WSC_OK)
        if (const hipError_t e = stage_wait(s, g); e != hipSuccess) rc = hip_fail("hipStreamSynchronize", e);
    if (rc == WSC_OK && (g.h_summary->overflow & 2u))
        rc = wsc::set_last_error(WSC_E_INTERNAL, "wsc_session: device look-back timeout: batch results are invalid");
    const uint32_t n = (uint32_t)g.seg_conn.size();
    for (uint32_t q = 0; q < n; ++q)
        if (Conn* c = g.seg_conn[q] == DEAD_SEG ? nullptr : lookup(s, g.seg_conn[q])) c->in_flight = false;
    g.done.assign(n, 0);
    bool split = false;
    if (rc == WSC_OK && (g.h_summary->overflow & 1u)) split = true;
    uint32_t nf = 0;
    if (rc == WSC_OK && !split) {
        nf = g.h_summary->n_frames;
        int crc = WSC_OK;
        auto D2H = [&](void* dst, const void* src, uint64_t bytes) {
            if (crc == WSC_OK) crc = stage_copy(s, g, dst, src, bytes, hipMemcpyDeviceToHost, 2);
        };
        const uint32_t pre = nf < g.frames_pre ? nf : g.frames_pre;   // (copied with the launch)
        D2H(g.h_frames + pre, (const wsc_frame*)g.d_frames + pre, (uint64_t)(nf - pre) * sizeof(wsc_frame));
        if (compact) {
            D2H(g.h_res, g.d_arena, g.h_summary->data_bytes + g.h_summary->ctrl_bytes);
            D2H(g.h_frame_dst, g.d_frame_dst, (uint64_t)nf * sizeof(uint64_t));
        }   // (in place the wire came back with the launch: launch_stage)
        if (crc == WSC_OK && (compact || nf > pre))
            if (const hipError_t e = stage_wait(s, g); e != hipSuccess) crc = hip_fail("hipStreamSynchronize", e);
        rc = crc;
        s->frames_hint = nf + nf / 8;
    }
    const double t1 = s->timing ? now_s() : 0;
    materialize_views(s, set ^ 1);   // the other set is filled next: its views must not dangle
    g.view_conns.clear();
    if (rc == WSC_OK && split) {
        rc = decode_range(s, set, 0, n, 0);   // records exceeded max_frames: halves, synchronously
    } else if (rc == WSC_OK) {
        for (uint32_t q = 0; q < n; ++q) {
            const uint32_t h = g.seg_conn[q];
            if (h == DEAD_SEG) continue;
            Conn* c = lookup(s, h);
            if (!c) continue;   // removed while in flight
            harvest(s, set, *c, h & SLOT_MASK, g.h_wire + g.seg_start[q], g.h_res, g.seg_len[q],
                    g.h_seg_out[q], g.h_state_out[q], g.h_frames, compact ? g.h_frame_dst : nullptr, 0);
            g.done[q] = 1;
            maybe_eof(s, *c);
        }
    }
    if (rc != WSC_OK && rc != WSC_E_CAPACITY) {
        // device failure: the batch's connections are closed (1011), their carried bytes kept
        for (uint32_t q = 0; q < n; ++q) {
            Conn* c = g.seg_conn[q] == DEAD_SEG ? nullptr : lookup(s, g.seg_conn[q]);
            if (!c || g.done[q]) continue;   // (a split decode may have finished some before failing)
            std::vector<uint8_t> keep(g.h_wire + g.seg_start[q], g.h_wire + g.seg_start[q] + g.seg_len[q]);
            keep.insert(keep.end(), c->spill.begin(), c->spill.end());
            c->carry.swap(keep);
            c->spill.clear();
            fail_conn(s, *c);
        }
    }
    g.in_flight = false;
    if (s->timing) {
        const double t2 = now_s();
        s->t_device += t1 - t0;
        s->t_harvest += t2 - t1;
    }
    return rc;
}

// one batched device pass over everything fed so far (submit + complete until nothing is left)
int wsc_session_decode(wsc_session* s) {
    if (!s) return WSC_E_INVAL;
    int rc = wsc_session_complete(s);   // a batch submitted earlier is finished first
    if (rc) return rc;
    for (int guard = 0; guard < 1 << 20; ++guard) {
        rc = wsc_session_submit(s);
        if (rc) return rc;
        if (!s->st[0].in_flight && !s->st[1].in_flight) return WSC_OK;   // nothing was pending
        rc = wsc_session_complete(s);
        if (rc) return rc;
        bool more = false;   // bytes left over (prefixes, spills that did not fit)
        for (const Conn& c : s->conns)
            if (c.live && !c.failed && c.st.status == WSC_SEG_OPEN && !c.spill.empty()) { more = true; break; }
        if (!more) return WSC_OK;
    }
    return WSC_E_CAPACITY;
}

// whether complete() would return without waiting: every launched set's last operation has
// finished (or its launch failed, which complete() reports at once)
int wsc_session_ready(wsc_session* s, int* ready) {
    if (!s || !ready) return WSC_E_INVAL;
    *ready = 1;
    for (const Stage& g : s->st)
        if (g.in_flight && g.launch_rc == WSC_OK && g.done_ev && hipEventQuery(g.done_ev) == hipErrorNotReady) *ready = 0;
    return WSC_OK;
}

// bytes fed but not yet submitted (the staging being filled + connections' spills): a poller calls
// submit again while this is non-zero, even in a round without new reads
int wsc_session_pending(wsc_session* s, uint64_t* bytes) {
    if (!s || !bytes) return WSC_E_INVAL;
    apply_removes(s);
    uint64_t n = s->st[s->fill].bytes;
    for (const Conn& c : s->conns)
        if (c.live && !c.failed && c.st.status == WSC_SEG_OPEN) n += c.spill.size();
    *bytes = n;
    return WSC_OK;
}

// The peer closed its side: a read returned 0 (BaseConnect.Read -> io.EOF, baseconnect.go:100-103).
// Every event of the bytes read before it is delivered first; then Close() (epoll.go:108-110).
int wsc_session_eof(wsc_session* s, uint32_t conn) {
    if (!s) return WSC_E_INVAL;
    apply_removes(s);
    Conn* c = lookup(s, conn);
    if (!c) return WSC_E_STATE;
    // a reservation not committed yet (reserve -> read() == 0 -> eof, commit left for later): the
    // read brought nothing, so drop it now -- a spill region held open would keep maybe_eof waiting
    // after the commit had shrunk it away (round-4 ADVICE)
    if (c->reserved) (void)wsc_session_commit(s, conn, 0);
    c->eof = true;
    // a read that returned 0 may follow a reserve that placed the connection in the staging being
    // filled with nothing in it: that empty region is dropped (else it would wait for a submit that
    // wsc_session_pending() == 0 never asks for, and Close() would never come)
    Stage& f = s->st[s->fill];
    if (c->fill_epoch == s->fill_epoch && c->seg < f.seg_conn.size() && f.seg_len[c->seg] == 0) {
        f.seg_conn[c->seg] = DEAD_SEG;
        c->fill_epoch = ~0ull;
    }
    maybe_eof(s, *c);
    return WSC_OK;
}

int wsc_session_set_max_message(wsc_session* s, uint64_t bytes) {
    if (!s) return WSC_E_INVAL;
    s->max_message = bytes;
    return WSC_OK;
}

int wsc_session_next(wsc_session* s, uint32_t conn, wsc_event* ev) {
    if (!s || !ev) return WSC_E_INVAL;
    apply_removes(s);
    Conn* c = lookup(s, conn);
    if (!c) return WSC_E_STATE;
    std::memset(ev, 0, sizeof(*ev));
    if (c->pending.empty()) { ev->type = WSC_EV_NONE; return WSC_OK; }   // (nil, EAGAIN)
    // the previous event's owned bytes stay valid until the next complete (a server may still be
    // sending them from a zero-copy reply queue): retired, not freed
    if (!c->current.data.empty()) s->retired.push_back(std::move(c->current.data));
    c->current = std::move(c->pending.front());
    c->pending.pop_front();
    *ev = c->current.ev;
    if (c->current.view) {
        ev->data = c->current.view_len ? c->current.view : nullptr;
        ev->len = c->current.view_len;
    } else {
        ev->data = c->current.data.empty() ? nullptr : c->current.data.data();
        ev->len = c->current.data.size();
    }
    return WSC_OK;
}

int wsc_session_inject_fault(wsc_session* s, uint64_t k) {
    if (!s) return WSC_E_INVAL;
    s->fault_at = k ? s->n_submits + k : 0;
    return WSC_OK;
}

int wsc_session_stats(wsc_session* s, uint64_t* out, uint32_t n) {
    if (!s || (n && !out)) return WSC_E_INVAL;
    const uint64_t v[5] = {s->st_read, s->st_h2d, s->st_resent, s->st_batches, s->st_pieces};
    for (uint32_t i = 0; i < n && i < 5; ++i) out[i] = v[i];
    return WSC_OK;
}

int wsc_session_state(wsc_session* s, uint32_t conn, wsc_conn_state* st, uint64_t* carry_bytes) {
    if (!s) return WSC_E_INVAL;
    apply_removes(s);
    Conn* c = lookup(s, conn);
    if (!c) return WSC_E_STATE;
    if (st) *st = c->st;
    if (carry_bytes) *carry_bytes = c->carry.size() + c->spill.size();
    return WSC_OK;
}

}  // extern "C"
