// wsc_session.cpp -- C++ host side above the ABI: the per-connection DecodePacket() mirror.
//
// In netman every poller goroutine calls conn.DecodePacket() once per readiness event
// (eventloop/epoll.go:105) and gets back at most one (IMessage, error) (server/websocket.go:82-212).
// Here a poller instead feeds each ready connection's bulk read into the session
// (wsc_session_feed), runs ONE batched device decode over all of them (wsc_session_decode), and
// then drains each connection's results one at a time with wsc_session_next(), which returns
// exactly what the reference's DecodePacket + epoll.go:104-140 would have produced, in order:
//   WSC_EV_MESSAGE  (Message, nil)          -> IWebsocketHandler.Message   (routermgr.go:101)
//   WSC_EV_PONG     pong() echo             -> push(encode(0x8A, payload)) (websocket_ctrl.go:128-153)
//   WSC_EV_CLOSE    CloseCode(code)         -> epoll.go:106-129 mapping of the sentinel
//   WSC_EV_STALL    unmasked frame (Q3)     -> nothing more is delivered
//   WSC_EV_NONE     (nil, syscall.EAGAIN)
// The per-connection state a goroutine kept in websocketProtocol (websocket.go:38-56) lives in
// Conn: the carried partial frame (the reference keeps it in the kernel socket buffer / rBuffer),
// continueBuffer for fragmented messages, and the device-visible wsc_conn_state.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "../../include/wscodec.h"

namespace {

struct Event {
    wsc_event ev;
    std::vector<uint8_t> data;     // owned copy (fragmented messages, earlier batches of a decode)
    const uint8_t* view = nullptr; // zero-copy: points into the pinned staging of the last batch
    uint64_t view_len = 0;
};

struct Conn {
    bool live = false;
    wsc_conn_state st{};
    std::vector<uint8_t> carry;   // undecoded tail of previous reads (starts at a frame header)
    std::vector<uint8_t> fed;     // bytes read since the last decode
    std::vector<uint8_t> cont;    // continueBuffer (unmasked fragments so far)
    std::deque<Event> pending;
    Event current;                // storage for the event last returned by next()
};

uint32_t close_code_for(uint32_t err) {   // eventloop/epoll.go:106-129
    return err == WSC_ERR_MUST_UTF8 ? 1007u : 1002u;
}

}  // namespace

struct wsc_session {
    wsc_ctx* ctx = nullptr;
    wsc_config cfg{};
    uint32_t flags = 0;
    std::vector<Conn> conns;
    std::vector<uint32_t> free_ids;
    // pinned staging
    uint8_t* h_wire = nullptr;
    uint8_t* h_arena = nullptr;
    uint64_t* h_seg_off = nullptr;
    wsc_conn_state* h_state_in = nullptr;
    wsc_conn_state* h_state_out = nullptr;
    wsc_seg_result* h_seg_out = nullptr;
    wsc_frame* h_frames = nullptr;
    uint64_t* h_frame_dst = nullptr;
    // WSC_SESSION_TIMING=1: seconds spent per phase of wsc_session_decode, printed at destroy
    bool timing = false;
    double t_pack = 0, t_device = 0, t_harvest = 0;
    uint64_t n_decodes = 0, n_bytes = 0;
};

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

extern "C" {

int wsc_session_destroy(wsc_session* s);

int wsc_session_create(int device, const wsc_config* cfg, uint32_t flags, wsc_session** out) {
    if (!out) return WSC_E_INVAL;
    *out = nullptr;
    wsc_session* s = new wsc_session();
    if (cfg) s->cfg = *cfg; else wsc_config_default(&s->cfg);
    s->flags = flags & WSC_F_COMPACT;
    int rc = wsc_create(device, &s->cfg, &s->ctx);
    if (rc) { delete s; return rc; }
    const wsc_config& g = s->cfg;
    void* p = nullptr;
    auto H = [&](uint64_t bytes) -> void* {
        p = nullptr;
        if (rc == WSC_OK) rc = wsc_host_alloc(bytes, &p);
        return p;
    };
    s->h_wire = (uint8_t*)H(g.max_batch_bytes + 64);
    s->h_arena = (uint8_t*)H(g.max_batch_bytes + 64);
    s->h_seg_off = (uint64_t*)H((g.max_segs + 1) * sizeof(uint64_t));
    s->h_state_in = (wsc_conn_state*)H(g.max_segs * sizeof(wsc_conn_state));
    s->h_state_out = (wsc_conn_state*)H(g.max_segs * sizeof(wsc_conn_state));
    s->h_seg_out = (wsc_seg_result*)H(g.max_segs * sizeof(wsc_seg_result));
    s->h_frames = (wsc_frame*)H((uint64_t)g.max_frames * sizeof(wsc_frame));
    s->h_frame_dst = (uint64_t*)H((uint64_t)g.max_frames * sizeof(uint64_t));
    if (rc) { wsc_session_destroy(s); return rc; }
    if (const char* e = std::getenv("WSC_SESSION_TIMING"); e && e[0] == '1') s->timing = true;
    *out = s;
    return WSC_OK;
}

int wsc_session_destroy(wsc_session* s) {
    if (!s) return WSC_OK;
    if (s->timing)
        fprintf(stderr, "wsc_session: %llu decodes, %llu bytes: pack %.4f s, device (H2D+kernels+D2H) %.4f s, harvest %.4f s\n",
                (unsigned long long)s->n_decodes, (unsigned long long)s->n_bytes, s->t_pack, s->t_device, s->t_harvest);
    void* ps[] = {s->h_wire, s->h_arena, s->h_seg_off, s->h_state_in, s->h_state_out,
                  s->h_seg_out, s->h_frames, s->h_frame_dst};
    for (void* p : ps)
        if (p) wsc_host_free(p);
    if (s->ctx) wsc_destroy(s->ctx);
    delete s;
    return WSC_OK;
}

int wsc_session_open(wsc_session* s, uint32_t* conn_out) {   // newWebsocketProtocol, websocket.go:59-79
    if (!s || !conn_out) return WSC_E_INVAL;
    uint32_t id;
    if (!s->free_ids.empty()) { id = s->free_ids.back(); s->free_ids.pop_back(); }
    else { id = (uint32_t)s->conns.size(); s->conns.emplace_back(); }
    s->conns[id] = Conn();
    s->conns[id].live = true;
    *conn_out = id;
    return WSC_OK;
}

int wsc_session_remove(wsc_session* s, uint32_t conn) {     // remove(), websocket_ctrl.go:73-96
    if (!s || conn >= s->conns.size() || !s->conns[conn].live) return WSC_E_STATE;
    s->conns[conn] = Conn();
    s->free_ids.push_back(conn);
    return WSC_OK;
}

int wsc_session_feed(wsc_session* s, uint32_t conn, const uint8_t* bytes, uint64_t n) {
    if (!s || conn >= s->conns.size() || !s->conns[conn].live) return WSC_E_STATE;
    if (n && !bytes) return WSC_E_INVAL;
    Conn& c = s->conns[conn];
    if (c.st.status != WSC_SEG_OPEN) return WSC_OK;   // closed / stalled: bytes are ignored
    c.fed.insert(c.fed.end(), bytes, bytes + n);
    return WSC_OK;
}

// turn one segment's frame records into the DecodePacket results the reference would return
// zero_copy: the staging stays untouched until the next wsc_session_decode (this is the decode's
// last device batch), so complete single-frame messages and PING payloads are handed out as views
// into it instead of copies; wsc_event.data's lifetime is exactly that (include/wscodec.h).
static void harvest(wsc_session* s, Conn& c, const uint8_t* seg, const wsc_seg_result& r,
                    const wsc_conn_state& so, uint64_t seg_base, bool zero_copy) {
    const bool compact = (s->flags & WSC_F_COMPACT) != 0;
    for (uint32_t i = r.frame_begin; i < r.frame_begin + r.frame_count; ++i) {
        const wsc_frame& f = s->h_frames[i];
        const uint8_t* p = compact ? s->h_arena + s->h_frame_dst[i]
                                   : seg + (f.hdr_off - seg_base) + f.hdr_len;
        Event e;
        std::memset(&e.ev, 0, sizeof(e.ev));
        switch (f.kind) {
        case WSC_FK_FRAG:                                     // websocket_frame.go:95-98
            c.cont.insert(c.cont.end(), p, p + f.payload_len);
            continue;
        case WSC_FK_MESSAGE:                                  // websocket_frame.go:62-91
            if (f.flags & WSC_FF_CONT_MSG) {
                e.data.swap(c.cont);
                e.data.insert(e.data.end(), p, p + f.payload_len);
            } else if (zero_copy) {
                e.view = p;
                e.view_len = f.payload_len;
            } else {
                e.data.assign(p, p + f.payload_len);
            }
            e.ev.type = WSC_EV_MESSAGE;
            e.ev.msg_id = f.msg_id;
            e.ev.opcode = f.mode;
            break;
        case WSC_FK_PING:                                     // websocket_ctrl.go:128-153
            if (zero_copy) {
                e.view = p;
                e.view_len = f.payload_len;
            } else {
                e.data.assign(p, p + f.payload_len);
            }
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
    c.st = so;
    if (r.status == WSC_SEG_OPEN) {
        const uint64_t seg_len = c.carry.size() + c.fed.size();
        std::vector<uint8_t> rest(seg + r.consumed, seg + seg_len);
        c.carry.swap(rest);
    } else {
        c.carry.clear();
        c.cont.clear();
    }
    c.fed.clear();
}

int wsc_session_decode(wsc_session* s) {
    if (!s) return WSC_E_INVAL;
    const wsc_config& g = s->cfg;
    std::vector<uint32_t> ids;
    for (uint32_t i = 0; i < s->conns.size(); ++i) {
        Conn& c = s->conns[i];
        for (Event& e : c.pending)   // undrained zero-copy views: the staging is about to be reused
            if (e.view) {
                e.data.assign(e.view, e.view + e.view_len);
                e.view = nullptr;
            }
        if (c.live && c.st.status == WSC_SEG_OPEN && !c.fed.empty()) ids.push_back(i);
    }
    size_t k = 0;
    while (k < ids.size()) {
        // pack as many connections as fit into one device batch
        const double t0 = s->timing ? now_s() : 0;
        uint64_t bytes = 0;
        uint32_t n = 0;
        size_t j = k;
        while (j < ids.size() && n < g.max_segs) {
            const Conn& c = s->conns[ids[j]];
            const uint64_t sl = c.carry.size() + c.fed.size();
            if (sl > g.max_batch_bytes) return WSC_E_CAPACITY;
            if (bytes + sl > g.max_batch_bytes && n > 0) break;
            s->h_seg_off[n] = bytes;
            uint8_t* dst = s->h_wire + bytes;
            if (!c.carry.empty()) std::memcpy(dst, c.carry.data(), c.carry.size());
            std::memcpy(dst + c.carry.size(), c.fed.data(), c.fed.size());
            s->h_state_in[n] = c.st;
            bytes += sl;
            ++n;
            ++j;
        }
        s->h_seg_off[n] = bytes;
        const double t1 = s->timing ? now_s() : 0;
        wsc_summary sm;
        int rc = wsc_decode_host(s->ctx, s->h_wire, bytes, s->h_seg_off, n, s->flags, s->h_state_in,
                                 s->h_state_out, s->h_seg_out, s->h_frames, g.max_frames, s->h_arena,
                                 s->h_frame_dst, &sm);
        if (rc) return rc;
        const double t2 = s->timing ? now_s() : 0;
        for (uint32_t q = 0; q < n; ++q) {
            Conn& c = s->conns[ids[k + q]];
            harvest(s, c, s->h_wire + s->h_seg_off[q], s->h_seg_out[q], s->h_state_out[q], s->h_seg_off[q],
                    j == ids.size());
        }
        if (s->timing) {
            const double t3 = now_s();
            s->t_pack += t1 - t0;
            s->t_device += t2 - t1;
            s->t_harvest += t3 - t2;
            s->n_decodes += 1;
            s->n_bytes += bytes;
        }
        k = j;
    }
    return WSC_OK;
}

int wsc_session_next(wsc_session* s, uint32_t conn, wsc_event* ev) {
    if (!s || !ev || conn >= s->conns.size() || !s->conns[conn].live) return WSC_E_STATE;
    Conn& c = s->conns[conn];
    std::memset(ev, 0, sizeof(*ev));
    if (c.pending.empty()) { ev->type = WSC_EV_NONE; return WSC_OK; }   // (nil, EAGAIN)
    c.current = std::move(c.pending.front());
    c.pending.pop_front();
    *ev = c.current.ev;
    if (c.current.view) {
        ev->data = c.current.view_len ? c.current.view : nullptr;
        ev->len = c.current.view_len;
    } else {
        ev->data = c.current.data.empty() ? nullptr : c.current.data.data();
        ev->len = c.current.data.size();
    }
    return WSC_OK;
}

int wsc_session_state(wsc_session* s, uint32_t conn, wsc_conn_state* st, uint64_t* carry_bytes) {
    if (!s || conn >= s->conns.size() || !s->conns[conn].live) return WSC_E_STATE;
    if (st) *st = s->conns[conn].st;
    if (carry_bytes) *carry_bytes = s->conns[conn].carry.size();
    return WSC_OK;
}

}  // extern "C"
