// session_stub.cpp -- TEST INFRASTRUCTURE: a host-memory stand-in for the device side of
// libwscodec, so the session host logic (netman_amd/csrc/wsc_session.cpp: staging, carry, prefix
// batches, record-overflow splits, views, cross-thread removal, device-failure policy) can run
// under ASan/UBSan and TSan on a machine without a GPU.  It provides the HIP runtime calls the
// session makes (memcpy / no-op streams) and a minimal frame walker for masked TEXT/BIN/CONT/
// PING/PONG/CLOSE frames (no UTF-8, no COMPACT) -- enough to drive every session code path.  It
// is NOT the product decoder and not the oracle; the GPU tests compare the real one with the oracle.
#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/wscodec.h"

struct wsc_ctx {
    wsc_config cfg;
};

static thread_local std::string g_err;
static std::mutex g_alloc_mu;

extern "C" {
const char* wsc_last_error(void) { return g_err.c_str(); }
int wsc_config_default(wsc_config* c) {
    std::memset(c, 0, sizeof(*c));
    c->max_batch_bytes = 64ull << 20;
    c->max_segs = 1u << 16;
    c->max_frames = 1u << 20;
    c->max_frame_len = 0xFFFFFFFFFFull;
    return WSC_OK;
}
int wsc_create(int, const wsc_config* cfg, wsc_ctx** out) {
    *out = new wsc_ctx{*cfg};
    return WSC_OK;
}
int wsc_destroy(wsc_ctx* c) {
    delete c;
    return WSC_OK;
}
int wsc_dev_alloc(wsc_ctx*, uint64_t bytes, void** out) {
    *out = std::calloc(1, bytes ? bytes : 16);
    return *out ? WSC_OK : WSC_E_NOMEM;
}
int wsc_dev_free(wsc_ctx*, void* p) {
    std::free(p);
    return WSC_OK;
}
int wsc_host_alloc(uint64_t bytes, void** out) {
    *out = std::calloc(1, bytes ? bytes : 16);
    return *out ? WSC_OK : WSC_E_NOMEM;
}
int wsc_host_free(void* p) {
    std::free(p);
    return WSC_OK;
}
}

// ---- the stand-in walk: one segment ----
static uint32_t rotr(uint32_t x, uint32_t r) { r &= 31; return r ? (x >> r) | (x << (32 - r)) : x; }
// unmask n bytes at p with the mask word phased to p (byte i takes mask byte i & 3)
static void xor_run(uint8_t* p, uint64_t n, uint32_t mask) {
    for (uint64_t i = 0; i < n; ++i) p[i] ^= (uint8_t)(mask >> (8 * (i & 3)));
}
static void walk(const wsc_ctx* c, uint8_t* w, uint64_t a, uint64_t b, uint32_t s, const wsc_conn_state* in,
                 wsc_conn_state* out, wsc_seg_result* r, wsc_frame* fr, uint32_t cap, uint32_t& nf) {
    wsc_conn_state st = in ? *in : wsc_conn_state{};
    uint64_t pos = a;
    uint32_t status = st.status, code = 0, err = 0, k0 = nf;
    // a streamed data frame's rest (ABI 3): one piece, the last one takes the frame's kind
    if (status == WSC_SEG_OPEN && st.frame_rem && b > pos) {
        const uint64_t take = b - pos < st.frame_rem ? b - pos : st.frame_rem;
        const uint32_t op = st.frame_hdr & 15, fin = st.frame_hdr >> 7;
        wsc_frame f{};
        f.hdr_off = pos;
        f.seg = s;
        f.msg_id = st.msg_id;
        f.opcode = (uint8_t)op;
        f.fin = (uint8_t)fin;
        f.mode = st.message_mode;
        f.payload_len = (uint32_t)take;
        f.payload_len_hi = (uint8_t)(take >> 32);
        f.mask = st.frame_mask;
        f.flags = WSC_FF_UNMASKED | WSC_FF_HEAD_PREV;
        xor_run(w + pos, take, st.frame_mask);
        if (take < st.frame_rem) {
            f.kind = WSC_FK_PIECE;
        } else if (op == 10) {   // a streamed PONG completes: discarded
            f.kind = WSC_FK_PONG;
            st.msg_id += 1;
        } else if (fin) {
            f.kind = WSC_FK_MESSAGE;
            if (op == 0 && st.cont_len) f.flags |= WSC_FF_CONT_MSG;
            st.cont_len = 0;
            st.message_mode = 0;
            st.msg_id += 1;
        } else {
            f.kind = WSC_FK_FRAG;
            st.cont_len += st.frame_len;
        }
        st.frame_rem -= take;
        st.frame_mask = rotr(st.frame_mask, 8 * (uint32_t)(take & 3));
        if (nf < cap) fr[nf] = f;
        ++nf;
        pos += take;
    }
    while (status == WSC_SEG_OPEN && st.frame_rem == 0 && b - pos >= 2) {
        const uint8_t b0 = w[pos], b1 = w[pos + 1];
        const uint32_t op = b0 & 15, fin = b0 >> 7, len7 = b1 & 127;
        const uint32_t ext = len7 == 126 ? 2 : (len7 == 127 ? 8 : 0);
        if (b - pos < 2 + ext) break;
        uint64_t plen = len7;
        if (ext) {
            plen = 0;
            for (uint32_t i = 0; i < ext; ++i) plen = plen << 8 | w[pos + 2 + i];
        }
        wsc_frame f{};
        f.hdr_off = pos;
        f.seg = s;
        f.msg_id = st.msg_id;
        f.opcode = (uint8_t)op;
        f.fin = (uint8_t)fin;
        f.mode = st.message_mode;
        if (!(b1 & 0x80)) {   // unmasked: stall (Q3)
            f.kind = WSC_FK_STALL;
            f.hdr_len = (uint8_t)(2 + ext);
            status = WSC_SEG_STALLED;
            if (nf < cap) fr[nf] = f;
            ++nf;
            break;
        }
        const uint32_t hl = 6 + ext;
        if (b - pos < hl) break;
        if (plen > c->cfg.max_frame_len) {
            f.kind = WSC_FK_ERROR;
            f.err = WSC_ERR_TOO_LARGE;
            f.hdr_len = (uint8_t)hl;
            status = WSC_SEG_ERROR; code = 1002; err = WSC_ERR_TOO_LARGE;
            if (nf < cap) fr[nf] = f;
            ++nf;
            pos += hl;
            break;
        }
        const bool data = op <= 2;
        const bool bad = data && ((op == 0 && st.message_mode == 0) || (op != 0 && st.cont_len));
        uint64_t take = plen;
        bool piece = false;
        if (b - pos < hl + plen) {
            if ((!data && op != 10) || bad) break;   // PING / CLOSE wait whole (errors checked first)
            take = b - pos - hl;
            piece = true;
        }
        const uint8_t* m = w + pos + hl - 4;
        uint32_t mask;
        std::memcpy(&mask, m, 4);
        if (!bad) xor_run(w + pos + hl, take, mask);
        f.hdr_len = (uint8_t)hl;
        f.payload_len = (uint32_t)take;
        f.payload_len_hi = (uint8_t)(take >> 32);
        f.mask = mask;
        f.flags = WSC_FF_UNMASKED;
        bool stop = false;
        if (data) {
            if (bad) {
                f.kind = WSC_FK_ERROR;
                f.err = WSC_ERR_OPCODE_FAIL;
                f.flags = 0;
                status = WSC_SEG_ERROR; code = 1002; err = WSC_ERR_OPCODE_FAIL;
                stop = true;
            } else if (piece) {
                f.kind = WSC_FK_PIECE;
                if (op) st.message_mode = (uint8_t)op;
                f.mode = st.message_mode;
                st.frame_rem = plen - take;
                st.frame_len = plen;
                st.frame_mask = rotr(mask, 8 * (uint32_t)(take & 3));
                st.frame_hdr = (uint8_t)(fin << 7 | op);
            } else if (fin) {
                f.kind = WSC_FK_MESSAGE;
                f.mode = op ? (uint8_t)op : st.message_mode;
                if (op == 0 && st.cont_len) f.flags |= WSC_FF_CONT_MSG;
                st.cont_len = 0;
                st.message_mode = 0;
                st.msg_id += 1;
            } else {
                f.kind = WSC_FK_FRAG;
                if (op) st.message_mode = (uint8_t)op;
                f.mode = st.message_mode;
                st.cont_len += plen;
            }
        } else if (op == 9) {
            f.kind = WSC_FK_PING;
            st.msg_id += 1;
        } else if (op == 10 && piece) {   // a PONG streams like a data frame (ABI 4)
            f.kind = WSC_FK_PIECE;
            st.frame_rem = plen - take;
            st.frame_len = plen;
            st.frame_mask = rotr(mask, 8 * (uint32_t)(take & 3));
            st.frame_hdr = (uint8_t)(fin << 7 | op);
        } else if (op == 10) {
            f.kind = plen ? WSC_FK_PONG : WSC_FK_PONG_EMPTY;
            if (plen) st.msg_id += 1;
            else { status = WSC_SEG_CLOSED; code = 1000; stop = true; }
        } else {
            f.kind = WSC_FK_CLOSE;
            status = WSC_SEG_CLOSED; code = 1000; stop = true;
        }
        if (nf < cap) fr[nf] = f;
        ++nf;
        pos += hl + (bad ? 0 : take);
        if (stop) break;
    }
    st.status = (uint8_t)status;
    if (status != WSC_SEG_OPEN) st.frame_rem = 0;
    *out = st;
    r->consumed = pos - a;
    r->frame_begin = k0;
    r->frame_count = nf - k0;
    r->status = status;
    r->close_code = code;
    r->err = err;
    r->pad = 0;
}

static void walk_batch(const wsc_ctx* c, uint8_t* w, const uint64_t* off, uint32_t n, const wsc_conn_state* in,
                       wsc_conn_state* out, wsc_seg_result* r, wsc_frame* fr, uint32_t cap, wsc_summary* sm) {
    uint32_t nf = 0;
    for (uint32_t s = 0; s < n; ++s) walk(c, w, off[s], off[s + 1], s, in ? in + s : nullptr, out + s, r + s, fr, cap, nf);
    std::memset(sm, 0, sizeof(*sm));
    sm->n_frames = nf;
    sm->n_spans = nf;
    sm->overflow = nf > cap ? 1u : 0u;
}

extern "C" {
int wsc_kcopy(wsc_ctx*, void* dst, const void* src, uint64_t bytes, void*) {   // "device" = host memory
    if (bytes) std::memcpy(dst, src, bytes);
    return WSC_OK;
}

int wsc_decode(wsc_ctx* c, const wsc_batch* b, void*) {
    if (b->flags & WSC_F_COMPACT) return WSC_E_INVAL;   // (the stand-in does in place only)
    walk_batch(c, b->wire, b->seg_off, b->n_segs, b->state_in, b->state_out, b->seg_out, b->frames, b->frames_cap,
               b->summary);
    return WSC_OK;
}
int wsc_decode_host(wsc_ctx* c, uint8_t* wire, uint64_t, const uint64_t* seg_off, uint32_t n_segs, uint32_t flags,
                    const wsc_conn_state* state_in, wsc_conn_state* state_out, wsc_seg_result* seg_out,
                    wsc_frame* frames, uint32_t frames_cap, uint8_t*, uint64_t*, wsc_summary* summary) {
    if (flags & WSC_F_COMPACT) return WSC_E_INVAL;
    walk_batch(c, wire, seg_off, n_segs, state_in, state_out, seg_out, frames, frames_cap, summary);
    if (summary->overflow & 1u) return WSC_E_CAPACITY;
    return WSC_OK;
}
}

namespace wsc {
int set_last_error(int code, const std::string& msg) {   // (wsc_api.cpp in the real library)
    g_err = msg;
    return code;
}
}  // namespace wsc

// ---- the HIP runtime calls the session makes ----
const char* hipGetErrorString(hipError_t) { return "stub HIP error"; }
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned int) {
    *s = reinterpret_cast<hipStream_t>(new int(0));
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
    delete reinterpret_cast<int*>(s);
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) {
    if (n) std::memmove(d, s, n);
    return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned int) {
    *e = reinterpret_cast<hipEvent_t>(new int(0));
    return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) {
    delete reinterpret_cast<int*>(e);
    return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventQuery(hipEvent_t) { return hipSuccess; }
