/*
 * ws_oracle.c -- CPU restatement of netman's websocket decode path.  TEST INFRASTRUCTURE ONLY:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, as the checker.
 * See ws_oracle.h for the list of reference functions restated; every function below cites the
 * reference file:line it follows.  The structure deliberately mirrors the Go code (one call of
 * decode_packet() == one DecodePacket() call) so the quirks of SURVEY.md table Q fall out of it.
 */
#include "ws_oracle.h"
#include <stdlib.h>
#include <string.h>

/* --- Go 1.16 unicode/utf8.Valid (table-driven: `first` + acceptRanges) ------------------------- */
enum { XX = 0xF1, AS = 0xF0, S1 = 0x02, S2 = 0x13, S3 = 0x03, S4 = 0x23, S5 = 0x34, S6 = 0x04, S7 = 0x44 };
static const uint8_t go_first[256] = {
#define R16(v) v, v, v, v, v, v, v, v, v, v, v, v, v, v, v, v
    R16(AS), R16(AS), R16(AS), R16(AS), R16(AS), R16(AS), R16(AS), R16(AS),      /* 0x00-0x7F */
    R16(XX), R16(XX), R16(XX), R16(XX),                                          /* 0x80-0xBF */
    XX, XX, S1, S1, S1, S1, S1, S1, S1, S1, S1, S1, S1, S1, S1, S1,              /* 0xC0-0xCF */
    R16(S1),                                                                     /* 0xD0-0xDF */
    S2, S3, S3, S3, S3, S3, S3, S3, S3, S3, S3, S3, S3, S4, S3, S3,              /* 0xE0-0xEF */
    S5, S6, S6, S6, S7, XX, XX, XX, XX, XX, XX, XX, XX, XX, XX, XX,              /* 0xF0-0xFF */
#undef R16
};
static const uint8_t go_accept_lo[5] = {0x80, 0xA0, 0x80, 0x90, 0x80};
static const uint8_t go_accept_hi[5] = {0xBF, 0xBF, 0x9F, 0xBF, 0x8F};

int wso_utf8_valid(const uint8_t* p, uint64_t n) {
    uint64_t i = 0;
    while (i < n) {
        uint8_t pi = p[i];
        if (pi < 0x80) { i++; continue; }
        uint8_t x = go_first[pi];
        if (x == XX) return 0;
        uint64_t size = x & 7;
        if (i + size > n) return 0;
        uint8_t lo = go_accept_lo[x >> 4], hi = go_accept_hi[x >> 4];
        uint8_t c = p[i + 1];
        if (c < lo || hi < c) return 0;
        if (size > 2) {
            c = p[i + 2];
            if (c < 0x80 || 0xBF < c) return 0;
            if (size > 3) {
                c = p[i + 3];
                if (c < 0x80 || 0xBF < c) return 0;
            }
        }
        i += size;
    }
    return 1;
}

/* websocket_frame.go:35-39 */
void wso_unmask(const uint8_t* in, uint8_t* out, uint64_t n, const uint8_t masks[4]) {
    for (uint64_t i = 0; i < n; i++) out[i] = in[i] ^ masks[i % 4];
}

/* --- growable byte buffer standing in for bytes.Buffer ------------------------------------------ */
typedef struct { uint8_t* p; uint64_t n, cap; } buf_t;
static void buf_write(buf_t* b, const uint8_t* s, uint64_t n) {
    if (b->n + n > b->cap) {
        uint64_t c = b->cap ? b->cap : 64;
        while (c < b->n + n) c *= 2;
        b->p = (uint8_t*)realloc(b->p, c);
        b->cap = c;
    }
    if (n) memcpy(b->p + b->n, s, n);
    b->n += n;
}
static void buf_reset(buf_t* b) { b->n = 0; }
static void buf_free(buf_t* b) { free(b->p); b->p = NULL; b->n = b->cap = 0; }

/* --- simulated non-blocking socket + BaseConnect.Read (baseconnect.go:84-106) ------------------- */
enum { E_NIL = 0, E_EAGAIN = 100, E_EOF = 101 };
typedef struct { const uint8_t* s; uint64_t avail, rpos; int eof; } sock_t;
/* unix.Read: -1/EAGAIN when nothing is buffered, 0 for a zero-length read or once the peer has
 * closed and nothing is buffered; BaseConnect.Read maps n<0 -> (0, err) and n==0 -> (0, io.EOF). */
static int64_t conn_read(sock_t* k, uint8_t* dst, uint64_t n, int* err) {
    if (n == 0) { *err = E_EOF; return 0; }
    if (k->rpos >= k->avail) { *err = k->eof ? E_EOF : E_EAGAIN; return 0; }
    uint64_t m = k->avail - k->rpos;
    if (m > n) m = n;
    memcpy(dst, k->s + k->rpos, m);
    k->rpos += m;
    *err = E_NIL;
    return (int64_t)m;
}

/* --- websocketProtocol state (websocket.go:38-56) ---------------------------------------------- */
enum { CONTINUATION = 0, TEXTMODE = 1, BINMODE = 2, CLOSE = 8, PING = 9, PONG = 10 };  /* :19-26 */
enum { parsePayloadLength = 1, parseMasks = 2 };                                         /* :33-36 */
static const uint16_t reservedCode[4] = {1004, 1005, 1006, 1015};                        /* :31 */

typedef struct {
    uint8_t final;
    uint64_t fragmentLength;
    buf_t packetBuffer, rBuffer, continueBuffer;
    int parseHeader;
    uint8_t opcode;
    uint8_t masks[4];
    int nmasks;
    uint32_t msgID;
    uint8_t messageMode;
    uint8_t parseHeaderStep;
    uint8_t headerBytes[2];
    int nheader;
    int closed;
    /* oracle bookkeeping (not reference state) */
    uint64_t hdr_off, payload_off;
    uint32_t msgid_at_hdr;
} ws_t;

typedef struct {
    sock_t k;
    ws_t c;
    uint64_t max_frame_len;
    uint8_t* inplace;
    wso_event* ev; uint32_t ev_cap, n_ev;
    wso_frame* fr; uint32_t fr_cap, n_fr;
    uint8_t* arena; uint64_t arena_cap, arena_used;
    int overflow;
} run_t;

/* websocket.go:304-312 */
static void ws_reset(ws_t* c) {
    c->parseHeader = 0;
    buf_reset(&c->rBuffer);
    c->nmasks = 0;
    c->opcode = 0;
    c->fragmentLength = 0;
    c->parseHeaderStep = 0;
    c->nheader = 0;
}

static uint64_t arena_put(run_t* r, const uint8_t* p, uint64_t n) {
    uint64_t off = r->arena_used;
    if (off + n > r->arena_cap) { r->overflow = 1; return off; }
    if (n) memcpy(r->arena + off, p, n);
    r->arena_used += n;
    return off;
}
static void emit_event(run_t* r, wso_event e) {
    if (r->n_ev >= r->ev_cap) { r->overflow = 1; return; }
    r->ev[r->n_ev++] = e;
}
/* header fields of the frame being decoded, captured before nextFrame()'s reset() clears them */
typedef struct {
    uint64_t hdr_off, payload_off, len;
    uint32_t mask, msg_id;
    uint8_t opcode, fin, mode, complete;
} snap_t;
static snap_t take_snap(const ws_t* c) {
    snap_t s;
    memset(&s, 0, sizeof(s));
    s.hdr_off = c->hdr_off;
    s.complete = (uint8_t)c->parseHeader;
    if (c->parseHeader) {
        s.payload_off = c->payload_off;
        s.len = c->fragmentLength;
        s.mask = (uint32_t)c->masks[0] | (uint32_t)c->masks[1] << 8 | (uint32_t)c->masks[2] << 16 |
                 (uint32_t)c->masks[3] << 24;
    }
    s.msg_id = c->msgID;
    s.opcode = c->opcode;
    s.fin = c->final;
    s.mode = c->messageMode;
    return s;
}
/* one log line per frame whose processing finished (delivered, consumed, or failed) */
static void log_frame(run_t* r, const snap_t* s, uint8_t kind, uint32_t err) {
    if (r->n_fr >= r->fr_cap) { r->overflow = 1; return; }
    wso_frame* f = &r->fr[r->n_fr++];
    memset(f, 0, sizeof(*f));
    f->hdr_off = s->hdr_off;
    f->payload_off = s->payload_off;
    f->payload_len = s->len;
    f->mask = s->mask;
    f->msg_id = s->msg_id;
    f->opcode = s->opcode;
    f->fin = s->fin;
    f->kind = kind;
    f->mode = s->mode;
    f->err = err;
}

/* websocket.go:271-302 */
static int parse_payload_length(run_t* r) {
    ws_t* c = &r->c;
    int err;
    if (c->fragmentLength <= 125) { c->parseHeaderStep = parsePayloadLength; return E_NIL; }
    if (c->fragmentLength == 126) {
        uint8_t lb[2];
        int64_t n = conn_read(&r->k, lb, 2, &err);
        if (n != 2 || err != E_NIL) return err;       /* Q1: a 1-byte read returns nil here */
        c->fragmentLength = ((uint64_t)lb[0] << 8) | lb[1];
        c->parseHeaderStep = parsePayloadLength;
        return E_NIL;
    }
    if (c->fragmentLength == 127) {
        uint8_t lb[8];
        int64_t n = conn_read(&r->k, lb, 8, &err);
        if (n != 8 || err != E_NIL) return err;
        uint64_t v = 0;
        for (int i = 0; i < 8; i++) v = (v << 8) | lb[i];
        c->fragmentLength = v;
        c->parseHeaderStep = parsePayloadLength;
    }
    return E_NIL;
}

/* websocket.go:214-269 */
static int parse_head_bytes(run_t* r) {
    ws_t* c = &r->c;
    uint8_t firstByte = c->headerBytes[0], secondByte = c->headerBytes[1];
    c->final = firstByte >> 7;                                           /* :217 */
    uint8_t rsv1 = 1 & (firstByte >> 4), rsv2 = 1 & (firstByte >> 5), rsv3 = 1 & (firstByte >> 6);
    c->opcode = firstByte & 0xf;                                         /* :222 */
    uint8_t maskd = secondByte >> 7;
    c->fragmentLength = secondByte & 127;                                /* :224 */
    if (rsv1 == 1 || rsv2 == 1 || rsv3 == 1) return WSO_ERR_RSV_FAIL;    /* :229-231 */
    if (c->opcode == TEXTMODE || c->opcode == BINMODE) c->messageMode = c->opcode;   /* :234-236 */
    if (c->parseHeaderStep < parsePayloadLength) {                       /* :239-243 */
        int e = parse_payload_length(r);
        if (e != E_NIL) return e;
    }
    if (maskd >= 1) {                                                    /* :246-266 */
        if (c->parseHeaderStep < parseMasks) {
            int length = 4 - c->nmasks;
            if (length > 0) {
                uint8_t mb[4];
                int err;
                int64_t n = conn_read(&r->k, mb, (uint64_t)length, &err);
                if (n <= 0 || err != E_NIL) return err;
                memcpy(c->masks + c->nmasks, mb, (size_t)n);
                c->nmasks += (int)n;
            }
            if (c->nmasks == 4) {
                c->parseHeaderStep = parseMasks;
                c->parseHeader = 1;
                c->nheader = 0;
                c->payload_off = r->k.rpos;
            }
        }
    }
    return E_NIL;
}

/* Q3 predicate: an unmasked header has been parsed, so DecodePacket returns EAGAIN forever */
static int unmasked_stall(const ws_t* c) {
    return !c->parseHeader && c->nheader == 2 && (c->headerBytes[1] >> 7) == 0 &&
           c->parseHeaderStep >= parsePayloadLength && (c->headerBytes[0] & 0x70) == 0;
}

/* what nextFrame() returned: an owned copy of Message.Data */
typedef struct { int has; uint32_t msg_id; uint8_t opcode; uint8_t* data; uint64_t len; } msg_t;

/* websocket_frame.go:13-103 */
static int next_frame(run_t* r, msg_t* out) {
    ws_t* c = &r->c;
    out->has = 0;
    if (c->fragmentLength > r->max_frame_len) return WSO_ERR_TOO_LARGE;  /* Q4: make() would panic */
    uint64_t rLen = c->fragmentLength - c->rBuffer.n;                    /* :16 */
    uint8_t* payloadBuffer = (uint8_t*)malloc(rLen ? rLen : 1);          /* :17 */
    int err;
    int64_t n = conn_read(&r->k, payloadBuffer, rLen, &err);             /* :18 */
    if (c->fragmentLength != 0) {                                        /* :21-25 */
        if (n <= 0 || err != E_NIL) { free(payloadBuffer); return err; }
    }
    buf_write(&c->rBuffer, payloadBuffer, (uint64_t)n);                  /* :28 */
    free(payloadBuffer);
    if (c->rBuffer.n != c->fragmentLength) return E_EAGAIN;              /* :31, :102 */

    if (c->nmasks == 4) {                                                /* :35-39 */
        uint8_t* decodeBuffer = (uint8_t*)malloc(c->fragmentLength ? c->fragmentLength : 1);
        for (uint64_t i = 0; i < c->rBuffer.n; i++) decodeBuffer[i] = c->rBuffer.p[i] ^ c->masks[i % 4];
        if (r->inplace && c->fragmentLength)
            memcpy(r->inplace + c->payload_off, decodeBuffer, c->fragmentLength);
        buf_write(&c->packetBuffer, decodeBuffer, c->fragmentLength);    /* :44 */
        free(decodeBuffer);
    } else {
        buf_write(&c->packetBuffer, c->rBuffer.p, c->rBuffer.n);         /* :40-41 (dead for clients) */
    }
    uint8_t opcode = c->opcode;                                          /* :46 */
    ws_reset(c);                                                         /* :49 */
    if (c->final == 1) {                                                 /* :52 */
        if (opcode == CONTINUATION && c->continueBuffer.n >= 1) {        /* :62-68 */
            buf_write(&c->continueBuffer, c->packetBuffer.p, c->packetBuffer.n);
            buf_t t = c->packetBuffer;
            c->packetBuffer = c->continueBuffer;
            c->continueBuffer = t;
            buf_reset(&c->continueBuffer);
        }
        if (c->messageMode == TEXTMODE && !wso_utf8_valid(c->packetBuffer.p, c->packetBuffer.n))
            return WSO_ERR_MUST_UTF8;                                    /* :71-73 */
        out->has = 1;                                                    /* :75-81 */
        out->msg_id = c->msgID;
        out->opcode = c->messageMode;
        out->len = c->packetBuffer.n;
        out->data = (uint8_t*)malloc(out->len ? out->len : 1);
        if (out->len) memcpy(out->data, c->packetBuffer.p, out->len);
        if (opcode == CONTINUATION || opcode == TEXTMODE || opcode == BINMODE) c->messageMode = 0;
        c->msgID += 1;                                                   /* :89 */
        buf_reset(&c->packetBuffer);                                     /* :90 */
        return E_NIL;
    }
    buf_write(&c->continueBuffer, c->packetBuffer.p, c->packetBuffer.n); /* :95 */
    buf_reset(&c->packetBuffer);                                         /* :98 */
    return E_EAGAIN;                                                     /* :102 */
}

/* websocket_ctrl.go:160-177 */
static int verify_close_code(uint16_t code) {
    if (code < 1000 || code >= 5000) return WSO_ERR_PROTOCOL_ERROR;
    if (code >= 1016 && code <= 2999) return WSO_ERR_PROTOCOL_ERROR;
    for (int i = 0; i < 4; i++)
        if (code == reservedCode[i]) return WSO_ERR_PROTOCOL_ERROR;
    return E_NIL;
}

/* CloseCode (websocket_ctrl.go:99-119): send a close frame, remove(), close the fd */
static void close_code(run_t* r, uint32_t code, uint32_t err) {
    wso_event e;
    memset(&e, 0, sizeof(e));
    e.type = WSO_EV_CLOSE;
    e.close_code = code;
    e.err = err;
    emit_event(r, e);
    r->c.closed = 1;
}

/*
 * One DecodePacket() call (websocket.go:82-212) followed by the poller's handling of its result
 * (epoll.go:104-140).  Returns 1 if the poller would stop for this readiness event (EAGAIN or a
 * closed connection), 0 to call again.  The handshake (:85-95) happened before the stream starts.
 */
static int decode_packet(run_t* r) {
    ws_t* c = &r->c;
    msg_t m = {0};
    int err = E_NIL;
    uint8_t kind = 0xFF;   /* frame-log kind once the frame's fate is known */
    snap_t s;

    if (!c->parseHeader) {                                               /* :98 */
        int length = 2 - c->nheader;
        if (length > 0) {                                                /* :101-110 */
            uint8_t hb[2];
            if (c->nheader == 0) c->hdr_off = r->k.rpos;
            int e2;
            int64_t n = conn_read(&r->k, hb, (uint64_t)length, &e2);
            if (n <= 0 || e2 != E_NIL) { err = e2; goto handle; }
            memcpy(c->headerBytes + c->nheader, hb, (size_t)n);
            c->nheader += (int)n;
        }
        if (c->nheader != 2) { err = E_EAGAIN; goto handle; }            /* :112-114 */
        err = parse_head_bytes(r);                                       /* :116 */
        if (err != E_NIL) {
            if (err == WSO_ERR_RSV_FAIL) { s = take_snap(c); log_frame(r, &s, WSO_FK_ERROR, err); }
            goto handle;
        }
    }
    if (!c->parseHeader) { err = E_EAGAIN; goto handle; }                /* :122-124 */

    s = take_snap(c);
    switch (c->opcode) {                                                 /* :136 */
    case CONTINUATION:
        if (c->messageMode < TEXTMODE) { err = WSO_ERR_OPCODE_FAIL; break; }
        err = next_frame(r, &m);                                         /* :211 */
        kind = c->final == 1 ? WSO_FK_MESSAGE : WSO_FK_FRAG;
        break;
    case TEXTMODE: case BINMODE:
        if (c->continueBuffer.n >= 1) { err = WSO_ERR_PING_PAYLOAD_OVERSIZE; break; }
        err = next_frame(r, &m);
        kind = c->final == 1 ? WSO_FK_MESSAGE : WSO_FK_FRAG;
        break;
    case CLOSE:                                                          /* :147-184 */
        if (!(c->fragmentLength == 0 || c->fragmentLength >= 2) || c->fragmentLength > 125) {
            err = WSO_ERR_PROTOCOL_ERROR;
            break;
        }
        if (c->fragmentLength >= 2) {
            uint8_t fin = c->final;
            err = next_frame(r, &m);
            if (err != E_NIL && err != WSO_ERR_MUST_UTF8) {
                if (err == E_EAGAIN && fin == 0 && !c->parseHeader) {
                    /* Q7: a fragmented CLOSE went into continueBuffer and the call returned EAGAIN */
                    log_frame(r, &s, WSO_FK_FRAG, 0);
                }
                break;
            }
            /* reason = the returned message, or -- when nextFrame's whole-payload utf8.Valid failed
             * under messageMode==TEXT (websocket_frame.go:71-73, error swallowed at :156) -- a
             * stand-in Message{DataLen: uint32(c.fragmentLength), Data: packetBuffer} (:160-167).
             * nextFrame's reset() (websocket_frame.go:49 -> websocket.go:309) has already zeroed
             * fragmentLength, so that stand-in has Len() == 0: the reason check below is skipped
             * and only the code (Data[:2], still the close payload) is verified. */
            const uint8_t* rp = m.has ? m.data : c->packetBuffer.p;
            uint64_t rn = m.has ? m.len : c->fragmentLength;
            if (rn > 2 && !wso_utf8_valid(rp + 2, rn - 2)) { err = WSO_ERR_MUST_UTF8; break; }   /* :170-172 */
            uint16_t code = (uint16_t)((rp[0] << 8) | rp[1]);                                   /* :175-176 */
            err = verify_close_code(code);
            if (err != E_NIL) break;
        }
        log_frame(r, &s, WSO_FK_CLOSE, 0);
        close_code(r, 1000, 0);                                          /* :183 -> Close() */
        if (m.has) free(m.data);
        return 1;
    case PING:                                                           /* :185-190 */
        if (c->final != 1) { err = WSO_ERR_CTRL_FRAGMENTED; break; }
        if (c->fragmentLength > 125) { err = WSO_ERR_PING_PAYLOAD_OVERSIZE; break; }   /* ctrl.go:130-132 */
        err = next_frame(r, &m);                                         /* ctrl.go:134 */
        if (err == E_NIL && m.has) {                                     /* ctrl.go:139-152: echo as PONG */
            wso_event e;
            memset(&e, 0, sizeof(e));
            e.type = WSO_EV_PONG;
            e.data_off = arena_put(r, m.data, m.len);
            e.data_len = m.len;
            emit_event(r, e);
            log_frame(r, &s, WSO_FK_PING, 0);
            free(m.data);
            return 0;                                                    /* (nil, nil) */
        }
        break;
    case PONG:                                                           /* :191-205 */
        if (c->final != 1) { err = WSO_ERR_CTRL_FRAGMENTED; break; }
        if (c->fragmentLength <= 0) {
            log_frame(r, &s, WSO_FK_PONG_EMPTY, 0);
            close_code(r, 1000, 0);
            return 1;
        }
        err = next_frame(r, &m);
        if (err == E_NIL) {
            log_frame(r, &s, WSO_FK_PONG, 0);
            if (m.has) free(m.data);
            return 0;
        }
        break;
    default:
        err = WSO_ERR_OPCODE_FAIL;                                       /* :206-207 */
        break;
    }

    if (err == E_NIL && m.has) {                                         /* data message delivered */
        log_frame(r, &s, WSO_FK_MESSAGE, 0);
        wso_event e;
        memset(&e, 0, sizeof(e));
        e.type = WSO_EV_MESSAGE;
        e.msg_id = m.msg_id;
        e.opcode = m.opcode;
        e.data_off = arena_put(r, m.data, m.len);
        e.data_len = m.len;
        emit_event(r, e);                                                /* epoll.go:136-140 */
        free(m.data);
        return 0;
    }
    if (err == E_EAGAIN && kind == WSO_FK_FRAG && !c->parseHeader)
        log_frame(r, &s, WSO_FK_FRAG, 0);                                /* fragment stored */
    if (err != E_NIL && err != E_EAGAIN && err != E_EOF)
        log_frame(r, &s, WSO_FK_ERROR, (uint32_t)err);

handle:                                                                  /* epoll.go:106-129 */
    if (m.has) free(m.data);
    switch (err) {
    case E_NIL:
        return 0;
    case E_EOF:
        close_code(r, 1000, 0);
        return 1;
    case WSO_ERR_OPCODE_FAIL: case WSO_ERR_RSV_FAIL: case WSO_ERR_CTRL_FRAGMENTED:
    case WSO_ERR_PROTOCOL_ERROR: case WSO_ERR_PING_PAYLOAD_OVERSIZE: case WSO_ERR_TOO_LARGE:
        close_code(r, 1002, (uint32_t)err);
        return 1;
    case WSO_ERR_MUST_UTF8:
        close_code(r, 1007, (uint32_t)err);
        return 1;
    default:   /* EAGAIN */
        return 1;
    }
}

int wso_run(const uint8_t* stream, uint64_t len, const uint64_t* chunk_ends, uint32_t n_chunks,
            uint64_t max_frame_len, uint8_t* inplace,
            wso_event* ev, uint32_t ev_cap, wso_frame* fr, uint32_t fr_cap,
            uint8_t* arena, uint64_t arena_cap, wso_result* res) {
    return wso_run_ex(stream, len, chunk_ends, n_chunks, max_frame_len, inplace, ev, ev_cap, fr, fr_cap, arena,
                      arena_cap, res, 0);
}

int wso_run_ex(const uint8_t* stream, uint64_t len, const uint64_t* chunk_ends, uint32_t n_chunks,
               uint64_t max_frame_len, uint8_t* inplace,
               wso_event* ev, uint32_t ev_cap, wso_frame* fr, uint32_t fr_cap,
               uint8_t* arena, uint64_t arena_cap, wso_result* res, uint32_t flags) {
    run_t r;
    memset(&r, 0, sizeof(r));
    r.k.s = stream;
    r.max_frame_len = max_frame_len;
    r.inplace = inplace;
    r.ev = ev; r.ev_cap = ev_cap;
    r.fr = fr; r.fr_cap = fr_cap;
    r.arena = arena; r.arena_cap = arena_cap;
    if (inplace && len) memcpy(inplace, stream, len);
    uint64_t one = len;
    if (!chunk_ends || n_chunks == 0) { chunk_ends = &one; n_chunks = 1; }
    int stalled = 0;
    for (uint32_t ci = 0; ci < n_chunks && !r.c.closed && !stalled; ci++) {
        r.k.avail = chunk_ends[ci] < len ? chunk_ends[ci] : len;
        /* level-triggered epoll: an event fires while unread bytes remain; the poller makes one
         * DecodePacket call per event */
        while (!r.c.closed && r.k.rpos < r.k.avail) {
            uint64_t before = r.k.rpos;
            uint32_t ev_before = r.n_ev;
            decode_packet(&r);
            if (unmasked_stall(&r.c) || (r.k.rpos == before && r.n_ev == ev_before && !r.c.closed)) {
                stalled = 1;   /* Q3: EAGAIN without reading anything: epoll would spin forever */
                break;
            }
        }
    }
    if ((flags & WSO_RUN_EOF) && !r.c.closed && !stalled) {
        /* the peer closed: epoll keeps reporting the fd readable and each DecodePacket reads
         * what is left, until a read returns 0 -> io.EOF -> Close() (epoll.go:108-110) */
        r.k.avail = len;
        r.k.eof = 1;
        while (!r.c.closed) {
            uint64_t before = r.k.rpos;
            uint32_t ev_before = r.n_ev;
            decode_packet(&r);
            if (unmasked_stall(&r.c) || (r.k.rpos == before && r.n_ev == ev_before && !r.c.closed)) {
                stalled = 1;
                break;
            }
        }
    }
    if (stalled) {
        snap_t s = take_snap(&r.c);
        log_frame(&r, &s, WSO_FK_STALL, 0);
        wso_event e;
        memset(&e, 0, sizeof(e));
        e.type = WSO_EV_STALL;
        emit_event(&r, e);
    }
    memset(res, 0, sizeof(*res));
    res->consumed = r.k.rpos;
    res->closed = (uint32_t)r.c.closed;
    res->stalled = (uint32_t)stalled;
    for (uint32_t i = 0; i < r.n_ev; i++)
        if (ev[i].type == WSO_EV_CLOSE) { res->close_code = ev[i].close_code; res->err = ev[i].err; }
    res->msg_id = r.c.msgID;
    res->message_mode = r.c.messageMode;
    res->cont_len = r.c.continueBuffer.n;
    res->n_events = r.n_ev;
    res->n_frames = r.n_fr;
    res->arena_used = r.arena_used;
    res->overflow = (uint32_t)r.overflow;
    buf_free(&r.c.packetBuffer);
    buf_free(&r.c.rBuffer);
    buf_free(&r.c.continueBuffer);
    return r.overflow ? -1 : 0;
}

/* ---- encode (server/websocket_ctrl.go:23-70) ------------------------------------------------ */
uint64_t wso_encode(uint8_t first_byte, const uint8_t* bs, uint64_t len, uint8_t* out) {
    uint64_t k = 0;
    out[k++] = first_byte;                              /* :28 binary.Write(firstByte) */
    if (len <= 125) {                                   /* :33-37 */
        out[k++] = (uint8_t)len;
    } else if (len >= 126 && len <= 65535) {           /* :39-49 uint8(126) + uint16 BE */
        out[k++] = 126;
        out[k++] = (uint8_t)(len >> 8);
        out[k++] = (uint8_t)len;
    } else {                                            /* :51-61 uint8(127) + uint64 BE */
        out[k++] = 127;
        for (int s = 56; s >= 0; s -= 8) out[k++] = (uint8_t)(len >> s);
    }
    if (len) memcpy(out + k, bs, len);                  /* :64-66 the payload, unmasked */
    return k + len;
}

uint64_t wso_encode_batch(const uint8_t* src, const uint64_t* src_off, const uint64_t* len,
                          const uint8_t* first_byte, uint32_t n, uint8_t* out, uint64_t* out_off) {
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; i++) {
        out_off[i] = pos;
        pos += wso_encode(first_byte[i], src + src_off[i], len[i], out + pos);
    }
    out_off[n] = pos;
    return pos;
}
