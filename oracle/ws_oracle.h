/*
 * ws_oracle.h -- CPU restatement of netman's websocket DECODE path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the MI355X frame codec.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may link, load or call anything under oracle/; the product path
 * (netman_amd/, libwscodec.so) never does.
 *
 * What it restates (reference = ikilobyte/netman @ /root/reference, pure Go, no tests of its own):
 *   server/websocket.go:82-212   DecodePacket  (header gate, opcode switch)
 *   server/websocket.go:214-269  parseHeadBytes
 *   server/websocket.go:271-302  parsePayloadLength
 *   server/websocket.go:304-312  reset
 *   server/websocket_frame.go:13-103  nextFrame (XOR unmask, reassembly, utf8, Message)
 *   server/websocket_ctrl.go:128-153  pong ; :160-177 verifyCloseCode ; websocket.go:31 reservedCode
 *   server/baseconnect.go:84-106      Read  (n<0 -> (0,err); n==0 -> io.EOF)
 *   eventloop/epoll.go:104-140        error -> close-code mapping, level-triggered re-fire
 *   util/errors.go:9-14               error sentinels
 *   Go 1.16 unicode/utf8.Valid        (go.mod:3) restated from its published table-driven algorithm
 *
 * The socket is simulated: the post-handshake byte stream arrives in chunks (chunk_ends); after each
 * chunk the "poller" calls DecodePacket while it makes progress, exactly like level-triggered epoll.
 * Because it is a faithful model of the read pattern, it also reproduces the split-header quirks
 * Q1/Q2 of SURVEY.md §8(a) when a chunk boundary falls inside a header.
 *
 * Parity pinning: RFC 6455 §5.7 known-answer frames and aiohttp 3.14.3 reader_py cross-checks
 * (tests/golden/), see DESIGN.md "Oracle".
 */
#ifndef WS_ORACLE_H
#define WS_ORACLE_H
#include <stdint.h>
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

/* error sentinels (util/errors.go:9-14); numeric values equal the codec's WSC_ERR_* on purpose */
enum {
    WSO_ERR_NONE = 0,
    WSO_ERR_OPCODE_FAIL = 1,            /* WebsocketOpcodeFail */
    WSO_ERR_RSV_FAIL = 2,               /* WebsocketRsvFail */
    WSO_ERR_PING_PAYLOAD_OVERSIZE = 3,  /* WebsocketPingPayloadOversize */
    WSO_ERR_CTRL_FRAGMENTED = 4,        /* WebsocketCtrlMessageMustNotFragmented */
    WSO_ERR_MUST_UTF8 = 5,              /* WebsocketMustUtf8 */
    WSO_ERR_PROTOCOL_ERROR = 6,         /* WebsocketProtocolError */
    WSO_ERR_TOO_LARGE = 7,              /* not in the reference: make() would panic (Q4) */
};

/* what the reference did with a frame (values equal the codec's WSC_FK_*) */
enum {
    WSO_FK_FRAG = 0,        /* FIN=0 frame through nextFrame: payload appended to continueBuffer */
    WSO_FK_MESSAGE = 1,     /* FIN=1 data frame: util.Message delivered */
    WSO_FK_PING = 2,        /* PING: payload echoed in a PONG */
    WSO_FK_PONG = 3,        /* PONG with payload: consumed */
    WSO_FK_CLOSE = 4,       /* CLOSE: peer close -> CloseCode(1000) */
    WSO_FK_PONG_EMPTY = 5,  /* PONG with no payload -> Close() (1000) */
    WSO_FK_ERROR = 6,       /* a sentinel error at this frame -> CloseCode(1002|1007) */
    WSO_FK_STALL = 7,       /* unmasked frame: EAGAIN forever (Q3) */
};

enum { WSO_EV_MESSAGE = 1, WSO_EV_PONG = 2, WSO_EV_CLOSE = 3, WSO_EV_STALL = 4 };

typedef struct {
    uint32_t type;        /* WSO_EV_* */
    uint32_t msg_id;      /* MESSAGE: Message.MsgID */
    uint32_t opcode;      /* MESSAGE: Message.Opcode (messageMode) */
    uint32_t close_code;  /* CLOSE: 1000 / 1002 / 1007 */
    uint32_t err;         /* CLOSE: sentinel that caused it (WSO_ERR_*), 0 for a normal close */
    uint32_t pad;
    uint64_t data_off;    /* MESSAGE/PONG payload: offset into the caller's arena */
    uint64_t data_len;
} wso_event;

typedef struct {
    uint64_t hdr_off;      /* stream offset of the frame's first header byte */
    uint64_t payload_off;  /* stream offset of the first payload byte (0 if header never completed) */
    uint64_t payload_len;  /* fragmentLength as parsed */
    uint32_t mask;         /* the 4 mask bytes as a little-endian u32 (wire byte 0 = bits 0..7) */
    uint32_t msg_id;       /* msgID before this frame */
    uint8_t opcode, fin, kind, mode;   /* mode = messageMode after the header */
    uint32_t err;          /* WSO_ERR_* for kind ERROR */
} wso_frame;

typedef struct {
    uint64_t consumed;     /* bytes the simulated socket handed out */
    uint32_t closed;       /* 1 once CloseCode/Close ran */
    uint32_t stalled;      /* 1 when the unmasked-frame stall was detected */
    uint32_t close_code;
    uint32_t err;
    uint32_t msg_id;       /* final msgID */
    uint32_t message_mode; /* final messageMode */
    uint64_t cont_len;     /* final continueBuffer length */
    uint32_t n_events, n_frames;
    uint64_t arena_used;
    uint32_t overflow;     /* an output array was too small */
    uint32_t pad;
} wso_result;

/*
 * Run one connection's post-handshake stream through the restated decoder.
 *   stream/len        the full byte stream
 *   chunk_ends        increasing chunk end offsets (last == len); NULL -> one chunk
 *   max_frame_len     frames longer than this give WSO_ERR_TOO_LARGE at the point the reference
 *                     would make() the payload buffer (websocket_frame.go:17)
 *   inplace           optional len-byte output: copy of stream with every payload the reference
 *                     unmasked (websocket_frame.go:35-39) XORed in place
 * Returns 0, or -1 on overflow of an output array (res->overflow set).
 */
int wso_run(const uint8_t* stream, uint64_t len, const uint64_t* chunk_ends, uint32_t n_chunks,
            uint64_t max_frame_len, uint8_t* inplace,
            wso_event* ev, uint32_t ev_cap, wso_frame* fr, uint32_t fr_cap,
            uint8_t* arena, uint64_t arena_cap, wso_result* res);

/* wso_run with flags: WSO_RUN_EOF -- after the last chunk the peer closes: the next read returns
 * 0, which BaseConnect.Read maps to io.EOF (baseconnect.go:100-103) and the poller answers with
 * Close() = CloseCode(1000, "") (epoll.go:108-110, websocket.go:401-404).  Level-triggered epoll
 * reports the EOF as readable, so DecodePacket is called until it returns that error. */
#define WSO_RUN_EOF 1u
int wso_run_ex(const uint8_t* stream, uint64_t len, const uint64_t* chunk_ends, uint32_t n_chunks,
               uint64_t max_frame_len, uint8_t* inplace,
               wso_event* ev, uint32_t ev_cap, wso_frame* fr, uint32_t fr_cap,
               uint8_t* arena, uint64_t arena_cap, wso_result* res, uint32_t flags);

/* Go 1.16 utf8.Valid restated */
int wso_utf8_valid(const uint8_t* p, uint64_t n);

/* server/websocket_frame.go:35-39 restated on its own: decodeBuffer[i] = buf[i] ^ masks[i%4] */
void wso_unmask(const uint8_t* in, uint8_t* out, uint64_t n, const uint8_t masks[4]);

/*
 * ENCODE side (server -> client framing), server/websocket_ctrl.go:23-70 encode(firstByte, bs):
 * firstByte, then len <= 125 -> one length byte; 126..65535 -> 126 + u16 big-endian;
 * otherwise 127 + u64 big-endian; then the payload, never masked.  Callers: Text 0x81 / Binary
 * 0x82 (websocket.go:378-398), pong 0x8A (websocket_ctrl.go:140-143), CloseCode 0x88
 * (websocket_ctrl.go:108-109).  Writes into out (room for len + 10) and returns the frame size.
 */
uint64_t wso_encode(uint8_t first_byte, const uint8_t* bs, uint64_t len, uint8_t* out);

/* A batch of encodes back to back: message i = src[src_off[i] .. +len[i]) with first_byte[i];
 * out_off[i] = where frame i starts, out_off[n] = total.  Returns the total. */
uint64_t wso_encode_batch(const uint8_t* src, const uint64_t* src_off, const uint64_t* len,
                          const uint8_t* first_byte, uint32_t n, uint8_t* out, uint64_t* out_off);

#ifdef __cplusplus
}
#endif
#endif
