/*
 * wscodec.h -- C ABI of the MI355X WebSocket frame codec (libwscodec.so).
 *
 * This is the drop-in boundary for netman's websocket DECODE path.  In the
 * reference (pure Go) the path sits behind the internal interface
 *     iface.IConnectEvent.DecodePacket() (IMessage, error)          iface/iconnect.go:38-39
 * implemented by websocketProtocol.DecodePacket                       server/websocket.go:82-212
 *   -> parseHeadBytes / parsePayloadLength                            server/websocket.go:214-302
 *   -> nextFrame (XOR unmask at :35-39, reassembly, utf8, Message)    server/websocket_frame.go:13-103
 * and its results reach the public iface.IWebsocketHandler.Message    iface/iwebsockethandler.go:4-8
 * with the error -> close-code mapping of eventloop/epoll.go:106-129.
 *
 * The ABI replaces that per-frame, per-read decode with ONE batched call over many connections'
 * bulk socket reads ("segments"), run as hand-written gfx950 kernels:
 *   wsc_decode()        device-resident batch (the hot path)        replaces websocket.go:82-302 +
 *                                                                   websocket_frame.go:13-103
 *   wsc_decode_host()   host buffers in/out through pinned staging  same, plus the readData copy
 *   wsc_session_*       per-connection DecodePacket() mirror        replaces IConnectEvent.DecodePacket
 *                       (pending-message queue, carry-over)         (iface/iconnect.go:38-39)
 * Plain pointers and sizes only; no exceptions cross the ABI; every function returns WSC_OK (0)
 * or a negative WSC_E_* code.  INTEGRATION.md shows the cgo binding a netman maintainer would add.
 */
#ifndef WSCODEC_H
#define WSCODEC_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define WSC_ABI_VERSION 5   /* 2: wsc_frame.payload_len_hi (40-bit payload lengths), staged split;
                               3: payloads streamed across batches (wsc_conn_state.frame_*, WSC_FK_PIECE);
                               4: PONG payloads stream too (wsc_conn_state.frame_utf8), session EOF,
                                  no-progress guard and per-connection message cap;
                               5: no environment variable is read: the walk variants the tests pin are
                                  wsc_config fields (walk_mode, u8_inline_max, walk_flags), the
                                  session's are wsc_session_create flags; wsc_session_inject_fault */

/* ---- return codes --------------------------------------------------------------------------- */
#define WSC_OK 0
#define WSC_E_INVAL (-1)     /* bad argument / shape */
#define WSC_E_DEVICE (-2)    /* HIP runtime error (wsc_last_error() has the text) */
#define WSC_E_NOMEM (-3)     /* allocation failed */
#define WSC_E_CAPACITY (-4)  /* batch exceeds the context's configured capacity */
#define WSC_E_NODEVICE (-5)  /* no usable gfx950 device */
#define WSC_E_STATE (-6)     /* session misuse (unknown / closed connection) */
#define WSC_E_INTERNAL (-7)  /* device-side look-back timeout: the batch's results are INVALID (never
                                silently reported as capacity; see wsc_summary.overflow bit 1)     */

/* ---- per-frame error sentinels: util/errors.go:9-14 (same order/values as the oracle) -------- */
#define WSC_ERR_NONE 0
#define WSC_ERR_OPCODE_FAIL 1            /* WebsocketOpcodeFail                     -> 1002 */
#define WSC_ERR_RSV_FAIL 2               /* WebsocketRsvFail                        -> 1002 */
#define WSC_ERR_PING_PAYLOAD_OVERSIZE 3  /* WebsocketPingPayloadOversize            -> 1002 */
#define WSC_ERR_CTRL_FRAGMENTED 4        /* WebsocketCtrlMessageMustNotFragmented   -> 1002 */
#define WSC_ERR_MUST_UTF8 5              /* WebsocketMustUtf8                       -> 1007 */
#define WSC_ERR_PROTOCOL_ERROR 6         /* WebsocketProtocolError                  -> 1002 */
#define WSC_ERR_TOO_LARGE 7              /* payload > max_frame_len (reference would panic, Q4) -> 1002 */
#define WSC_ERR_DEVICE 8                 /* session only: the connection's batch hit a device error
                                            -> CloseCode(1011); see wsc_session_* below           */
#define WSC_ERR_NO_PROGRESS 9            /* session only: a whole batch of the connection's bytes decoded
                                            nothing (a header or PING/CLOSE frame longer than
                                            max_batch_bytes, which must be >= 139 to rule it out)
                                            -> CloseCode(1009) instead of re-sending it forever    */
#define WSC_ERR_MSG_TOO_BIG 10           /* session only: the connection's buffered message passed the
                                            cap set by wsc_session_set_max_message (off by default:
                                            the reference has none, Q4) -> CloseCode(1009)          */

/* ---- what the decoder did with a frame (websocket.go:136-208 / websocket_frame.go:52-102) --- */
#define WSC_FK_FRAG 0        /* FIN=0 through nextFrame: payload appended to continueBuffer      */
#define WSC_FK_MESSAGE 1     /* FIN=1 data frame: util.Message{MsgID=msg_id, Opcode=mode}        */
#define WSC_FK_PING 2        /* PING: reply PONG echoing the payload (websocket_ctrl.go:128-153) */
#define WSC_FK_PONG 3        /* PONG with payload: consumed                                      */
#define WSC_FK_CLOSE 4       /* CLOSE frame: reply CloseCode(1000) and close                     */
#define WSC_FK_PONG_EMPTY 5  /* PONG without payload: Close() (websocket.go:198-201)             */
#define WSC_FK_ERROR 6       /* sentinel `err` at this frame: CloseCode(1002|1007)               */
#define WSC_FK_STALL 7       /* unmasked client frame: reference returns EAGAIN forever (Q3)     */
#define WSC_FK_PIECE 8       /* the payload bytes of a data frame or PONG that is not complete at the
                                end of its segment (nextFrame's partial read into rBuffer,
                                websocket_frame.go:16-31): unmasked, nothing delivered yet.  The
                                frame continues in the connection's next segment (state_out.frame_*);
                                its last piece carries the frame's real kind (MESSAGE, FRAG or PONG) */

/* Streaming (ABI 3; PONG since ABI 4).  A data frame (opcode 0/1/2) or a PONG -- the reference puts
 * no size limit on a PONG and accumulates its payload over reads like any frame's
 * (websocket.go:191-205, websocket_frame.go:16-31) -- whose header is complete is consumed as its
 * payload arrives: each batch unmasks the bytes it holds and records them (WSC_FK_PIECE, then the
 * final kind on the piece that completes the frame), and the connection carries only
 * {frame_rem, frame_mask, frame_hdr, frame_len} -- never the payload -- to its next segment, which
 * starts with the rest of that payload.  A record whose header lay in an earlier batch has
 * WSC_FF_HEAD_PREV, hdr_len 0 and hdr_off = its first payload byte; its `mask` is phased to that
 * byte.  The frame's data is the concatenation of its pieces' payloads, in order.  A PONG's pieces go
 * to the control region in COMPACT mode; under messageMode TEXT the PONG payload alone is UTF-8
 * checked when its last piece arrives (Q6), its DFA state carried in frame_utf8.  PING and CLOSE
 * frames (<= 125 B by rule) and incomplete headers are still carried whole (seg_result.consumed
 * stops before them: at most 139 bytes).                                                         */

/* wsc_frame.flags */
#define WSC_FF_UNMASKED 0x01  /* payload went through nextFrame and was XOR-unmasked             */
#define WSC_FF_CONT_MSG 0x02  /* MESSAGE whose data = continueBuffer || this payload (:62-68)    */
#define WSC_FF_U8_PART 0x04   /* internal: FRAG of a TEXT chain (utf8 state carried)            */
#define WSC_FF_U8_SELF 0x08   /* internal: payload alone must be valid utf8                     */
#define WSC_FF_U8_CHAIN 0x10  /* internal: continueBuffer || payload must be valid utf8          */
#define WSC_FF_U8_REASON 0x20 /* internal: CLOSE reason payload[2:] must be valid utf8          */
#define WSC_FF_CTRL_ARENA 0x40 /* COMPACT: payload placed in the control region of the arena    */
#define WSC_FF_HEAD_PREV 0x80  /* the frame's header was in an earlier batch (hdr_len 0)          */

/* ---- per-connection terminal status ---------------------------------------------------------- */
#define WSC_SEG_OPEN 0      /* connection continues; bytes [consumed, len) are carried over        */
#define WSC_SEG_CLOSED 1    /* CLOSE frame or empty PONG: CloseCode(1000, "")                       */
#define WSC_SEG_ERROR 2     /* protocol error: CloseCode(close_code = 1002 | 1007), see err        */
#define WSC_SEG_STALLED 3   /* unmasked frame: nothing more is ever delivered (Q3)                  */

/* batch flags */
#define WSC_F_COMPACT 0x1   /* write unmasked payloads compacted into `arena` instead of unmasking
                               the wire buffer in place.  Arena layout: segments in order, each as
                               [data payloads (continuation chains contiguous)][control payloads]; a
                               frame's payload is at frame_dst[i]                                  */

/* session flags (wsc_session_create; batch flags above apply too) */
#define WSC_SESSION_BLOCKING_WAIT 0x100   /* complete() sleeps on a blocking-sync event instead of
                                             spinning in hipStreamSynchronize: the poller's core is
                                             free for recv/send while the device works (many pollers
                                             on few cores)                                          */
#define WSC_SESSION_TIMING 0x200          /* diagnostics: seconds per phase (pack, launch, device
                                             wait, harvest) printed to stderr at destroy            */
#define WSC_SESSION_COPY_ENGINE 0x400     /* every staging copy by hipMemcpyAsync (the copy engines);
                                             by default the wire's H2D is a wsc_kcopy kernel        */
#define WSC_SESSION_KCOPY_ALL 0x800       /* every staging copy by wsc_kcopy kernels                */

/* Decoder state carried between batches for one connection (subset of websocket.go:38-56).   */
typedef struct wsc_conn_state {
    uint64_t cont_len;     /* continueBuffer length (bytes of an unfinished fragmented message)  */
    uint32_t msg_id;       /* msgID: next Message.MsgID                                          */
    uint8_t message_mode;  /* messageMode: 0, 1 (text) or 2 (binary)                             */
    uint8_t cont_utf8;     /* utf8 DFA state after continueBuffer and the in-progress frame's
                              bytes so far (0 = complete characters)                              */
    uint8_t status;        /* WSC_SEG_*; a connection that is not OPEN decodes nothing           */
    uint8_t frame_hdr;     /* in-progress frame (frame_rem != 0): FIN << 7 | opcode              */
    uint64_t frame_rem;    /* payload bytes of the in-progress frame still to come; 0 = the next
                              byte starts a header (websocket_frame.go:16 rLen)                   */
    uint64_t frame_len;    /* its whole payload length (fragmentLength)                          */
    uint32_t frame_mask;   /* its mask, phased so that the next payload byte takes wire byte 0   */
    uint8_t frame_utf8;    /* an in-progress PONG under messageMode TEXT: utf8 DFA state after its
                              bytes so far (its own check, Q6; cont_utf8 stays the message's)     */
    uint8_t pad[3];
} wsc_conn_state;          /* 40 B.  Once status is not OPEN only status is meaningful (a closed
                              connection decodes nothing more); frame_* are then zero           */

/* One record per frame whose header was parsed and acted on, in stream order.                  */
typedef struct wsc_frame {
    uint64_t hdr_off;      /* batch offset of the frame's first header byte                      */
    uint32_t payload_len;  /* fragmentLength, low 32 bits (the reference parses 64: websocket.go:291-299) */
    uint32_t mask;         /* the 4 mask bytes, wire byte 0 in bits 0..7                         */
    uint32_t seg;          /* segment (connection slot) index                                    */
    uint32_t msg_id;       /* msgID before this frame (Message.MsgID for WSC_FK_MESSAGE)         */
    uint8_t opcode;        /* header opcode                                                      */
    uint8_t fin;           /* header FIN bit                                                     */
    uint8_t kind;          /* WSC_FK_*                                                           */
    uint8_t mode;          /* messageMode after this header (Message.Opcode for MESSAGE)        */
    uint8_t err;           /* WSC_ERR_* for WSC_FK_ERROR                                         */
    uint8_t hdr_len;       /* 6 / 8 / 14 for complete masked headers; payload_off = hdr_off+hdr_len */
    uint8_t flags;         /* WSC_FF_*                                                           */
    uint8_t payload_len_hi; /* fragmentLength bits 32..39: length = payload_len | hi << 32         */
} wsc_frame;               /* 32 B */

/* Per-segment result.                                                                          */
typedef struct wsc_seg_result {
    uint64_t consumed;     /* bytes of the segment fully decoded (carry = [consumed, seg_len))   */
    uint32_t frame_begin;  /* index of the segment's first wsc_frame                             */
    uint32_t frame_count;
    uint32_t status;       /* WSC_SEG_*                                                          */
    uint32_t close_code;   /* 1000 / 1002 / 1007 when status is CLOSED or ERROR                  */
    uint32_t err;          /* WSC_ERR_* when status == WSC_SEG_ERROR                             */
    uint32_t pad;
} wsc_seg_result;          /* 32 B */

/* Batch totals written by the device.                                                          */
typedef struct wsc_summary {
    uint64_t data_bytes;   /* COMPACT: data payload bytes in the arena (all segments)            */
    uint64_t ctrl_bytes;   /* COMPACT: control payload bytes in the arena                         */
    uint32_t n_frames;     /* records written to `frames` (a segment's frame_count can be smaller:
                              a late UTF-8 verdict stops a segment at its failing frame)          */
    uint32_t n_spans;      /* payload spans unmasked                                              */
    uint32_t overflow;     /* bit0: n_frames > frames_cap (records beyond the cap were dropped);
                              bit1: internal look-back timeout (results invalid).  Callers of the
                              async wsc_decode check it with wsc_summary_status() or, for many
                              batches at once, wsc_error_flags()                                  */
    uint32_t pad;
} wsc_summary;

typedef struct wsc_batch {
    uint8_t* wire;                   /* device: n_bytes, all segments back to back               */
    uint64_t n_bytes;
    const uint64_t* seg_off;         /* device: n_segs+1 offsets, [0]=0, [n_segs]=n_bytes        */
    uint32_t n_segs;
    uint32_t flags;                  /* WSC_F_*                                                  */
    const wsc_conn_state* state_in;  /* device: n_segs (NULL = fresh connections)               */
    wsc_conn_state* state_out;       /* device: n_segs                                           */
    wsc_seg_result* seg_out;         /* device: n_segs                                           */
    wsc_frame* frames;               /* device: frames_cap                                       */
    uint32_t frames_cap;
    uint32_t pad;
    uint8_t* arena;                  /* device, COMPACT only: >= n_bytes + 64 bytes              */
    uint64_t* frame_dst;             /* device, COMPACT only: per-frame arena offset             */
    wsc_summary* summary;            /* device: 1                                                */
} wsc_batch;

typedef struct wsc_config {
    uint64_t max_batch_bytes;  /* largest n_bytes a batch may have                               */
    uint32_t max_segs;         /* largest n_segs                                                 */
    uint32_t max_frames;       /* largest number of frames in one batch                          */
    uint64_t max_frame_len;    /* payloads above this -> WSC_ERR_TOO_LARGE (<= 2^40 - 1, the
                                  default: the record width; the reference has no limit until
                                  make() fails, Q4).  Independent of max_batch_bytes: payloads
                                  stream across batches                                          */
    uint32_t unmask_window;    /* bytes per wave-window in the unmask kernel: 4096 (0 = 4096)       */
    uint32_t unmask_waves_per_cu; /* unmask grid sizing (0 = one window per wave, the default)    */
    uint32_t unmask_nt;        /* cache policy of the unmask: 0 or the default (in place: non-temporal
                                  loads and stores; COMPACT: non-temporal loads); other policies were
                                  measured slower and are not built (WSC_E_INVAL)                  */
    uint32_t unmask_minw;      /* reserved (0); was an occupancy hint, measured no gain        */
    /* ABI 5: the header-walk variants (same results; tests pin them, wsc_walk_info reports them) */
    uint32_t walk_mode;        /* 0 = automatic; 16, 32, 64, 65, 66, 256, 257 (fused walks) or 3 (the
                                  tiled walk) pins the geometry                                    */
    uint32_t u8_inline_max;    /* TEXT payloads up to this many bytes are UTF-8 validated inside the
                                  walk, larger ones chip-wide after the unmask (default 256; 0 = all
                                  chip-wide; values above 4095 act as 4095)                        */
    uint32_t walk_flags;       /* WSC_WALK_* below (default 0)                                      */
    uint32_t pad;
} wsc_config;

#define WSC_WALK_NO_QUAD_PRE 0x1   /* the fused walk without its quad pre-pass (modes 65, 16)        */
#define WSC_WALK_NO_HDR_CACHE 0x2  /* the tiled walk re-reads each segment's first header          */
#define WSC_WALK_HDR_NT 0x4        /* non-temporal header loads for in-place batches too (COMPACT
                                      batches always use them)                                      */
#define WSC_WALK_DEBUG_STAMPS 0x8  /* per-block s_memrealtime stamps of the walk (wsc_debug_stamps) */

typedef struct wsc_ctx wsc_ctx;

int wsc_abi_version(void);
const char* wsc_last_error(void);
int wsc_config_default(wsc_config* cfg);

int wsc_create(int device, const wsc_config* cfg, wsc_ctx** out);
int wsc_destroy(wsc_ctx* ctx);

int wsc_dev_alloc(wsc_ctx* ctx, uint64_t bytes, void** out);
int wsc_dev_free(wsc_ctx* ctx, void* p);
int wsc_host_alloc(uint64_t bytes, void** out);   /* pinned (hipHostMalloc) */
int wsc_host_free(void* p);
/* Enqueue a copy of `bytes` between device memory and pinned host memory (wsc_host_alloc; either
 * side, or both device) done by a kernel, which reads or writes the host buffer over PCIe: the
 * call returns once the kernel is queued.  On this platform a hipMemcpyAsync to or from pinned
 * memory can hold the calling thread for about the copy's duration (a poller then waited ~3-7 ms
 * per 20 MB round at 4-8 pollers), so wsc_session makes its copies with this.  Any alignment
 * (16-byte chunks between 16-byte aligned ends are fastest); the source must stay unchanged
 * until the stream passes the copy.  WSC_E_INVAL for memory the device cannot reach (pageable
 * host memory): checked on the host, never faulted on.                                          */
int wsc_kcopy(wsc_ctx* ctx, void* dst, const void* src, uint64_t bytes, void* hip_stream);

/* Enqueue the decode of one device-resident batch on `hip_stream` (a hipStream_t; NULL = the
 * default stream, as everywhere in HIP).  Asynchronous: results are valid once the stream is
 * synchronised (wsc_sync with the same stream).  Inputs must be ready on that stream.
 * A batch whose summary has overflow bit 0 set (records beyond frames_cap) is INVALID as a whole:
 * besides the dropped records, its chip-wide UTF-8 verdicts were not applied (a TEXT frame that
 * should have closed with 1007 may read as a MESSAGE) -- re-decode it in smaller parts, as
 * wsc_session does.  Check with wsc_summary_status() or wsc_error_flags(). */
int wsc_decode(wsc_ctx* ctx, const wsc_batch* batch, void* hip_stream);
int wsc_sync(wsc_ctx* ctx, void* hip_stream);

/* Map a batch's (host copy of) wsc_summary to a return code: WSC_OK, WSC_E_INTERNAL (bit 1:
 * results invalid) or WSC_E_CAPACITY (bit 0: records dropped).  Pure host function.            */
int wsc_summary_status(const wsc_summary* summary);

/* Sticky error bits of every decode / encode run on this context since it was created or last
 * cleared: bit0 frame capacity exceeded, bit1 decode look-back timeout, bit2 encode look-back
 * timeout.  Synchronises the device.  `clear` != 0 resets them.  Lets a caller that pipelines
 * many async batches (bench, a poller) verify all of them with one call.                        */
int wsc_error_flags(wsc_ctx* ctx, uint32_t* flags, int clear);

/* Split pipeline: the header walk runs on `walk_stream`, the UTF-8 check and unmask on
 * `unmask_stream`, joined by the context's events.  The walk waits for this context's previous
 * split decode to finish, so batches of different contexts overlap: the walk of one batch runs
 * beside the unmask of the other.  Inputs must be ready on `walk_stream`; results are valid once
 * `unmask_stream` is synchronised.  Pair it with CU-masked streams (wsc_stream_create) so that
 * the walk has CUs the unmask grid does not occupy.  As with wsc_decode, a context runs one
 * decode at a time: order a split decode and any other call on the same context yourself.     */
int wsc_decode_split(wsc_ctx* ctx, const wsc_batch* batch, void* walk_stream, void* unmask_stream);

/* The split decode in two calls, for a host that pipelines batches: wsc_decode_walk enqueues
 * the header walk on `walk_stream`; wsc_decode_finish enqueues the rest (UTF-8 check, unmask) on
 * `unmask_stream`, joined to the walk by a stream wait only if it has not completed yet, and
 * without the check's launch when the completed walk deferred no text.  The staged unmask records
 * no event: its last workgroup signals the host through a pinned word, and the context's next
 * decode waits for that on the host before it reuses the walk's scratch (so a host that pipelines
 * keeps two or more contexts).  wsc_walk_wait blocks the host until the context's last walk has
 * completed: calling it between the two (while the device still unmasks the previous batch) makes
 * the unmasks of consecutive batches follow each other on their stream with nothing in between.
 * Results of a finished decode are read after synchronising `unmask_stream` as usual.        */
int wsc_decode_walk(wsc_ctx* ctx, const wsc_batch* batch, void* walk_stream);
int wsc_decode_finish(wsc_ctx* ctx, const wsc_batch* batch, void* unmask_stream);
int wsc_walk_wait(wsc_ctx* ctx);

/* A non-blocking stream on the context's device, restricted to the CUs whose bits are set in
 * cu_mask[0..mask_words) (hipExtStreamCreateWithCUMask); cu_mask NULL = all CUs.             */
int wsc_stream_create(wsc_ctx* ctx, const uint32_t* cu_mask, uint32_t mask_words, void** out);
/* Same, with a queue priority: priority > 0 = the device's greatest stream priority, < 0 = its
 * least, 0 = wsc_stream_create.  A prioritised stream spans all CUs (cu_mask must be NULL): the
 * staged pipeline's walk stream, beside unmasks on a normal stream.  (The walk's waves also raise
 * their SIMD issue priority, s_setprio, whatever stream they run on.)                          */
int wsc_stream_create_ex(wsc_ctx* ctx, const uint32_t* cu_mask, uint32_t mask_words, int priority, void** out);
int wsc_stream_destroy(wsc_ctx* ctx, void* stream);

/* Host-buffer path: copies wire/offsets/state to the device through the context's pinned
 * staging, decodes, and copies results back (synchronous).  In-place mode rewrites `wire`;
 * COMPACT mode fills `arena` (host, >= n_bytes + 64).  `frames` has room for `frames_cap`. */
int wsc_decode_host(wsc_ctx* ctx, uint8_t* wire, uint64_t n_bytes, const uint64_t* seg_off,
                    uint32_t n_segs, uint32_t flags, const wsc_conn_state* state_in,
                    wsc_conn_state* state_out, wsc_seg_result* seg_out, wsc_frame* frames,
                    uint32_t frames_cap, uint8_t* arena, uint64_t* frame_dst, wsc_summary* summary);

/* ---- encode: batched server -> client framing ------------------------------------------------
 * Replaces websocketProtocol.encode(firstByte, bs) (server/websocket_ctrl.go:23-70) as used by
 * Text / Binary (server/websocket.go:378-398), pong (websocket_ctrl.go:140-143) and CloseCode
 * (websocket_ctrl.go:108-109): each message becomes firstByte, a minimal 7/16/64-bit big-endian
 * length, then the payload, unmasked.  A batch frames many messages (many connections) back to
 * back into one output buffer in one device call.                                              */
typedef struct wsc_out_msg {
    uint64_t src_off;      /* payload offset in `src`                                            */
    uint64_t len;          /* payload length                                                     */
    uint8_t first_byte;    /* 0x81 Text, 0x82 Binary, 0x8A pong, 0x88 close (FIN | opcode)       */
    uint8_t pad[7];
} wsc_out_msg;             /* 24 B */

/* Enqueue the framing of n_msgs messages (device-resident `msgs`, `src`; both `src` and `out`
 * 16-byte aligned).  Frame i is written at out + out_off[i]; out_off[n_msgs] = total bytes.
 * Bytes at or past out_cap are never written: the caller checks out_off[n_msgs] <= out_cap.
 * Capacity: n_msgs <= max_frames, out_cap <= max_batch_bytes + 16 * max_frames.  Async on
 * hip_stream (NULL = default stream); the context runs one decode or encode at a time.          */
int wsc_encode(wsc_ctx* ctx, const wsc_out_msg* msgs, uint32_t n_msgs, const uint8_t* src,
               uint64_t src_bytes, uint8_t* out, uint64_t out_cap, uint64_t* out_off, void* hip_stream);

/* Host-buffer encode (synchronous): H2D of msgs + src, wsc_encode, D2H of out_off and the frames.
 * Returns WSC_E_CAPACITY if the frames need more than out_cap bytes.                            */
int wsc_encode_host(wsc_ctx* ctx, const wsc_out_msg* msgs, uint32_t n_msgs, const uint8_t* src,
                    uint64_t src_bytes, uint8_t* out, uint64_t out_cap, uint64_t* out_off);

/* Timing helper for the benchmark: run `iters` back-to-back decodes of a device batch and
 * return the per-kernel average device time (ms) measured with hipEvents on the launch stream.
 * out_ms[0] = fused header walk (incl. inline utf8), [1] = chip-wide utf8 check of deferred text,
 * [2], [4] = 0 (reserved), [3] = unmask,
 * [5] = whole decode.  A context runs one decode at a time (its scratch is shared). */
int wsc_profile(wsc_ctx* ctx, const wsc_batch* batch, int iters, double* out_ms);

/* Diagnostics: with WSC_WALK_DEBUG_STAMPS in wsc_config.walk_flags at wsc_create, the header-walk kernel
 * records per block 8 u64 slots of s_memrealtime stamps (100 MHz): start, counted, look-back done,
 * emitted, quad pre-pass done (0 if none), 3 reserved.  `out` has room for 8 * max_blocks.     */
int wsc_debug_stamps(wsc_ctx* ctx, uint64_t* out, uint32_t max_blocks);

/* Diagnostics: the header-walk geometry the context's last decode launched (*mode: 16, 32, 64, 65,
 * 66, 256, 257 = fused walks, 3 = tiled; 0 before any decode) and its block count.
 * Tests use it to check that a geometry pinned with wsc_config.walk_mode really ran.            */
int wsc_walk_info(wsc_ctx* ctx, uint32_t* mode, uint32_t* blocks);

/* ---- session: the per-connection DecodePacket() mirror (C++ host side above the ABI) ---------
 * One session per poller thread (eventloop/epoll.go:36-143).  Per round the poller reads each
 * ready connection once -- straight into the session's pinned staging with wsc_session_reserve +
 * recv + wsc_session_commit (the only host copy is the kernel's socket copy), or with
 * wsc_session_feed (one memcpy) -- then wsc_session_decode (= submit + complete), and drains every
 * connection with wsc_session_next, which yields what DecodePacket + epoll.go:104-140 would have
 * (one message / PONG reply / close per call, in order).  Double-buffered variant: submit round
 * r+1 and send round r's replies while its H2D + kernels run, then complete it.
 *
 * Threading: wsc_session_remove may be called from ANY thread at any time (netman calls Close()
 * -> remove() from handler and heartbeat goroutines, websocket_ctrl.go:73-96); it only queues the
 * handle and the owning poller thread applies it at its next session call, after which the handle
 * is invalid (WSC_E_STATE) and nothing more is delivered for it.  All other functions belong to
 * the single thread that owns the session.  Handles carry a generation: a stale handle of a
 * removed connection never touches a newer connection in the same slot.
 *
 * Capacity is per connection: frames of any size up to max_frame_len stream through batches of
 * any size (each batch unmasks the payload bytes it holds; the session appends them to the
 * connection's rBuffer and delivers the message when its last byte has been decoded, as
 * websocket_frame.go:16-31 does), so every wire byte crosses PCIe once except an incomplete header
 * or control frame at a segment's end (<= 139 B, sent again with the next bytes); a connection
 * with more bytes than a batch holds is decoded from a prefix and continues in the next batch; a
 * batch with more frame records than max_frames is re-decoded in halves.
 *
 * Ordering: reads (reserve/commit, feed) are accepted at any time, including while a submitted
 * batch is in flight; a connection whose previous bytes are in that batch gets its new bytes
 * staged behind the batch's undecoded tail, which complete() establishes -- they are placed in a
 * batch only after it.
 *
 * Device failure (WSC_E_DEVICE / WSC_E_INTERNAL from decode/complete): the connections of the
 * failed batch get WSC_EV_CLOSE with close_code 1011 and err WSC_ERR_DEVICE, keep their carried
 * bytes (wsc_session_state) and decode nothing more; other connections are untouched.  There is
 * no CPU fallback.  (The reference drops all of a poller's connections when epoll_wait fails,
 * eventloop/epoll.go:41-49.)
 *
 * EOF rule.  In the reference a read returning 0 becomes io.EOF (BaseConnect.Read,
 * baseconnect.go:100-103) and the poller then calls Close() (epoll.go:108-110) -- but only after
 * every frame read before it was delivered, since each DecodePacket consumes at most one frame and
 * the EOF read comes once the socket buffer is empty.  A bulk reader must keep that order: on a
 * zero-byte read call wsc_session_eof(conn) and keep draining wsc_session_next as usual.  The
 * session decodes every byte read before the EOF (submit / complete as usual: wsc_session_pending
 * stays non-zero while any is left), delivers their events, and then yields WSC_EV_CLOSE with
 * close_code 1000 and err 0 -- Close() -- as the connection's last event; an incomplete frame at
 * the EOF is dropped (the reference's next read of it returns io.EOF).  Do NOT close the socket on
 * the zero-byte read itself: that loses the messages still queued or in flight.
 *
 * Byte source and TLS.  The staging takes the connection's POST-TLS byte stream: exactly what the
 * reference's readData returns (baseconnect.go:347-353) -- unix.Read on the fd for a plain
 * connection, tls.Conn.Read on the layer built at baseconnect.go:56-63 when TLS is on (wss; the
 * poller completes the TLS handshake first, epoll.go:85-102).  The codec never sees ciphertext.  A
 * tls.Conn returns at most one record's plaintext per Read and keeps the rest in its own buffers,
 * which level-triggered epoll cannot see: a TLS reader fills its reserved room with repeated Reads
 * until the layer reports EAGAIN (or the room is full, and then reads again next round without
 * waiting for EPOLLIN), and maps the layer's io.EOF to wsc_session_eof.  INTEGRATION.md has both
 * branches of the Go shim.
 *
 * Livelock guard: a batch in which one connection's whole segment (max_batch_bytes of its bytes)
 * decoded nothing -- possible only for a header or PING / CLOSE frame longer than the batch, i.e.
 * max_batch_bytes < 139 -- closes that connection (WSC_EV_CLOSE 1009, WSC_ERR_NO_PROGRESS) instead
 * of re-sending the same bytes forever.  PONG and data payloads of any length stream.            */
typedef struct wsc_session wsc_session;

/* events popped by wsc_session_next(); mirrors what DecodePacket + epoll.go:104-140 produce   */
#define WSC_EV_NONE 0      /* (nil, EAGAIN): nothing pending for this connection               */
#define WSC_EV_MESSAGE 1   /* (Message, nil): deliver to IWebsocketHandler.Message             */
#define WSC_EV_PONG 2      /* PING answered: send a PONG frame with `data`                     */
#define WSC_EV_CLOSE 3     /* CloseCode(close_code); err = sentinel (0 for a normal close)      */
#define WSC_EV_STALL 4     /* unmasked frame: nothing more will be delivered (Q3)              */

typedef struct wsc_event {
    uint32_t type;        /* WSC_EV_* */
    uint32_t msg_id;      /* MESSAGE: Message.MsgID */
    uint32_t opcode;      /* MESSAGE: Message.Opcode (1 text, 2 binary) */
    uint32_t close_code;  /* CLOSE */
    uint32_t err;         /* CLOSE: WSC_ERR_* */
    uint32_t pad;
    const uint8_t* data;  /* MESSAGE / PONG payload.  Valid until the FIRST of: the next
                             wsc_session_complete / wsc_session_decode, or the connection's
                             removal being applied -- so a round's replies can be sent straight
                             from it (writev) while the next batch decodes.  Copy it to keep it
                             longer (the reference hands each handler a fresh buffer,
                             websocket_frame.go:90).                                           */
    uint64_t len;
} wsc_event;

int wsc_session_create(int device, const wsc_config* cfg, uint32_t flags, wsc_session** out);
int wsc_session_destroy(wsc_session* s);
int wsc_session_open(wsc_session* s, uint32_t* conn_out);            /* newWebsocketProtocol */
int wsc_session_remove(wsc_session* s, uint32_t conn);               /* remove(): any thread */
/* Room for up to max_bytes of conn's next socket read: *ptr / *avail (avail may be smaller when
 * the staging is nearly full; *ptr == NULL when the connection is closed: read nothing).  Follow
 * with wsc_session_commit(conn, bytes actually read) before any other call for this session.   */
int wsc_session_reserve(wsc_session* s, uint32_t conn, uint64_t max_bytes, uint8_t** ptr, uint64_t* avail);
int wsc_session_commit(wsc_session* s, uint32_t conn, uint64_t n);
int wsc_session_feed(wsc_session* s, uint32_t conn, const uint8_t* bytes, uint64_t n);   /* reserve+memcpy+commit */
int wsc_session_submit(wsc_session* s);    /* async device pass over everything fed (one batch)  */
int wsc_session_complete(wsc_session* s);  /* wait for it, queue each connection's events        */
int wsc_session_decode(wsc_session* s);    /* submit + complete until everything fed is decoded  */
/* Bytes fed but not yet submitted (a batch takes what fits; the rest waits in per-connection
 * spills): a double-buffered poller submits again while this is non-zero, new reads or not.   */
int wsc_session_pending(wsc_session* s, uint64_t* bytes);
/* *ready = 1 when wsc_session_complete would not wait for the device (nothing in flight, or the
 * submitted batch's work has finished), 0 otherwise.  Lets a thread that shares a session among
 * pollers (one batching thread per device) hold the session's lock only for calls that do not
 * block: submit, poll ready without the lock, then complete.                                   */
int wsc_session_ready(wsc_session* s, int* ready);
int wsc_session_next(wsc_session* s, uint32_t conn, wsc_event* ev);  /* DecodePacket() */
/* The peer closed: a read returned 0 (see the EOF rule above).  Reads for conn stop; its queued
 * and still-undecoded bytes are delivered, then WSC_EV_CLOSE 1000 / err 0.                      */
int wsc_session_eof(wsc_session* s, uint32_t conn);
/* Optional per-connection memory cap: a message whose bytes (its fragments and streamed pieces
 * so far included) pass `bytes` closes the connection with WSC_EV_CLOSE 1009 /
 * WSC_ERR_MSG_TOO_BIG instead of being buffered.  0 (the default) = no cap, like the reference
 * (Q4: it buffers any size until make() fails), so one peer can make the session buffer up to
 * max_frame_len bytes per frame and any number of fragments.                                    */
int wsc_session_set_max_message(wsc_session* s, uint64_t bytes);
int wsc_session_state(wsc_session* s, uint32_t conn, wsc_conn_state* st, uint64_t* carry_bytes);
/* Byte accounting since create: out[0] bytes read (committed / fed), out[1] bytes sent to the
 * device (H2D of batch wires), out[2] of those, bytes sent again (carried incomplete headers and
 * control frames), out[3] batches, out[4] bytes of streamed payload pieces delivered into
 * messages.  n = how many of these to write (<= 5).                                            */
int wsc_session_stats(wsc_session* s, uint64_t* out, uint32_t n);
/* Test hook: the session's k-th device submission from now (k >= 1; 0 = off) fails as a failed
 * launch would (WSC_E_DEVICE): its connections get the 1011 closes of the device-failure rule.    */
int wsc_session_inject_fault(wsc_session* s, uint64_t k);

#ifdef __cplusplus
}
#endif
#endif /* WSCODEC_H */
