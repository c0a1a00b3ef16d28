/*
 * wsgpu.h — C ABI of the MI355X-native RFC 6455 frame codec (libwsgpu.so).
 *
 * This is the drop-in boundary for snf4j-websocket's frame codec stages.  A JNI
 * shim binds these entry points from Java; nothing here
 * depends on jni.h, torch or any C++ type.  All functions return an int status
 * (0 = success, <0 = API error); protocol errors found in the data are NOT API
 * errors — they are reported per session in wsg_session_result, exactly like
 * the reference reports them per session by throwing InvalidFrameException.
 *
 * Reference interfaces replaced (paths relative to the snf4j tree):
 *   FrameDecoder        snf4j-websocket/.../websocket/frame/FrameDecoder.java:41-403
 *                       (IBaseDecoder<ByteBuffer,Frame>, core/codec/IBaseDecoder.java:49-94)
 *   FrameUtf8Validator  snf4j-websocket/.../websocket/frame/FrameUtf8Validator.java:40-100
 *   Utf8 (DFA)          snf4j-websocket/.../websocket/frame/Utf8.java:28-102
 *   FrameEncoder        snf4j-websocket/.../websocket/frame/FrameEncoder.java:41-136
 *                       (IEncoder<Frame,ByteBuffer>, core/codec/IEncoder.java:44-67)
 * Install point kept unchanged: IWebSocketSessionConfig.switchDecoders/switchEncoders
 *   (IWebSocketSessionConfig.java:123,133; DefaultWebSocketSessionConfig.java:271-281),
 *   pipeline keys "ws-decoder"/"ws-encoder"/"ws-utf8-validator" (IWebSocketSessionConfig.java:61-75).
 */
#ifndef WSGPU_H
#define WSGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WSG_ABI_VERSION 1

/* ------------------------------------------------------------------------ */
/* Per-frame / per-session status codes.                                     */
/* Each code names the exact InvalidFrameException message the reference     */
/* throws (FrameDecoder.java / FrameUtf8Validator.java line cited); the      */
/* numeric argument of the message is wsg_session_result.detail.             */
/* ------------------------------------------------------------------------ */
typedef enum wsg_status {
    WSG_OK = 0,
    WSG_E_OPCODE = 1,          /* "Unexpected opcode value (%d)"                      FrameDecoder.java:200 */
    WSG_E_RSV = 2,             /* "Unexpected non-zero RSV bits (%d)"                 :207 */
    WSG_E_MASKING = 3,         /* "Unexpected payload masking"                        :215 */
    WSG_E_FRAG_CONTROL = 4,    /* "Fragmented control frame"                          :220 */
    WSG_E_CONTROL_LEN = 5,     /* "Invalid payload length (%d) in control frame"      :223 */
    WSG_E_CLOSE_LEN = 6,       /* "Invalid payload length (%d) in close frame"        :226 */
    WSG_E_CONT_OUTSIDE = 7,    /* "Continuation frame outside fragmented message"     :231 */
    WSG_E_NONCONT_INSIDE = 8,  /* "Non-continuation frame while inside fragmented massage" :235 */
    WSG_E_MIN_LEN = 9,         /* "Invalid minimal payload length"                    :241,250 */
    WSG_E_MAX_PAYLOAD = 10,    /* "Invalid maximum payload length"                    :247 */
    WSG_E_TOO_LONG = 11,       /* "Maximum frame length (%d) has been exceeded"       :255 */
    WSG_E_CLOSE_STATUS = 12,   /* "Invalid close frame status code (%d)"              :127 */
    WSG_E_CLOSE_REASON = 13,   /* "Invalid close frame reason value: bytes are not UTF-8" :131 (1007) */
    WSG_E_TEXT_UTF8 = 14,      /* "Invalid text frame payload: bytes are not UTF-8"   FrameUtf8Validator.java:31 (1007) */
    WSG_E_NEG_LEN = 15,        /* "Negative payload length (%d)"        FrameDecoder.available :390 */
    WSG_E_EXT_LEN = 16,        /* "Extended payload length (%d) > %d"   FrameDecoder.available :393
                                  (detail = plen, detail2 = Integer.MAX_VALUE - need) */
    WSG_E_BATCH = 17,          /* frame extent in the batch does not match its header
                                  (a caller bug: never produced by the reference) */
    WSG_E_AGG_TOO_BIG = 18,    /* "Too big payload for aggregated frame"  FrameAggregator.java:93 (1009) */
    WSG_E_INFLATE = 19,        /* InvalidFrameException(DecompressionException("decompression failure: invalid
                                  compressed data format")): its message is the cause's toString()
                                  (ZlibDecoder.java:256, DeflateDecoder.java:73-76,104-106) (1002) */
    WSG_E_INFLATE_NO_DATA = 20,/* "Inflating of input data produced no data"  DeflateDecoder.java:129 (1002) */
    WSG_E_INFLATE_CAPACITY = 21/* the session's output region is too small (a caller contract, never
                                  produced by the reference): nothing of the session is committed */
} wsg_status;

/* API return codes (<0). */
#define WSG_API_OK 0
#define WSG_API_EINVAL (-1)
#define WSG_API_EHIP (-2)
#define WSG_API_ENOMEM (-3)
#define WSG_API_ERANGE (-4)

/* Close codes the reference writes with writenf(new CloseFrame(code)). */
#define WSG_CLOSE_PROTOCOL_ERROR 1002  /* CloseFrame.PROTOCOL_ERROR */
#define WSG_CLOSE_NON_UTF8 1007        /* CloseFrame.NON_UTF8 */
#define WSG_CLOSE_TOO_BIG 1009         /* CloseFrame.TOO_BIG */

/* RFC 6455 opcodes (Opcode.java:33-98). */
#define WSG_OP_CONTINUATION 0
#define WSG_OP_TEXT 1
#define WSG_OP_BINARY 2
#define WSG_OP_CLOSE 8
#define WSG_OP_PING 9
#define WSG_OP_PONG 10

/* Decoder configuration: the FrameDecoder constructor arguments
 * (FrameDecoder.java:76) plus whether the "ws-utf8-validator" stage
 * (FrameUtf8Validator) is fused into the decode pass. */
typedef struct wsg_decoder_cfg {
    int32_t client_mode;       /* FrameDecoder.clientMode: 1 = expect unmasked frames */
    int32_t allow_extensions;  /* FrameDecoder.allowExtensions: RSV bits allowed */
    int64_t max_payload_len;   /* FrameDecoder.maxPayloadLen */
    int32_t validate_utf8;     /* 1 = FrameUtf8Validator runs after the decoder */
    int32_t flags;             /* WSG_CFG_* */
} wsg_decoder_cfg;
/* wsg_decoder_cfg.flags: frames need not be adjacent in `wire` (frame k's extent is its
 * header's, frame_off[k + 1] is not its end; frames must not overlap and must lie in
 * wire[0, wire_len)): the native batcher lands each session's reads where they fall. */
#define WSG_CFG_SPARSE 1

/* Per-session carry state, passed explicitly in and out of every batch.
 * It is the part of FrameDecoder / FrameUtf8Validator state that survives a
 * complete frame (FrameDecoder.java:49,63; FrameUtf8Validator.java:42):
 *   fragmentation : FrameDecoder.fragmentation
 *   text_open     : FrameUtf8Validator.context != null (inside a text message)
 *   closed        : FrameDecoder.closed (all further input is swallowed)
 *   tail[0..tail_len) : the last (<=3) payload bytes of the open text message,
 *                   which determine the UTF-8 DFA state carried across fragments.
 * Partial frames never enter a batch: the host buffers them (FrameDecoder.java:276-283). */
typedef struct wsg_session_state {
    uint8_t fragmentation;
    uint8_t text_open;
    uint8_t closed;
    uint8_t tail_len;
    uint8_t tail[3];
    uint8_t reserved;
} wsg_session_state; /* 8 bytes */

/* One decoded frame (the device-side form of Frame, Frame.java:33-143). */
typedef struct wsg_frame_desc {
    uint64_t payload_off;  /* byte offset of the unmasked payload in payload_out (16-B aligned) */
    uint32_t payload_len;  /* payload length */
    uint8_t opcode;        /* Opcode value */
    uint8_t flags;         /* bit7 = FIN, bits4..6 = RSV (Frame.getRsvBits()<<4), bit0 = was masked */
    uint16_t status;       /* wsg_status of this frame (meaningful up to the session's first error) */
} wsg_frame_desc; /* 16 bytes */

/* Per-session outcome of one batch. Frames [first, first+n_delivered) of the
 * session are delivered to the handler in order; if error != 0, frame
 * first+n_delivered failed with that error, the session wrote
 * CloseFrame(close_code) and latched closed (FrameDecoder.java:92-102). */
typedef struct wsg_session_result {
    uint32_t n_delivered;
    uint16_t error;       /* wsg_status */
    uint16_t close_code;  /* 1002, 1007, or 0 */
    int64_t detail;       /* numeric argument of the exception message */
} wsg_session_result; /* 16 bytes */

/* One frame to encode (FrameEncoder.encode input: a Frame + its mask key). */
typedef struct wsg_encode_frame {
    uint64_t payload_off;  /* offset of the (unmasked) payload in the payload buffer */
    uint32_t payload_len;
    uint8_t opcode;
    uint8_t flags;         /* bit7 = FIN, bits4..6 = RSV */
    uint8_t reserved[2];
    uint8_t mask[4];       /* mask key (client mode); the reference draws it from
                              java.util.Random (FrameEncoder.java:43,111) — here it is injected */
    uint32_t reserved2;
} wsg_encode_frame; /* 24 bytes */

typedef struct wsg_ctx wsg_ctx;

/* ---------------- context ---------------- */
int wsg_version(void);
/* Open a context on HIP device `device`. `stream` is a hipStream_t (NULL = the
 * context creates its own non-blocking stream, which is NOT ordered with the
 * null stream: to run on the null stream, call wsg_set_stream(ctx, NULL)). */
int wsg_open(int device, void* stream, wsg_ctx** out);
int wsg_close(wsg_ctx* ctx);
/* Measurement and test switches of a context (the defaults are the product; each
 * alternative is kept to A/B the choice it documents in DESIGN.md):
 *   WSG_TUNE_INFLATE_TOKENS  0: no lane pre-decode, the serial inflate decodes every frame
 *   WSG_TUNE_INFLATE_FAST    0: no parallel token replay; 2 (tests only): the replay alone,
 *                            sessions it does not take are left unprocessed
 *   WSG_TUNE_INFLATE_LDS     0: the lane pre-decode keeps its tables in HBM
 *   WSG_TUNE_INFLATE_ORDER   0: lanes take frames in batch order (not longest first)
 *   WSG_TUNE_INFLATE_LANES   k_infl_tok lanes at most (multiple of 64)
 *   WSG_TUNE_INFLATE_SPLIT   the split-lane decode (two lanes a message): 0 never (default), 1 when a
 *                            lane a frame would leave half the chip's resident lanes idle, 2 always
 *   WSG_TUNE_INFLATE_TABS    HBM table blocks (3,880 B each) for the lanes whose message needs the
 *                            HBM-table decoder (default 32768; beyond, such messages take the
 *                            serial decoder)
 *   WSG_TUNE_FUSED_SCAN      0: always launch k_scan (k_link does not fold block aggregates)
 *   WSG_TUNE_AGG_UNITS       aggregator gather units per wave: 1, 2 (default) or 4
 *   WSG_TUNE_AGG_GRID        aggregator gather waves at most (default 65536)
 *   WSG_TUNE_DEFLATE_SERIAL  1: permessage-deflate compression runs zlib's loop one lane a session at
 *                            every level (the parallel form for levels 4-9 is the default; tests)
 *   WSG_TUNE_AGG_FOLD_MAX    aggregator plans of up to this many 512-frame blocks fold the block
 *                            sums in k_agg_b / k_agg_c (default: as many as LDS allows, 3,072);
 *                            larger ones run k_agg_scan (0 forces it: the tests' way to reach it)
 *   WSG_TUNE_STAGE_FAIL      n > 0: the n-th stage-chain step a batcher on this context begins from now
 *                            fails as a device error would (tests of the error path)
 *   WSG_TUNE_DEFLATE_LDS     0: the deflate match search walks every chain in global memory (the
 *                            LDS-resident walk of a session's window is the default; tests, A/B) */
enum {
    WSG_TUNE_INFLATE_TOKENS = 1,
    WSG_TUNE_INFLATE_FAST = 2,
    WSG_TUNE_INFLATE_LDS = 3,
    WSG_TUNE_INFLATE_ORDER = 4,
    WSG_TUNE_INFLATE_LANES = 5,
    WSG_TUNE_FUSED_SCAN = 6,
    WSG_TUNE_AGG_UNITS = 7,
    WSG_TUNE_AGG_GRID = 8,
    WSG_TUNE_INFLATE_TABS = 9,
    WSG_TUNE_INFLATE_SPLIT = 10,
    WSG_TUNE_AGG_FOLD_MAX = 11,
    WSG_TUNE_DEFLATE_SERIAL = 12,
    WSG_TUNE_STAGE_FAIL = 13,
    WSG_TUNE_DEFLATE_LDS = 14
};
int wsg_set_tuning(wsg_ctx* ctx, int key, int64_t value);
/* Use `stream` for all later work (NULL = the null stream); a private stream is synchronised and destroyed. */
int wsg_set_stream(wsg_ctx* ctx, void* stream);
/* The hipStream_t the context enqueues its kernels on (for a caller that orders its
 * own copies or kernels with the codec's). */
int wsg_get_stream(wsg_ctx* ctx, void** stream);
const char* wsg_last_error(wsg_ctx* ctx);
/* Pre-size device workspace so later batch calls do no allocation (graph-capture safe). */
int wsg_reserve(wsg_ctx* ctx, uint64_t max_frames, uint32_t max_sessions, uint64_t max_wire_len);
/* The same for permessage-deflate batches (wsg_inflate_batch_*): frames, sessions and
 * compressed payload bytes of the largest batch.  Kept apart from wsg_reserve because
 * the inflate workspace is ~7 B per compressed byte (token and literal regions). */
int wsg_reserve_inflate(wsg_ctx* ctx, uint64_t max_frames, uint32_t max_sessions, uint64_t max_payload_len);

/* Messages the split-lane decode (WSG_TUNE_INFLATE_SPLIT) has decoded on this context since
 * it was created: a lane pair joined the head's and the tail's halves of each.  Waits for
 * the context's stream.  (A measurement and test hook; no reference counterpart.) */
int wsg_inflate_split_count(wsg_ctx* ctx, uint64_t* count);
int wsg_sync(wsg_ctx* ctx);

/* Kernel timing (hipEvents recorded around each kernel on the ctx stream).
 * enable: 0 off, 1 every kernel, 2 only the streaming kernels (k_piecesN,
 * k_enc_piecesN, k_agg_gather) — each event pair adds queue time, so a timed step uses 2. */
int wsg_set_timing(wsg_ctx* ctx, int enable);
/* Mode 2 brackets one launch in `every` of each streaming kernel (default 1): an
 * event pair costs ~12 us of queue time (tools/ubench_graph.hip), so a timed region
 * samples the kernel's duration instead of paying that on every step. */
int wsg_set_timing_every(wsg_ctx* ctx, uint32_t every);
/* out_ms[i] = accumulated milliseconds of kernel i since the last reset, out_count[i] = launches.
 * Kernel ids: see wsg_kernel_name(). Syncs the stream. */
int wsg_get_timing(wsg_ctx* ctx, double* out_ms, uint64_t* out_count, int max_kernels);
int wsg_reset_timing(wsg_ctx* ctx);
const char* wsg_kernel_name(int kernel_id);
int wsg_num_kernels(void);

/* ---------------- decode (FrameDecoder [+ FrameUtf8Validator]) ---------------- */
/* Upper bound of payload_out bytes for a batch. */
uint64_t wsg_decode_payload_bound(uint64_t wire_len, uint64_t n_frames);

/* Device-resident batch decode; every pointer is a device pointer; the work is
 * enqueued on the ctx stream and the call returns without synchronising.
 *   wire[0..wire_len)            concatenated wire bytes of all sessions
 *   frame_off[0..n_frames]       frame k occupies wire[frame_off[k], frame_off[k+1]),
 *                                ascending; each entry is what FrameDecoder.available()
 *                                returned for a complete frame (FrameDecoder.java:357-401)
 *   session_first[0..n_sessions] session s owns frames [session_first[s], session_first[s+1])
 *   state[n_sessions]            carry state in / out
 *   payload_out                  unmasked payloads, 16-B aligned slot per frame
 *   desc_out[n_frames], result_out[n_sessions]
 * Equivalent to calling FrameDecoder.decode (FrameDecoder.java:180-288) once per
 * frame per session, followed by FrameUtf8Validator.decode (FrameUtf8Validator.java:59-98). */
int wsg_decode_batch_device(wsg_ctx* ctx, const wsg_decoder_cfg* cfg,
                            const uint8_t* wire, uint64_t wire_len,
                            const uint64_t* frame_off, uint64_t n_frames,
                            const uint32_t* session_first, uint32_t n_sessions,
                            wsg_session_state* state,
                            uint8_t* payload_out, uint64_t payload_cap,
                            wsg_frame_desc* desc_out, wsg_session_result* result_out);

/* Same contract with host pointers (pinned or pageable): H2D, decode, D2H,
 * synchronise. This is the end-to-end (PCIe-inclusive) path of the JNI shim. */
int wsg_decode_batch_host(wsg_ctx* ctx, const wsg_decoder_cfg* cfg,
                          const uint8_t* wire, uint64_t wire_len,
                          const uint64_t* frame_off, uint64_t n_frames,
                          const uint32_t* session_first, uint32_t n_sessions,
                          wsg_session_state* state,
                          uint8_t* payload_out, uint64_t payload_cap,
                          wsg_frame_desc* desc_out, wsg_session_result* result_out);

/* Pipelined form for a continuous flow of host batches: enqueues the uploads on
 * the context's copy-in stream, the kernels on its stream and the downloads on
 * its copy-out stream, through one of two device staging slots, and returns.
 * Successive calls overlap: batch i's download runs beside batch i+1's upload
 * (PCIe is full duplex; each direction needs its own stream).  A batch whose
 * slot is still busy waits (host side) for that slot's previous batch.
 * Host buffers must stay valid (and should be pinned, or the copies serialise)
 * until wsg_sync(ctx).  The carry state of batch i+1 is uploaded only after
 * batch i's state came back, so successive batches may share sessions and one
 * host state array.  payload_cap >= wire_len + 16 * n_frames: the whole payload
 * region is copied back, its used size being known only on the device.
 * payload_out == NULL: the payloads stay on the device (descriptors, results and
 * state are still downloaded); the native batcher's stages read them there. */
int wsg_decode_batch_host_async(wsg_ctx* ctx, const wsg_decoder_cfg* cfg,
                                const uint8_t* wire, uint64_t wire_len,
                                const uint64_t* frame_off, uint64_t n_frames,
                                const uint32_t* session_first, uint32_t n_sessions,
                                wsg_session_state* state,
                                uint8_t* payload_out, uint64_t payload_cap,
                                wsg_frame_desc* desc_out, wsg_session_result* result_out);

/* FrameUtf8Validator alone — the "ws-utf8-validator" stage (FrameUtf8Validator.java:59-98)
 * over frames whose payloads are already plain, for sessions where the fused
 * validation cannot run (permessage-deflate: validation follows inflate,
 * PerMessageDeflateExtension.java:316-326).  Every pointer is a device pointer.
 *   desc[n_frames]                frame k: opcode, flags (FIN/RSV), payload at
 *                                 payload[payload_off, +payload_len); ranges disjoint
 *   session_first[0..n_sessions]  session s owns frames [session_first[s], session_first[s+1])
 *   state[n_sessions]             carry in / out (text_open, tail; closed latches on failure)
 *   result_out[n_sessions]        n_delivered = frames that passed; error WSG_E_TEXT_UTF8 (1007)
 * A decode batch for such sessions runs with validate_utf8 = 0. */
int wsg_validate_batch_device(wsg_ctx* ctx, const wsg_frame_desc* desc, uint64_t n_frames,
                              const uint32_t* session_first, uint32_t n_sessions,
                              const uint8_t* payload, uint64_t payload_len,
                              wsg_session_state* state, wsg_session_result* result_out);
/* Same contract with host pointers: H2D, validate, D2H, synchronise. */
int wsg_validate_batch_host(wsg_ctx* ctx, const wsg_frame_desc* desc, uint64_t n_frames,
                            const uint32_t* session_first, uint32_t n_sessions,
                            const uint8_t* payload, uint64_t payload_len,
                            wsg_session_state* state, wsg_session_result* result_out);

/* FrameDecoder.available(ISession, byte[], off, len) for a decoder with no
 * pending partial payload (FrameDecoder.java:357-401): returns 0 if the header
 * is incomplete, the full frame length if available, otherwise len.  On the
 * u64-length errors it returns -1 and sets *err (WSG_E_NEG_LEN / WSG_E_EXT_LEN)
 * and *detail / *detail2.  Host-only, no device work. */
int64_t wsg_frame_available(const uint8_t* buf, uint64_t len, int32_t* err,
                            int64_t* detail, int64_t* detail2);

/* Header-rule check of one (possibly partial) frame whose header is complete:
 * applies FrameDecoder.decode's rules that need only the header
 * (FrameDecoder.java:197-256) given the fragmentation flag. Returns wsg_status,
 * sets *detail.  Used by the host to fail early on partial frames, as the
 * reference does, before the payload is complete. Host-only. */
int32_t wsg_check_header(const wsg_decoder_cfg* cfg, int fragmentation,
                         const uint8_t* buf, uint64_t len, int64_t* detail);

/* ---------------- encode (FrameEncoder) ---------------- */
/* Exact wire length of a frame (FrameEncoder.length(), FrameEncoder.java:122-135). */
uint64_t wsg_encoded_length(uint32_t payload_len, int client_mode);

/* Device-resident batch encode (FrameEncoder.encode, FrameEncoder.java:69-120).
 *   payload[...]                 unmasked payload bytes, frames reference them by offset
 *   frames[n_frames]             frames in session order
 *   session_first[0..n_sessions] session s owns frames [session_first[s], session_first[s+1])
 *   closed[n_sessions]           FrameEncoder.closed carry in / out (a CLOSE frame latches it
 *                                and every later frame of the session is dropped, :71-76)
 *   wire_out                     concatenated wire bytes (no padding between frames)
 *   wire_off[0..n_frames]        frame k occupies wire_out[wire_off[k], wire_off[k+1]);
 *                                a dropped frame has an empty range
 *   client_mode                  1 = mask with frames[k].mask (clientMode)  */
int wsg_encode_batch_device(wsg_ctx* ctx, int client_mode,
                            const uint8_t* payload, uint64_t payload_len,
                            const wsg_encode_frame* frames, uint64_t n_frames,
                            const uint32_t* session_first, uint32_t n_sessions,
                            uint8_t* closed,
                            uint8_t* wire_out, uint64_t wire_cap, uint64_t* wire_off);

int wsg_encode_batch_host(wsg_ctx* ctx, int client_mode,
                          const uint8_t* payload, uint64_t payload_len,
                          const wsg_encode_frame* frames, uint64_t n_frames,
                          const uint32_t* session_first, uint32_t n_sessions,
                          uint8_t* closed,
                          uint8_t* wire_out, uint64_t wire_cap, uint64_t* wire_off);

/* ---------------- host boundary: cross-session batcher + pinned pool ---------------- */
/* The native core of the JNI shim: every session's socket bytes
 * go in (wsg_batcher_feed, on the loop threads' behalf), frames are delimited on
 * the host exactly as the session read loop does (FrameDecoder.available,
 * FrameDecoder.java:357-401; StreamSession.java:798-854) with the header rules
 * applied as soon as a header is complete (FrameDecoder.java:197-256), and
 * wsg_batcher_flush decodes every complete frame of every session in one device
 * batch.  Partial frames stay in the batcher.  One thread drives a batcher (a
 * selector loop's: the sessions of one loop share it); wsg_batcher_feed_many spreads
 * the sessions of its reads over worker threads itself. */
typedef struct wsg_batcher wsg_batcher;

typedef struct wsg_batch_view {  /* valid until the next flush / close */
    uint64_t n_frames;
    uint64_t wire_bytes;
    uint32_t n_sessions;
    uint32_t reserved;
    const uint32_t* session_first;      /* [n_sessions + 1] */
    const wsg_frame_desc* desc;         /* [n_frames] */
    const uint8_t* payload;             /* unmasked payloads (desc.payload_off) */
    const wsg_session_result* result;   /* [n_sessions]: frames delivered + the first error,
                                           device-found or a header error found on the host */
    const int64_t* detail2;             /* [n_sessions]: the message's second argument, for
                                           WSG_E_EXT_LEN (Integer.MAX_VALUE - the header's length,
                                           FrameDecoder.java:393); 0 otherwise */
} wsg_batch_view;

int wsg_batcher_open(wsg_ctx* ctx, const wsg_decoder_cfg* cfg, uint32_t n_sessions, wsg_batcher** out);
int wsg_batcher_close(wsg_batcher* b);
const char* wsg_batcher_last_error(wsg_batcher* b);
/* Append bytes read from session `sid`'s socket (copied into the open batch's pinned
 * arena, after the session's carried partial frame; the caller may reuse `data`, as
 * the reference releases its buffer after decode, FrameDecoder.java:285-287). */
int wsg_batcher_feed(wsg_batcher* b, uint32_t sid, const uint8_t* data, uint64_t len);
/* Decode all complete frames fed since the last flush; synchronises. */
int wsg_batcher_flush(wsg_batcher* b, wsg_batch_view* out);
/* Many socket reads at once (e.g. one selector-loop iteration's): reads of one
 * session in order; the sessions are fed by up to 16 threads (sid mod T). */
int wsg_batcher_feed_many(wsg_batcher* b, uint32_t n, const uint32_t* sids, const uint8_t* const* data,
                          const uint64_t* lens);
/* The pipelined flush: flush_async gathers every complete frame into pinned
 * staging and queues H2D, decode and D2H (wsg_decode_batch_host_async) without
 * waiting, so the next feeds and the next gather overlap the device and PCIe
 * work; wsg_batcher_wait returns the oldest queued flush's results (a view valid
 * until that slot is flushed again, WSG_BATCHER_MAX_INFLIGHT flushes later).  At
 * most WSG_BATCHER_MAX_INFLIGHT flushes in flight (WSG_API_ERANGE beyond); the
 * carry state chains through them on the device side, and host changes (a slot
 * reset, a header error found on the host) apply to the next batch queued.  With
 * stages, a flush's chain starts once its decode is done (flush_async starts those
 * of the flushes queued before it; wsg_batcher_wait collects the oldest flush's chain
 * and advances the chains behind it: inflate + validator launched, the output gather
 * of the next one queued), so they run while the caller feeds: keeping four in
 * flight gives the chain three flushes of lead (4 since round 5: the steady-state
 * stage line 22.9 -> 26.0 GiB/s against 3).
 * wsg_batcher_flush = wait for the queued ones (results dropped) + flush_async + wait. */
#define WSG_BATCHER_MAX_INFLIGHT 4
int wsg_batcher_flush_async(wsg_batcher* b);
int wsg_batcher_wait(wsg_batcher* b, wsg_batch_view* out);
int wsg_batcher_session_state(wsg_batcher* b, uint32_t sid, wsg_session_state* st);
/* Completion across threads (the selector loop must not block on the device):
 * flush_async queues flush number t = 1, 2, ...; wsg_batcher_ticket returns the last
 * queued ticket.  wsg_batcher_await blocks until a flush with a ticket > `seen` has
 * finished its device work (downloads done; a host function on the download stream
 * signals it) or `timeout_ms` passes (0: do not block, < 0: no limit), and returns the
 * highest finished ticket.  It is the one batcher call that may run on another thread
 * than the one driving the batcher (stop that thread before wsg_batcher_close): a
 * completion thread awaits a flush, then re-enters the selector loop
 * (SelectorLoop.executenf, InternalSelectorLoop.java:990-1011), whose task collects
 * it with wsg_batcher_wait without waiting.  With stages (wsg_batcher_set_stages) the
 * ticket marks the decode; wsg_batcher_wait then runs the stage chain on the calling
 * thread (a stage thread that ran it as soon as the decode was done measured 8-20%
 * slower on the stage lines: DESIGN.md §8c).  Replaces nothing in the reference (its
 * decode is synchronous on the loop thread). */
uint64_t wsg_batcher_ticket(wsg_batcher* b);
int64_t wsg_batcher_await(wsg_batcher* b, uint64_t seen, int64_t timeout_ms);
/* Size every pinned and device buffer of the three flush slots for flushes of up to
 * `max_wire` bytes and `max_frames` frames, so those flushes allocate nothing (with
 * stages, wsg_batcher_reserve_stages sizes theirs).  wsg_batcher_alloc_count is the
 * number of pinned/device allocations all batchers and contexts of the process have
 * made (batcher buffers and device workspaces).
 * Precondition: no flush in flight (it moves the slots' buffers, which a queued flush
 * still reads and writes): WSG_API_ERANGE otherwise, nothing changed. */
int wsg_batcher_reserve(wsg_batcher* b, uint64_t max_wire, uint64_t max_frames);
uint64_t wsg_batcher_alloc_count(void);
/* With stages (call after wsg_batcher_set_stages and wsg_batcher_reserve): every stage
 * buffer sized for flushes within the reserved wire/frame sizes whose stages deliver up
 * to `max_out_bytes` bytes in up to `max_out_frames` frames (inflated or aggregated
 * messages): the stage arena, the pinned output and its copy list, the stage lists
 * uploaded and downloaded, the stage context's workspace.  Such flushes allocate
 * nothing.  A flush beyond grows what it needs.  WSG_API_ERANGE with a flush in
 * flight, WSG_API_EINVAL before set_stages.  Replaces nothing in the reference (its
 * buffers come from the session allocator, IByteBufferAllocator.java:47-73). */
int wsg_batcher_reserve_stages(wsg_batcher* b, uint64_t max_out_bytes, uint64_t max_out_frames);
/* The decoders after "ws-decoder" that a flush runs in the same device batch, in the
 * pipeline order the reference builds (DefaultWebSocketSessionConfig.java:276-281,
 * PerMessageDeflateExtension.java:316-326; a FrameAggregator the application puts
 * after them):
 *   ws-decoder -> [inflate: PerMessageDeflateDecoder(noContext)] ->
 *   [validate: FrameUtf8Validator] -> [aggregate: FrameAggregator(max)]
 * With inflate on, the decode runs with the fused UTF-8 check off and `validate`
 * is the ws-utf8-validator stage after inflate (wsg_validate_batch_*); without
 * inflate, `validate` is the fused check (cfg.validate_utf8).  Every stage sees
 * the frames the stage before it delivered, per session in order, and keeps its
 * own carry between flushes: the inflater state and 32 KiB window, the frames of
 * a compressed message a batch leaves open (re-sent with the next batch), the
 * validator context, the aggregated message in progress and its bytes.  A
 * session's result is that of the LAST stage that failed it (its failure is the
 * earliest in the stream), n_delivered counts the flush's output frames, and any
 * failure latches the session closed.  Output frames: desc.flags bit 0x02
 * (WSG_OUT_AGGREGATED) marks an aggregated message (AggregatedTextFrame /
 * AggregatedBinaryFrame, FrameAggregator.java:76-99); payloads are in the view's
 * payload region.  Call before the first feed. */
typedef struct wsg_stage_cfg {
    uint8_t inflate;             /* PerMessageDeflateDecoder after the decoder */
    uint8_t inflate_no_context;  /* its noContext (PerMessageDeflateDecoder.java:52-56) */
    uint8_t validate;            /* FrameUtf8Validator (ws-utf8-validator) */
    uint8_t aggregate;           /* FrameAggregator */
    uint32_t reserved;
    int64_t max_aggregated_len;  /* FrameAggregator(maxAggregatedLength) */
} wsg_stage_cfg;
#define WSG_OUT_AGGREGATED 0x02
int wsg_batcher_set_stages(wsg_batcher* b, const wsg_stage_cfg* stages);
/* The context the stages run on (the batcher's own, opened by wsg_batcher_set_stages on the
 * batcher context's device, with that context's wsg_set_tuning switches), or NULL before
 * set_stages: for wsg_inflate_split_count and the like.  Owned by the batcher. */
wsg_ctx* wsg_batcher_stage_context(wsg_batcher* b);
/* Give slot `sid` to a new session: drops the pending partial frame and any bytes
 * fed since the last flush, and zeroes the carry (fragmentation, UTF-8 context,
 * closed latch), as a freshly constructed FrameDecoder + FrameUtf8Validator
 * (FrameDecoder.java:43-63, FrameUtf8Validator.java:42).  The JNI shim calls it
 * from the decoder's session-end hook (IEventDrivenCodec.event ENDING /
 * removed, IEventDrivenCodec.java:36-62). */
int wsg_batcher_session_reset(wsg_batcher* b, uint32_t sid);

/* ---------------- host boundary: cross-session encode batcher ---------------- */
/* FrameEncoder.encode (FrameEncoder.java:69-120) for all sessions of a selector
 * loop, one device batch per flush (the encode side of the loop batching, as
 * EncodeTask.java:333-407 hands each write to the session's encoder chain).
 * add() copies a frame's payload into a pinned arena and queues it; flush() orders
 * the queued frames by session (each session's in arrival order) and encodes them
 * in one device batch; the close latch (:71-76) persists per session.
 * Not thread-safe: one loop thread drives it. */
typedef struct wsg_enc_batcher wsg_enc_batcher;

typedef struct wsg_enc_view {  /* valid until the next add / flush / close */
    uint64_t n_frames;
    uint64_t wire_bytes;
    uint32_t n_sessions;
    uint32_t reserved;
    const uint32_t* session_first;  /* [n_sessions + 1]: session s's frames [sf[s], sf[s+1]) */
    const uint64_t* wire_off;       /* [n_frames + 1]: frame k's wire bytes [off[k], off[k+1]),
                                       empty for a frame dropped after the session's CLOSE */
    const uint8_t* wire;            /* session s's frames are contiguous: [off[sf[s]], off[sf[s+1]]) */
} wsg_enc_view;

int wsg_enc_batcher_open(wsg_ctx* ctx, int client_mode, uint32_t n_sessions, wsg_enc_batcher** out);
int wsg_enc_batcher_close(wsg_enc_batcher* b);
const char* wsg_enc_batcher_last_error(wsg_enc_batcher* b);
/* Queue Frame(opcode, flags = FIN << 7 | RSV << 4, payload) of session `sid`;
 * `mask` (client mode) is the 4-byte key, FrameEncoder.java:109-118. */
int wsg_enc_batcher_add(wsg_enc_batcher* b, uint32_t sid, uint8_t opcode, uint8_t flags, const uint8_t* mask,
                        const uint8_t* payload, uint32_t len);
/* Many frames in one call (a loop iteration's writes), as n add() calls in order;
 * masks: 4 bytes a frame (client mode) or NULL. */
int wsg_enc_batcher_add_many(wsg_enc_batcher* b, uint32_t n, const uint32_t* sids, const uint8_t* opcodes,
                             const uint8_t* flags, const uint8_t* masks, const uint8_t* const* payloads,
                             const uint32_t* lens);
int wsg_enc_batcher_flush(wsg_enc_batcher* b, wsg_enc_view* out);
/* Pipelined form: flush_async queues the encode of everything added so far (H2D on
 * the batcher's upload stream, kernels on the context's stream, D2H on its download
 * stream) and returns; add() then fills the next of three slots.  wait() returns the
 * oldest flush's view (valid until that slot is flushed again).  At most two in
 * flight.  A session reset while its frames are in flight drops them from the view. */
int wsg_enc_batcher_flush_async(wsg_enc_batcher* b);
int wsg_enc_batcher_wait(wsg_enc_batcher* b, wsg_enc_view* out);
/* slot `sid` for a new session: its queued frames are dropped, the close latch cleared
 * (and, with deflate on, a new deflater) */
int wsg_enc_batcher_session_reset(wsg_enc_batcher* b, uint32_t sid);
/* The "permessage-deflate-encoder" stage in front of the encoder for every session of the
 * batcher: PerMessageDeflateEncoder(level, noContext) as PerMessageDeflateExtension.
 * updateEncoders installs it (PerMessageDeflateExtension.java:303-313).  Each flush then
 * compresses its frames on the device first — wsg_deflate_batch_device's rules and bytes
 * (byte-identical to java.util.zip.Deflater), the deflater state and its window | head | prev
 * kept per session on the device (WSG_DEFLATE_SESSION_BYTES each: n_sessions x 192 KiB of
 * HBM) — and frames what it hands on, still without a host synchronisation (the workspace is
 * sized from the frames' lengths).  Once, before the first add; level 0-9. */
int wsg_enc_batcher_set_deflate(wsg_enc_batcher* b, int level, int no_context);
/* as wsg_batcher_ticket / _await / _reserve, for the encode batcher (max_payload:
 * payload bytes a flush may hold; reserve: WSG_API_ERANGE with a flush in flight) */
uint64_t wsg_enc_batcher_ticket(wsg_enc_batcher* b);
int64_t wsg_enc_batcher_await(wsg_enc_batcher* b, uint64_t seen, int64_t timeout_ms);
int wsg_enc_batcher_reserve(wsg_enc_batcher* b, uint64_t max_frames, uint64_t max_payload);

/* ---------------- device per selector loop (multi-GPU policy) ---------------- */
/* Sessions shard over the node's GPUs by selector loop, with no cross-device
 * exchange (a session belongs to one loop, DefaultWebSocketSessionConfig.java:
 * 276-281, one decoder per session): the JNI shim opens each loop's batcher on
 * wsg_device_for_loop(loop id).  A new loop goes to the device with the fewest
 * loops, ties to the one with the fewest wire bytes accounted (wsg_device_account
 * after each flush); a loop keeps its device until released.  Process-wide,
 * thread-safe.  wsg_device_policy_init fixes the device count (else the HIP count). */
int wsg_device_policy_init(int n_devices);
int wsg_device_for_loop(uint64_t loop_id);                 /* device index, or < 0 */
int wsg_device_account(int device, uint64_t wire_bytes);
int wsg_device_release_loop(uint64_t loop_id);

/* Pinned host buffers for socket reads (the role of IByteBufferAllocator,
 * IByteBufferAllocator.java:38-149): power-of-two size classes, recycled on
 * release, thread-safe.  wsg_host_alloc returns NULL on failure. */
void* wsg_host_alloc(uint64_t capacity);
int wsg_host_release(void* p);
uint64_t wsg_host_capacity(const void* p);  /* 0 if p is not from the pool */
int wsg_host_trim(void);                    /* frees the pool's idle buffers */

/* ---------------- aggregate (FrameAggregator) ---------------- */
/* Per-session carry of FrameAggregator.frame (FrameAggregator.java:44): the
 * aggregated frame in progress.  Its bytes from earlier batches stay with the
 * caller, as PayloadAggregator keeps its fragment list (PayloadAggregator.java:34). */
typedef struct wsg_agg_state {
    uint8_t open;      /* an aggregated frame is in progress (frame != null) */
    uint8_t opcode;    /* its opcode: TEXT or BINARY */
    uint8_t rsv;       /* its RSV bits (Frame.getRsvBits) */
    uint8_t reserved;
    uint32_t length;   /* IAggregatedFrame.getPayloadLength(): its bytes so far */
} wsg_agg_state; /* 8 bytes */

/* wsg_frame_desc.flags bits of aggregator output (besides FIN / RSV) */
#define WSG_AGG_IN_AGG 0x02    /* payload in agg_out (else the frame's own slot in the decoder's payload) */
#define WSG_AGG_PREFIXED 0x04  /* the message began in an earlier batch: its bytes from earlier
                                  batches (held by the caller) come first */
#define WSG_AGG_PENDING 0x08   /* not a frame: this batch's bytes of a message still open at the
                                  end of the batch, for the caller to hold (replacing what it held
                                  unless also PREFIXED) */

/* Device-resident FrameAggregator over a decoded batch (FrameAggregator.decode,
 * FrameAggregator.java:72-104, applied to each delivered frame of each session in
 * order).  Inputs are the decoder's outputs for the batch:
 *   desc[n_frames], payload       wsg_decode_batch_* desc_out / payload_out (payload_len = its
 *                                 size in bytes, e.g. the decoder's payload_cap)
 *   session_first[0..n_sessions]  as for the decode
 *   dec_result[n_sessions]        only the first n_delivered frames of a session are aggregated
 *   state[n_sessions]             carry in / out
 * Outputs:
 *   agg_out[agg_cap]              the bytes of every fragmented message, back to back in frame
 *                                 order (agg_cap >= the batch's total payload bytes)
 *   out_desc[n_frames+n_sessions] session s's output frames at out_desc[session_first[s] + s + i],
 *                                 i < out_result[s].n_delivered: pass-through frames reference
 *                                 `payload`, aggregated ones agg_out (WSG_AGG_IN_AGG); then, if the
 *                                 session ends the batch inside a message, one WSG_AGG_PENDING entry
 *   out_result[n_sessions]        error WSG_E_AGG_TOO_BIG (close 1009) with detail = the index of the
 *                                 failing input frame within the session; nothing after it is output
 *   agg_total (device, 1 x u64)   bytes written to agg_out */
int wsg_aggregate_batch_device(wsg_ctx* ctx, int64_t max_aggregated_len,
                               const wsg_frame_desc* desc, uint64_t n_frames,
                               const uint32_t* session_first, uint32_t n_sessions,
                               const wsg_session_result* dec_result,
                               const uint8_t* payload, uint64_t payload_len,
                               wsg_agg_state* state, uint8_t* agg_out, uint64_t agg_cap,
                               wsg_frame_desc* out_desc, wsg_session_result* out_result,
                               uint64_t* agg_total);

/* Same contract with host pointers: H2D, aggregate, D2H of the used agg_out
 * bytes, descriptors, results and state; synchronises.  *agg_total is a host
 * pointer here. */
int wsg_aggregate_batch_host(wsg_ctx* ctx, int64_t max_aggregated_len,
                             const wsg_frame_desc* desc, uint64_t n_frames,
                             const uint32_t* session_first, uint32_t n_sessions,
                             const wsg_session_result* dec_result,
                             const uint8_t* payload, uint64_t payload_len,
                             wsg_agg_state* state, uint8_t* agg_out, uint64_t agg_cap,
                             wsg_frame_desc* out_desc, wsg_session_result* out_result,
                             uint64_t* agg_total);

/* ---------------- permessage-deflate decode (PerMessageDeflateDecoder) ---------------- */
/* Per-session carry of PerMessageDeflateDecoder / DeflateDecoder / its raw ZlibDecoder
 * (PerMessageDeflateDecoder.java:41, DeflateDecoder.java:47-58, ZlibDecoder.java:54-58). */
typedef struct wsg_inflate_state {
    uint8_t compressing;   /* PerMessageDeflateDecoder.compressing */
    uint8_t has_decoder;   /* DeflateDecoder.decoder != null (an inflater exists) */
    uint8_t finished;      /* its ZlibDecoder.finished: a final block ended the stream, later data
                              passes through unchanged */
    uint8_t reserved;
    uint16_t window_len;   /* bytes of inflate history in window[s] (<= 32768) */
    uint16_t window_phase; /* window[s] is a ring image: the history byte at stream position q
                              sits at window[s][(q + window_phase) & 32767], the next position
                              being q = 0 (opaque to the caller; zero for a new session) */
} wsg_inflate_state; /* 8 bytes */

#define WSG_INFLATE_WINDOW 32768
#define WSG_DESC_REPLAY 0x02   /* input desc.flags: a frame of a message left open by the previous
                                  batch, decoded again (from the message start) but not delivered */
#define WSG_DESC_INFLATED 0x02 /* output desc.flags: payload in `out` (else the input payload) */

/* Device-resident PerMessageDeflateDecoder over decoded frames (its decode() once per
 * frame per session in order, PerMessageDeflateDecoder.java:68-105 + DeflateDecoder.java:
 * 78-141): frames of TEXT/BINARY with RSV1, and continuations of such a message, are
 * inflated (raw DEFLATE, RFC 1951; the 4-byte tail 00 00 FF FF appended after a final
 * fragment), RSV1 is cleared; other frames pass through.  One workgroup per session.
 *   desc[n_frames], payload[payload_len]   the decoder's frames (desc.flags WSG_DESC_REPLAY
 *                                 marks frames re-sent for a message the previous batch left open)
 *   session_first[0..n_sessions]  session s owns frames [session_first[s], session_first[s+1])
 *   state[n_sessions], window[n_sessions * 32768]   carry in / out
 *   out, out_off[n_sessions + 1]  session s writes its inflated bytes to out[out_off[s], out_off[s+1])
 *   out_desc[n_frames]            per non-replay frame: inflated (WSG_DESC_INFLATED, offset in out)
 *                                 or passed through (offset in payload)
 *   out_result[n_sessions]        n_delivered = non-replay frames before the first error
 *   replay_from[n_sessions]       if the batch ends inside a compressed message: the index (within
 *                                 the session's frames of this batch) of its first frame, to be
 *                                 re-sent with WSG_DESC_REPLAY; the state stays at that message's
 *                                 start.  0xFFFFFFFF otherwise.
 * no_context: PerMessageDeflateDecoder(noContext) — a new inflater (empty window) per message. */
int wsg_inflate_batch_device(wsg_ctx* ctx, int no_context,
                             const wsg_frame_desc* desc, uint64_t n_frames,
                             const uint32_t* session_first, uint32_t n_sessions,
                             const uint8_t* payload, uint64_t payload_len,
                             wsg_inflate_state* state, uint8_t* window,
                             uint8_t* out, const uint64_t* out_off,
                             wsg_frame_desc* out_desc, wsg_session_result* out_result,
                             uint32_t* replay_from);
/* Same contract with host pointers: H2D, inflate, D2H of out, descriptors, results,
 * state and window; synchronises. */
int wsg_inflate_batch_host(wsg_ctx* ctx, int no_context,
                           const wsg_frame_desc* desc, uint64_t n_frames,
                           const uint32_t* session_first, uint32_t n_sessions,
                           const uint8_t* payload, uint64_t payload_len,
                           wsg_inflate_state* state, uint8_t* window,
                           uint8_t* out, const uint64_t* out_off,
                           wsg_frame_desc* out_desc, wsg_session_result* out_result,
                           uint32_t* replay_from);

/* ---------------- permessage-deflate encode (PerMessageDeflateEncoder) ---------------- */
/* Per-session carry of PerMessageDeflateEncoder / DeflateEncoder / its raw ZlibEncoder's
 * java.util.zip.Deflater (PerMessageDeflateEncoder.java:41, DeflateEncoder.java:42-46,
 * ZlibEncoder.java:49): the scalars of zlib's deflate_state that outlive a
 * deflate(Z_SYNC_FLUSH) call; the window and hash tables are in the session's
 * WSG_DEFLATE_SESSION_BYTES block (zlib's layout: window[65536], head[32768] and
 * prev[32768] as 16-bit window indices). */
typedef struct wsg_deflate_state {
    uint32_t strstart;     /* deflate_state.strstart: window index of the next byte */
    uint32_t high_water;   /* .high_water: window bytes ever written or zeroed */
    uint16_t insert;       /* .insert: trailing strings not yet hashed (<= 2) */
    uint8_t has_deflater;  /* DeflateEncoder.encoder != null (a Deflater exists) */
    uint8_t compressing;   /* PerMessageDeflateEncoder.compressing */
    uint32_t reserved;
} wsg_deflate_state; /* 16 bytes; zeros = a new session */

#define WSG_DEFLATE_SESSION_BYTES (65536u + 2u * 32768u * 2u) /* window + head + prev */
#define WSG_DESC_DEFLATED 0x02 /* output desc.flags: payload in `out` (else the input payload) */

/* Device-resident PerMessageDeflateEncoder over a batch of outgoing frames: its encode()
 * once per frame per session in order (PerMessageDeflateEncoder.java:81-99 over
 * DeflateEncoder.java:62-104 and ZlibEncoder.encode, ZlibEncoder.java:223-287).  A
 * TEXT/BINARY frame without RSV1, and the continuations of such a message, are compressed:
 * one zlib deflate(Z_SYNC_FLUSH) of the payload on the session's raw deflater (windowBits
 * -15, memLevel 8, `level`), byte-identical to java.util.zip.Deflater's; the 00 00 FF FF
 * tail is removed from a final fragment, an empty payload becomes one 00 byte, RSV1 is set
 * on TEXT/BINARY.  Other frames pass through.  no_context: PerMessageDeflateEncoder(level,
 * true) — the deflater is dropped after every final fragment.
 *   desc[n_frames], payload      the frames to send (payload_off / payload_len / opcode /
 *                                flags: bit 7 FIN, bits 4-6 RSV)
 *   session_first[0..n_sessions] session s owns frames [session_first[s], session_first[s+1])
 *   state[n_sessions], session_mem[n_sessions * WSG_DEFLATE_SESSION_BYTES]   carry in / out
 *   out[out_cap]                 compressed payloads (a 16-B aligned slot per frame, up to
 *                                ZlibEncoder.deflateBound(len) bytes)
 *   out_desc[n_frames]           per frame: the payload to send — in `out` (WSG_DESC_DEFLATED)
 *                                or the input payload — and its opcode, FIN and RSV bits
 *   *out_total (host)            bytes of `out` the batch's slots span
 * Synchronises once (the slot sizes are planned on the device and read back).  Returns
 * WSG_API_ERANGE when out_cap is too small (nothing compressed, the state unchanged). */
int wsg_deflate_batch_device(wsg_ctx* ctx, int level, int no_context,
                             const wsg_frame_desc* desc, uint64_t n_frames,
                             const uint32_t* session_first, uint32_t n_sessions,
                             const uint8_t* payload, uint64_t payload_len,
                             wsg_deflate_state* state, uint8_t* session_mem,
                             uint8_t* out, uint64_t out_cap, wsg_frame_desc* out_desc,
                             uint64_t* out_total);
/* Same contract with host pointers: H2D, compress, D2H of the used out bytes, descriptors,
 * state and session_mem; synchronises. */
int wsg_deflate_batch_host(wsg_ctx* ctx, int level, int no_context,
                           const wsg_frame_desc* desc, uint64_t n_frames,
                           const uint32_t* session_first, uint32_t n_sessions,
                           const uint8_t* payload, uint64_t payload_len,
                           wsg_deflate_state* state, uint8_t* session_mem,
                           uint8_t* out, uint64_t out_cap, wsg_frame_desc* out_desc,
                           uint64_t* out_total);

/* ---------------- opening handshake, server side ------- */
/* Replaces, for a batch of server sessions whose handshake request arrives
 * together (a connection storm), the read-loop pair
 *   HandshakeDecoder.available/decode   handshake/HandshakeDecoder.java:141-235
 *     (HttpUtils.available/splitRequestLine/splitHeaderField HttpUtils.java:77-220,
 *      HandshakeFactory.parse/parseFields HandshakeFactory.java:47-127,
 *      HandshakeFrame.addValue HandshakeFrame.java:74-91)
 *   Handshaker.handshake(request) -> accept   handshake/Handshaker.java:208-405,555-578
 *     (HandshakeUtils.parseKey/generateAnswerKey HandshakeUtils.java:93-115, Base64Util)
 * and formats the response the way HandshakeEncoder/HandshakeFactory.format do
 * (HandshakeFactory.java:129-158).  One GPU lane per request.
 *
 * The lane resolves every request whose form it can decide exactly; the rest come
 * back as WSG_HS_DEFER for the Java Handshaker (the policy layer that stays on the
 * host): folded or name-continued header lines, a repeated Upgrade/Connection/
 * Host/Sec-WebSocket-* field, non-ASCII bytes in the request line or those fields,
 * request URIs outside [A-Za-z0-9-._~!*'()/?=&+,;$] and %XX (java.net.URI decides
 * the rest), Host values outside [A-Za-z0-9.-:], subprotocol / extension offers
 * when the config supports any, a config with its own acceptRequestUri or
 * customizeHeaders, and frames of more lines than one HandshakeDecoder chunk (50). */
#define WSG_HS_RESP_STRIDE 160   /* response bytes reserved per request */

typedef struct wsg_hs_config {
    uint32_t max_length;      /* getMaxHandshakeFrameLength() (65536) */
    uint8_t ignore_host;      /* ignoreHostHeaderField() */
    uint8_t subprotocols;     /* getSupportedSubProtocols() != null: offers are deferred */
    uint8_t extensions;       /* getSupportedExtensions() != null: offers are deferred */
    uint8_t host_policy;      /* acceptRequestUri/customizeHeaders overridden: accepts are deferred */
} wsg_hs_config;

typedef enum wsg_hs_kind {
    WSG_HS_NEED_MORE = 0,     /* no complete frame yet (available() == 0) */
    WSG_HS_DEFER = 1,         /* the Java HandshakeDecoder/Handshaker takes this request */
    WSG_HS_PARSE_ERROR = 2,   /* HandshakeDecoder: writenf(HandshakeResponse(status)) + exception (:194-203) */
    WSG_HS_ACCEPT = 3,        /* Handshaker.accept returned a response (101 or a refusal) */
    /* client side (wsg_handshake_validate_batch_*) */
    WSG_HS_FINISHED = 4,      /* Handshaker.validate(response) true: the session switches (:557-560) */
    WSG_HS_CLOSING = 5        /* validate false: the session closes with getClosingReason() (:561-563) */
} wsg_hs_kind;

typedef enum wsg_hs_cause {
    WSG_HSC_NONE = 0,
    WSG_HSC_BAD_REQUEST_LINE = 1,    /* "Invalid http request"              HandshakeFactory.java:100 */
    WSG_HSC_BAD_VERSION = 2,         /* "Invalid http request version"      :103 */
    WSG_HSC_FORBIDDEN = 3,           /* "Forbidden http request command"    :106 (403) */
    WSG_HSC_TOO_LARGE = 4,           /* "Handshake frame too large"         HandshakeDecoder.java:169 (413) */
    WSG_HSC_MISSING_VERSION = 5,     /* "Missing websocket version"         Handshaker.java:232 */
    WSG_HSC_INCORRECT_VERSION = 6,   /* "Incorrect websocket version: %s"   :219 (detail = the token) */
    WSG_HSC_UNSUPPORTED_VERSION = 7, /* "Unsupported websocket version: %s" :229 (426; detail = the value) */
    WSG_HSC_MISSING_UPGRADE = 8,     /* "Missing websocket upgrade"         :425 */
    WSG_HSC_MISSING_CONNECTION = 9,  /* "Missing websocket connection"      :429 */
    WSG_HSC_INVALID_UPGRADE = 10,    /* "Invalid websocket upgrade: %s"     :441 */
    WSG_HSC_INVALID_CONNECTION = 11, /* "Invalid websocket connection: %s"  :437 */
    WSG_HSC_MISSING_HOST = 12,       /* "Missing websocket request host"    :336 */
    WSG_HSC_MISSING_KEY = 13,        /* "Missing websocket key"             :254 */
    WSG_HSC_INVALID_KEY = 14,        /* "Invalid websocket key: %s"         :251 */
    /* client side: HandshakeDecoder(clientMode) exceptions and Handshaker.validate reasons */
    WSG_HSC_BAD_RESPONSE_LINE = 15,     /* "Invalid http response"          HandshakeFactory.java:110 */
    WSG_HSC_BAD_RESPONSE_VERSION = 16,  /* "Invalid http response version"  :113 */
    WSG_HSC_BAD_RESPONSE_STATUS = 17,   /* "Invalid http response status"   :119 */
    WSG_HSC_INVALID_STATUS = 18,        /* "Invalid websocket response status: %d" Handshaker.java:542 (http_status) */
    WSG_HSC_MISSING_ACCEPT = 19,        /* "Missing websocket key challenge" :458 */
    WSG_HSC_INVALID_ACCEPT = 20,        /* "Invalid websocket key challenge. Actual: %s. Expected: %s" :455
                                           (detail = actual; expected = the 28 bytes at expected_out) */
    WSG_HSC_MISSING_SUBPROTOCOL = 21,   /* "Missing websocket sub protocol" :476 */
    WSG_HSC_INVALID_SUBPROTOCOL = 22,   /* "Invalid websocket sub protocol: %s" :483 */
    WSG_HSC_INVALID_EXTENSIONS = 23,    /* validateExtensions false with no reason set (:529-532): null */
    /* why a request was deferred (WSG_HS_DEFER) */
    WSG_HSC_D_LINE_FORM = 32, WSG_HSC_D_REPEATED = 33, WSG_HSC_D_NON_ASCII = 34, WSG_HSC_D_URI = 35,
    WSG_HSC_D_HOST = 36, WSG_HSC_D_SUBPROTOCOL = 37, WSG_HSC_D_EXTENSION = 38, WSG_HSC_D_POLICY = 39,
    WSG_HSC_D_LINES = 40
} wsg_hs_cause;

typedef struct wsg_hs_result {
    uint32_t frame_len;    /* handshake frame bytes (HandshakeDecoder.available); the rest of the
                              request buffer is the first WebSocket bytes of the session */
    uint16_t http_status;  /* 101, 400, 403, 413, 426 (0 for NEED_MORE / DEFER) */
    uint8_t kind;          /* wsg_hs_kind */
    uint8_t cause;         /* wsg_hs_cause: the exception message or Handshaker closing reason */
    uint16_t resp_len;     /* bytes of the formatted response at resp + i * WSG_HS_RESP_STRIDE */
    uint16_t detail_len;   /* the %s of the cause: request bytes [detail_off, +detail_len) */
    uint32_t detail_off;
} wsg_hs_result; /* 16 bytes */

/* HttpUtils.available over one request buffer with HandshakeDecoder's default chunk
 * (50 lines): the frame length, or 0 (no complete frame / the chunk is full). */
int wsg_handshake_available(const uint8_t* data, uint64_t len);

/* Requests i in [0, n): req[req_off[i], req_off[i+1]) (device pointers, req and resp
 * 16-B aligned).  Writes
 * result[i] and, for PARSE_ERROR / ACCEPT, the response bytes to
 * resp[i * WSG_HS_RESP_STRIDE, + resp_len). */
int wsg_handshake_accept_batch_device(wsg_ctx* ctx, const wsg_hs_config* cfg, const uint8_t* req,
                                      const uint64_t* req_off, uint32_t n, uint8_t* resp, wsg_hs_result* result);
/* Same with host pointers (H2D, kernel, D2H). */
int wsg_handshake_accept_batch_host(wsg_ctx* ctx, const wsg_hs_config* cfg, const uint8_t* req,
                                    const uint64_t* req_off, uint32_t n, uint8_t* resp, wsg_hs_result* result);

/* Client side of the opening handshake (a client opening many connections at once):
 *   HandshakeDecoder(clientMode = true).available/decode   HandshakeDecoder.java:141-235
 *     (HandshakeFactory.parse, response branch            HandshakeFactory.java:108-123)
 *   Handshaker.handshake(response) -> validate            Handshaker.java:420-544, 555-566
 *     (validateBasicFields / validateKeyChallenge / validateSubProtocol / validateExtensions)
 * Response i is resp[resp_off[i], resp_off[i+1]) (the bytes the session has received;
 * resp and expected_out 16-B aligned, keys 4-B aligned);
 * keys[24 i, +24) is the Sec-WebSocket-Key the session sent (HandshakeUtils.generateKey:
 * Base64 of 16 bytes).  result[i].kind is NEED_MORE, DEFER, PARSE_ERROR (the exception
 * HandshakeDecoder throws in client mode: no response is written), FINISHED or CLOSING
 * (cause = the closing reason, http_status = the response status).  expected_out[32 i,
 * +28) receives Base64(SHA-1(key + GUID)) once the frame is complete (resp_len = 28).
 * cfg: max_length; subprotocols / extensions = the config lists are non-empty.
 * Deferred to the Java Handshaker: the header forms the server side defers (folded or
 * name-only lines, repeats of Upgrade/Connection/Sec-WebSocket-Accept/-Protocol/
 * -Extensions, non-ASCII bytes in those), a Sec-WebSocket-Protocol answer when the
 * config lists subprotocols (a string match against the list), and an extensions
 * answer when it lists extensions (IExtension.validateResponse). */
#define WSG_HS_EXPECTED_STRIDE 32
int wsg_handshake_validate_batch_device(wsg_ctx* ctx, const wsg_hs_config* cfg, const uint8_t* resp,
                                        const uint64_t* resp_off, const uint8_t* keys, uint32_t n,
                                        uint8_t* expected_out, wsg_hs_result* result);
/* Same with host pointers (H2D, kernel, D2H). */
int wsg_handshake_validate_batch_host(wsg_ctx* ctx, const wsg_hs_config* cfg, const uint8_t* resp,
                                      const uint64_t* resp_off, const uint8_t* keys, uint32_t n,
                                      uint8_t* expected_out, wsg_hs_result* result);

#ifdef __cplusplus
}
#endif
#endif /* WSGPU_H */
