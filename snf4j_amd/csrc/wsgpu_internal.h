// wsgpu_internal.h — device workspace layout and launch interface shared by the
// kernels (decode.hip, encode.hip, ...) and the C ABI (api.hip).
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "ws_rules.h"

namespace ws {

// Per-frame record of the decode pipeline (24 B, written once by k_parse; k_link's
// per-frame outputs are the frame's wsg_frame_desc and vflag).
struct FrameRec {
  uint64_t src;      // absolute wire offset of the payload
  uint32_t len;      // payload length (0 when the header failed a rule)
  uint32_t mask;     // mask key, little-endian u32 of the 4 wire bytes
  uint32_t code;     // packed: see CODE_*
  uint32_t sess;     // owning session
};

// FrameRec.code packing
constexpr uint32_t CODE_PRE_SHIFT = 0;      // 5 bits: rule error before the fragmentation test
constexpr uint32_t CODE_POST_SHIFT = 5;     // 5 bits: length / close rules after it
constexpr uint32_t CODE_FRAG_SHIFT = 10;    // 5 bits: fragmentation error (k_link)
constexpr uint32_t CODE_FIN = 1u << 16;
constexpr uint32_t CODE_RSV_SHIFT = 17;     // 3 bits
constexpr uint32_t CODE_MASKED = 1u << 20;
constexpr uint32_t CODE_OP_SHIFT = 24;      // 4 bits

__host__ __device__ inline uint32_t code_pre(uint32_t c) { return (c >> CODE_PRE_SHIFT) & 31u; }
__host__ __device__ inline uint32_t code_post(uint32_t c) { return (c >> CODE_POST_SHIFT) & 31u; }
__host__ __device__ inline uint32_t code_frag(uint32_t c) { return (c >> CODE_FRAG_SHIFT) & 31u; }
__host__ __device__ inline uint32_t code_op(uint32_t c) { return (c >> CODE_OP_SHIFT) & 15u; }
__host__ __device__ inline bool code_is_data(uint32_t c) { return code_op(c) <= 2u && !code_pre(c); }
__host__ __device__ inline bool code_is_start(uint32_t c) {
  return (code_op(c) == 1u || code_op(c) == 2u) && !code_pre(c);
}

constexpr int BLOCK = 256;    // frames per block in the encode passes
#ifndef WSG_AGG_BLOCK
#define WSG_AGG_BLOCK 512  // (256 and 1024 measured slower: profiles/r04_ab_aggblock.txt)
#endif
constexpr int ABLOCK = WSG_AGG_BLOCK;  // frames (threads) per block in the aggregator's plan passes
#ifndef WSG_DBLOCK
#define WSG_DBLOCK 256
#endif
constexpr int DBLOCK = WSG_DBLOCK;  // frames (threads) per block in the decode parse / link passes
constexpr uint32_t PIECE = 1024;  // payload-output bytes per wave in k_pieces (64 lanes x 16 B)
constexpr int PIECES_PER_WAVE = 2; // pieces one k_piecesN wave takes (tools/ubench_unmask)
#ifndef WSG_VPIECES
#define WSG_VPIECES 4
#endif
constexpr int VPIECES_PER_WAVE = WSG_VPIECES;  // validate-only mode (read-only stream)
#ifndef WSG_ENC_PIECES
#define WSG_ENC_PIECES 2
#endif
constexpr int ENC_PIECES_PER_WAVE = WSG_ENC_PIECES;  // k_enc_piecesN (1 and 2 within 1% once no array is promoted to LDS)

// Pieces needed for a batch, bounded from host-known sizes: the 16-B aligned
// payload slots total sum(align16(len)) <= wire_len - 2F + 15F.
__host__ __device__ inline uint64_t piece_bound(uint64_t wire_len, uint64_t n_frames) {
  return (wire_len + 16 * n_frames) / PIECE + 1;
}

// One 1 KiB piece of the payload output (16 B, one scalar load per wave).
struct PieceDesc {
  uint64_t info;  // bits 0-47: wire offset of the piece's first payload byte; 48-58: payload bytes in
                  // the piece (1..1024); 59: validate; 60: piece starts its frame; 61: spans several slots;
                  // 62: piece holds its frame's last payload byte; 63: the frame is FIN
  uint32_t mask;  // frame mask key (payload phase 0 at the piece start)
  uint32_t frame; // frame index | PDF_CONT
};
constexpr uint32_t PDF_INDEX = 0x3fffffffu;  // PieceDesc.frame: the frame index
constexpr uint32_t PDF_CONT = 0x80000000u;   // the frame is a continuation (its head is k_link's)
constexpr uint64_t PD_SRC_MASK = (1ull << 48) - 1;
constexpr uint32_t PD_NB_SHIFT = 48;
constexpr uint64_t PD_VALIDATE = 1ull << 59;
constexpr uint64_t PD_FIRST = 1ull << 60;
constexpr uint64_t PD_MULTI = 1ull << 61;
constexpr uint64_t PD_LAST = 1ull << 62;
constexpr uint64_t PD_FIN = 1ull << 63;

struct DecodeArgs {
  // inputs
  const uint8_t* wire;
  uint64_t wire_len;
  const uint64_t* frame_off;
  uint64_t n_frames;
  const uint32_t* session_first;
  uint32_t n_sessions;
  int32_t client_mode, allow_ext, validate;
  int64_t max_payload;
  // validator-only mode (wsg_validate_batch_*): frames come as descriptors of plain
  // payloads in `wire` (k_vparse instead of k_parse), no fragmentation rules, no stores
  int32_t validator_only;
  const wsg_frame_desc* in_desc;
  int32_t sparse;  // WSG_CFG_SPARSE: a frame's extent is its header's (frames need not be adjacent)
  // in/out
  wsg_session_state* state;
  // outputs
  uint8_t* payload_out;
  wsg_frame_desc* desc;
  wsg_session_result* result;
  // workspace
  FrameRec* rec;
  uint8_t* vflag;      // [n_frames]: the frame is validated (a text-message frame that passed every rule)
  int32_t* slink;      // [3][n_sessions]: of the session's last frame, the last data frame, the last
                       // message start (<= it) and the validator carry through it (k_link -> k_final)
  uint32_t* edge;      // [2][n_frames]: first 3 / last 3 payload bytes (unmasked); the last 3 only
                       // for non-FIN data frames (the carry into the next fragment or batch)
  uint64_t* blk_sum;   // [nblk] slot-bytes per block -> exclusive prefix
  int32_t* blk_max;    // [4][nblk] per-block max indices and UTF-8 carry -> exclusive prefix
  uint64_t* chunk_sum; // [nblk / SCAN_CHUNK + 1] k_scan chunk totals (grids beyond FUSED_SCAN_MAX_BLOCKS)
  int32_t* chunk_max;  // [nblk / SCAN_CHUNK + 1][4]
  uint64_t* sess_err;  // [n_sessions] first failing frame (~0 = none)
  uint64_t* total;     // [1] total payload slot bytes
  struct PieceDesc* pieces;  // [piece_bound]: per-piece work descriptor (k_link)
  uint64_t n_pieces;   // pieces the grid covers (piece_bound): slots beyond are a malformed batch
  uint32_t nblk;
  int32_t fused_scan;  // k_link reduces the block aggregates itself (nblk <= FUSED_SCAN_MAX_BLOCKS)
};

// grids up to this many parse/link blocks (DBLOCK frames each) skip the k_scan launch
constexpr uint32_t FUSED_SCAN_MAX_BLOCKS = 4096;
constexpr uint32_t SCAN_CHUNK = 4096;  // block aggregates per k_scan workgroup

struct EncodeArgs {
  int32_t client_mode;
  const uint8_t* payload;
  uint64_t payload_len;
  const wsg_encode_frame* frames;
  uint64_t n_frames;
  const uint32_t* session_first;
  uint32_t n_sessions;
  uint8_t* closed;
  uint8_t* wire_out;
  uint64_t wire_cap;
  uint64_t* wire_off;  // [n_frames+1]
  // workspace
  uint32_t* sess;      // [n_frames]
  uint64_t* blk_sum;   // [nblk]
  int32_t* blk_max;    // [nblk] last CLOSE frame index
  int32_t* last_close; // [n_frames] last CLOSE frame before k
  struct PieceDesc* pieces;  // [n_pieces]: 1 KiB pieces of wire_out (k_enc_desc -> k_enc_pieces)
  uint64_t n_pieces;
  uint32_t* pidx;      // [n_idx]: frame holding wire byte q * 64 KiB (k_enc_fix / k_enc_plan1)
  uint64_t n_idx;
  uint32_t nblk;
};

struct AggArgs {
  int64_t max_len;
  const wsg_frame_desc* desc;
  uint64_t n_frames;
  const uint32_t* session_first;
  uint32_t n_sessions;
  const wsg_session_result* dec_result;
  const uint8_t* payload;
  wsg_agg_state* state;
  uint8_t* agg_out;
  uint64_t agg_cap;
  wsg_frame_desc* out_desc;
  wsg_session_result* out_result;
  uint64_t* agg_total;
  // workspace
  uint32_t* code;      // [n] AG_* bits
  uint32_t* sess;      // [n]
  int32_t* last;       // [2][n] last start / last end before k (batch index, -1 = none)
  uint64_t* pl;        // [n] block-local exclusive member bytes
  uint64_t* cl;        // [n] block-local exclusive (emitted frames | gather units << 32)
  uint64_t* blk_sum;   // [nblk] member bytes of the block (k_agg_b)
  uint64_t* blk_cnt;   // [nblk] (emitted frames | gather units << 32) of the block (k_agg_b)
  uint64_t* pre_sum;   // [nblk] exclusive prefix of blk_sum (k_agg_c's fold, or k_agg_scan)
  uint64_t* pre_cnt;   // [nblk] exclusive prefix of blk_cnt
  int32_t* blk_max;    // [2][nblk] block maxima of start / end -> exclusive prefix
  uint64_t* sess_err;  // [n_sessions] first failing frame (~0 = none), idle between batches
  uint64_t* n_units;   // [1] gather units of the batch (k_agg_scan)
  struct PieceDesc* pieces;  // [n_pieces]: gather units (k_agg_c -> k_agg_gather)
  uint64_t n_pieces;         // bound on the units (agg_units_bound)
  uint32_t fold_max;         // plans of up to this many blocks fold their block aggregates
                             // (min(WSG_TUNE_AGG_FOLD_MAX, the LDS bound)); larger: k_agg_scan
  uint32_t nblk;
};

struct InflArgs {
  int32_t no_context;
  const wsg_frame_desc* desc;
  uint64_t n_frames;
  const uint32_t* session_first;
  uint32_t n_sessions;
  const uint8_t* payload;
  uint64_t payload_len;
  wsg_inflate_state* state;
  uint8_t* window;
  uint8_t* out;
  const uint64_t* out_off;
  wsg_frame_desc* out_desc;
  wsg_session_result* result;
  uint32_t* replay_from;
  // message-parallel pre-decode (k_infl_tok); tstat == nullptr: k_inflate decodes every frame
  uint32_t* tok;              // token regions (per frame: payload_off + 80 k words)
  uint8_t* lit;               // literal regions (per frame: 3 payload_off + 80 k bytes, 4-B aligned)
  uint64_t lit_len;           // bytes allocated at lit
  struct InflTokStat* tstat;  // [n_frames]
  uint8_t* tab;               // n_tab table blocks for the lanes that take the HBM-table decoder
  uint32_t n_tab;             //   (a lane takes one when it first needs it, from *tab_cnt;
  uint32_t* tab_cnt;          //   with none left its message goes to the serial decoder)
  uint32_t n_lanes;
  uint8_t* fast_done;         // [n_sessions]: k_infl_fast finished the session (k_inflate skips it)
  int tok_lds;                // k_infl_tok decodes single-frame messages from LDS tables (else HBM tables)
  uint32_t* order;            // [n_frames] frame order for k_infl_tok's lanes (longest first), or null
  uint32_t* ord_cnt;          // [ORD_BUCKETS] its counting-sort buckets
  int split;                  // k_infl_tok<true>: lane pairs, split-lane decode of each message
  uint32_t* tok2;             // the split's tail regions (laid out as tok / lit)
  uint8_t* lit2;
  unsigned long long* split_cnt;  // [1] messages a split decoded (accumulates), or null
  const uint32_t* tmap;       // [n_frames] frame k's index in the pre-decode's own frame list (the
                              // batcher's two-phase inflate: ~0u = not pre-decoded), or null: k
};

struct InflTokStat {
  uint32_t ok, n_tok, n_lit, out_len;
};

// permessage-deflate compression (deflate.hip).  Per frame: DF_* flags; per session the
// planned sizes of its regions (S stream, output, symbols, match chunks), scanned into bases.
constexpr uint32_t DF_KIND = 3u;          // PMD_PASS / PMD_CALL / PMD_EMPTY
constexpr uint32_t DF_DROP = 1u << 2;     // the deflater is discarded after this frame (noContext, FIN)
constexpr uint32_t DF_SEG = 1u << 3;      // a CALL that starts a new deflater (fresh window)
constexpr uint32_t DF_RSV_SHIFT = 4;      // 3 bits: RSV after encoding
constexpr uint32_t DF_FIN = 1u << 9;
constexpr uint32_t DF_START_SLID = 1u << 10;  // geometry: the call-start slide put strstart at MAX_DIST
constexpr uint32_t DF_TAIL_OK = 1u << 11;     // geometry: a slide can fall inside the frame's last bytes
constexpr uint32_t DF_PERSIST = 1u << 12;     // the call's deflater outlives the batch
constexpr uint32_t DEFL_CH = 256;         // positions a k_defl_match wave takes
constexpr uint32_t DEFL_TAILN = 264;      // positions whose match reads pass the frame's end
constexpr uint32_t DEFL_HIST = 32768;     // S-region bytes before the first call (the history)
constexpr uint32_t DEFL_PAD = 288;        // S-region bytes after the last call
constexpr uint32_t DEFL_RING = 49152;     // k_defl_match_lds: stream positions its LDS ring holds
constexpr uint32_t DEFL_LDS_MAXLEN = DEFL_RING - 32506 - 16;   // frames up to this long take the LDS walk

struct DeflFrame {   // per CALL frame (k_defl_plan)
  uint32_t s_rel;    // S-region offset of the frame's first byte (stream position)
  uint32_t start_w;  // strstart after the call-start fill_window
  uint32_t len;
  uint32_t sess;
  uint32_t blk_rel;  // first block slot within the session's (k_defl_plan)
  uint32_t nblk;     // blocks zlib flushes for the frame (k_defl_parse)
};

// One deflate block (k_defl_parse -> k_defl_trees -> k_defl_emit).
struct DeflBlock {
  uint64_t sym0;        // first symbol (index into the symbol buffers)
  uint32_t nsym;        // 0: an unused slot
  uint32_t stored_s;    // the block's bytes: session-local stream position, length
  uint32_t stored_len;
  uint32_t bits;        // static / dynamic: bits after the 3-bit header (k_defl_trees)
  uint8_t stored_ok;    // zlib's block_start >= 0 (a stored block is possible)
  uint8_t type;         // 0 stored, 1 static trees, 2 dynamic trees
  uint8_t dcodes, blcodes;
  uint16_t lcodes, pad;
  uint32_t ltab[286];   // dynamic: literal/length code | length << 16
  uint32_t dtab[30];    // distance codes
  uint32_t btab[19];    // bit-length codes, by bit-length symbol
  uint16_t freq[286 + 30];   // symbol frequencies (k_defl_hist): literal/length, then distance
};
constexpr uint32_t defl_blk_cap(uint32_t len) { return len / 16383u + 1u; }   // blocks a frame can need

struct DeflSess {    // per session (k_defl_plan; k_defl_prep fills hw)
  uint32_t sw_final;    // strstart after the batch's last call (before a slide in its tail)
  uint32_t hw_final;    // high_water after it (k_defl_prep)
  uint32_t last_call;   // frame index of the last call, ~0u none
  uint8_t has_deflater, compressing, first_fresh, persist;
};

struct DeflArgs {
  int32_t level, no_context, serial;
  int32_t match_lds;        // k_defl_match_lds walks the frames up to DEFL_LDS_MAXLEN (their fast range)
  const wsg_frame_desc* desc;
  uint64_t n_frames;
  const uint32_t* session_first;
  uint32_t n_sessions;
  const uint8_t* payload;
  wsg_deflate_state* state;
  uint8_t* smem;            // n_sessions * WSG_DEFLATE_SESSION_BYTES: window | head | prev
  uint8_t* out;
  uint64_t out_cap;
  wsg_frame_desc* out_desc;
  // workspace
  uint32_t* fflags;         // [n_frames] DF_*
  uint64_t* fout;           // [n_frames] output offset within the session's output region
  uint64_t* fsym;           // [n_frames] symbol-buffer offset within the session's region (words)
  DeflFrame* ff;            // [n_frames]
  DeflSess* fs;             // [n_sessions]
  uint64_t* sums;           // [5][n_sessions + 1]: S bytes, output bytes, symbol words, chunks, block slots
                            // -> exclusive
  uint8_t* S;               // stream regions
  uint16_t* link;           // [S]: distance to the previous string of its hash (0: none / >= 32 KiB)
  uint32_t* res;            // [2 x S]: match_at results at the calls' positions (full, quarter)
  uint32_t* tres;           // [n_frames][DEFL_TAILN][2]: the same after a slide in the frame's tail
  uint8_t* strips;          // [n_frames][2][zd::STRIP]: window bytes after the frame's end (before/after)
  uint8_t* ftail;           // [n_frames]: the parse saw a slide in the frame's tail
  uint64_t* chunks;         // [chunk bound]: frame | chunk << 32 | tail variant << 63
  uint64_t chunk_cap;
  uint32_t* sym;            // symbol buffers
  DeflBlock* blocks;        // block slots
  void* tw;                 // zd::TreeWork per parse lane
  uint32_t n_lanes;         // parse lanes (grid-stride over frames)
  uint32_t* ssym;           // serial path: [n_sessions][zd::LIT_BUFSIZE]
};

// kernel ids for timing
enum KernelId {
  K_PARSE = 0, K_SCAN, K_LINK, K_UNMASK, K_FINAL,
  K_ENC_LEN, K_ENC_SCAN, K_ENC_EMIT, K_ENC_FINAL, K_ENC_DESC, K_AGG, K_AGG_GATHER, K_INFLATE, K_HS_ACCEPT, K_INFL_TOK, K_INFL_FAST, K_HS_VALIDATE,
  K_DEFL_PLAN, K_DEFL_PREP, K_DEFL_MATCH, K_DEFL_PARSE, K_DEFL_FINAL, K_DEFL_SERIAL, K_DEFL_TREES, K_DEFL_EMIT,
  K_DEFL_HIST, K_DEFL_MATCH_LDS, K_DEFL_LINKS, K_COUNT
};

// launchers (enqueue on `s`; the timing hook wraps each one)
// the context's pipelined host path (api.hip), for the native batcher: wait until the
// previous async batch's state download is done; record `e` after everything queued
// on the copy-out stream
hipError_t ctx_wait_prev_state(wsg_ctx* c);
hipError_t ctx_record_out(wsg_ctx* c, hipEvent_t e);
// the context's kernel stream, and the device payload of its last async batch (valid
// in stream order until a later batch reuses that staging slot)
hipStream_t ctx_stream(wsg_ctx* c);
hipStream_t ctx_out_stream(wsg_ctx* c);
void ctx_copy_tuning(wsg_ctx* dst, const wsg_ctx* src);  // where ctx_record_out records (the download stream)
int ctx_device(wsg_ctx* c);
bool ctx_inflate_two_phase(const wsg_ctx* c);
uint8_t* ctx_async_payload(wsg_ctx* c);
bool ctx_stage_fail(wsg_ctx* c);  // WSG_TUNE_STAGE_FAIL: this stage step is the one to fail
uint64_t ctx_alloc_count();  // device workspace allocations of every context so far
int ctx_reserve_stages(wsg_ctx* c, uint64_t max_frames, uint32_t max_sessions, uint64_t payload_len,
                       uint64_t agg_cap);
// permessage-deflate in two phases (the batcher's pipelined stage chain): the message-
// parallel pre-decode of a flush's frames on context `tokc` (k_infl_tok; it needs no
// inflater state, so it runs ahead of the previous flush's replay), then the replay and
// the serial decoder on context c over a frame list whose frame k is the pre-decode's
// frame tmap[k] (the list may add replayed frames); tokc's workspace must hold that
// pre-decode until the replay has run (its stream ordered after tokc's by the caller).
int inflate_tok_phase(wsg_ctx* tokc, const wsg_frame_desc* desc, uint64_t n_frames, const uint32_t* session_first,
                      uint32_t n_sessions, const uint8_t* payload, uint64_t payload_len);
int inflate_replay_phase(wsg_ctx* c, wsg_ctx* tokc, const uint32_t* tmap, int no_context, const wsg_frame_desc* desc,
                         uint64_t n_frames, const uint32_t* session_first, uint32_t n_sessions, const uint8_t* payload,
                         uint64_t payload_len, wsg_inflate_state* state, uint8_t* window, uint8_t* out,
                         const uint64_t* out_off, wsg_frame_desc* out_desc, wsg_session_result* out_result,
                         uint32_t* replay_from);

void launch_parse(const DecodeArgs& a, hipStream_t s);
void launch_scan(const DecodeArgs& a, hipStream_t s);
void launch_link(const DecodeArgs& a, hipStream_t s);
void launch_pieces(const DecodeArgs& a, hipStream_t s, uint64_t n_pieces_bound);
void launch_vparse(const DecodeArgs& a, hipStream_t s);
void launch_vpieces(const DecodeArgs& a, hipStream_t s, uint64_t n_pieces_bound);
void launch_final(const DecodeArgs& a, hipStream_t s);

void launch_enc_len(const EncodeArgs& a, hipStream_t s);
void launch_enc_scan(const EncodeArgs& a, hipStream_t s);
void launch_enc_desc(const EncodeArgs& a, hipStream_t s);
void launch_enc_pieces(const EncodeArgs& a, hipStream_t s);
void launch_enc_final(const EncodeArgs& a, hipStream_t s);

uint32_t agg_fold_bound();  // the largest plan (blocks) k_agg_c's LDS can fold
void launch_agg_plan(const AggArgs& a, hipStream_t s);
void launch_agg_gather(const AggArgs& a, hipStream_t s, uint64_t src_lim, int per_wave, uint32_t grid_cap);

void launch_inflate(const InflArgs& a, hipStream_t s);
void launch_infl_tok(const InflArgs& a, hipStream_t s);
void launch_infl_fast(const InflArgs& a, hipStream_t s);
uint64_t infl_tok_words(uint64_t payload_len, uint64_t n_frames);
uint64_t infl_lit_bytes(uint64_t payload_len, uint64_t n_frames);
uint64_t infl_ord_words(uint64_t n_frames);  // order + bucket counts
uint64_t infl_tab_bytes();

// Upper bounds of the plan's five region totals (S bytes, output bytes, symbol words, match
// chunks, block slots) from the frames' lengths alone: _add per frame, _session per session
// with frames.  deflate_launch with bounds sizes its workspace from them and reads nothing back.
struct DeflBounds {
  uint64_t tot[5] = {0, 0, 0, 0, 0};
};
void deflate_bounds_add(DeflBounds& b, uint32_t len);
void deflate_bounds_session(DeflBounds& b);
int deflate_launch(wsg_ctx* c, int level, int no_context, const wsg_frame_desc* desc, uint64_t n_frames,
                   const uint32_t* session_first, uint32_t n_sessions, const uint8_t* payload,
                   wsg_deflate_state* state, uint8_t* session_mem, uint8_t* out, uint64_t out_cap,
                   wsg_frame_desc* out_desc, const DeflBounds* bounds, uint64_t* out_total);

void launch_defl_plan(const DeflArgs& a, hipStream_t s);    // k_defl_plan + k_defl_scan
void launch_defl_prep(const DeflArgs& a, hipStream_t s);
void launch_defl_match(const DeflArgs& a, hipStream_t s);
void launch_defl_match_lds(const DeflArgs& a, hipStream_t s);
void launch_defl_links(const DeflArgs& a, hipStream_t s);
void launch_defl_parse(const DeflArgs& a, hipStream_t s);
void launch_defl_hist(const DeflArgs& a, hipStream_t s, uint64_t n_blocks);
void launch_defl_trees(const DeflArgs& a, hipStream_t s, uint64_t n_blocks);
void launch_defl_emit(const DeflArgs& a, hipStream_t s);
void launch_defl_final(const DeflArgs& a, hipStream_t s);
void launch_defl_serial(const DeflArgs& a, hipStream_t s);
size_t defl_treework_bytes();
constexpr uint64_t zd_lit_bufsize() { return 16384; }   // zd::LIT_BUFSIZE
constexpr uint64_t zd_strip() { return 260; }         // zd::STRIP

void launch_hs_accept(const wsg_hs_config& cfg, const uint8_t* req, const uint64_t* req_off, uint32_t n,
                      uint8_t* resp, wsg_hs_result* result, hipStream_t s);
void launch_hs_validate(const wsg_hs_config& cfg, const uint8_t* resp, const uint64_t* resp_off, const uint8_t* keys,
                        uint32_t n, uint8_t* expected, wsg_hs_result* result, hipStream_t s);
__host__ __device__ int hs_frame_len(const uint8_t* d, int64_t len, int* capped, int64_t* lines_end);


}  // namespace ws
