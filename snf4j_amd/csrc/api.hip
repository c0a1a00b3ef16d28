// api.hip — the C ABI of libwsgpu.so (include/wsgpu.h): context, workspace,
// kernel timing, device/host batch entry points, host-side framing helpers.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <vector>

#include "wsgpu_internal.h"

using namespace ws;

namespace {

std::atomic<uint64_t> g_ctx_allocs{0};  // device workspace allocations of every context

const char* const kKernelNames[K_COUNT] = {"k_parse",   "k_scan",     "k_link",     "k_piecesN",
                                           "k_final",    "k_enc_len",  "k_enc_scan",
                                           "k_enc_piecesN", "k_enc_final", "k_enc_desc", "k_agg_plan", "k_agg_gather", "k_inflate", "k_hs_accept", "k_infl_tok", "k_infl_fast", "k_hs_validate",
                                           "k_defl_plan", "k_defl_prep", "k_defl_match", "k_defl_parse", "k_defl_final", "k_defl_serial",
                                           "k_defl_trees", "k_defl_emit", "k_defl_hist", "k_defl_match_lds", "k_defl_links"};

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  // (re)allocate to >= bytes; a fresh allocation is filled with `fill` (>= 0) on stream s
  hipError_t ensure(size_t bytes, int fill = -1, hipStream_t s = nullptr) {
    if (bytes <= n && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    size_t want = bytes < 256 ? 256 : bytes;
    hipError_t e = hipMalloc(&p, want);
    g_ctx_allocs.fetch_add(1, std::memory_order_relaxed);
    if (e != hipSuccess) return e;
    n = want;
    return fill >= 0 ? hipMemsetAsync(p, fill, want, s) : hipSuccess;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

struct EventPair {
  int kid;
  hipEvent_t a, b;
};

// One staging slot of the pipelined host path (wsg_decode_batch_host_async).
struct HostSlot {
  DevBuf wire, off, sf, state, payload, desc, result;
  hipEvent_t ev_in = nullptr, ev_k = nullptr, ev_state = nullptr, ev_out = nullptr;
  bool used = false;
};

}  // namespace

struct wsg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;
  // decode workspace
  DevBuf rec, vflag, slink, edge, blk_sum, blk_max, chunk, sess_err, total, pieces;
  // encode workspace
  DevBuf esess, elast_close, epieces, epidx;
  // aggregate workspace
  DevBuf a_code, a_last, a_pl, a_cl, a_blk, a_sess_err, a_pieces;
  DevBuf v_desc;  // validator-only mode: per-frame status scratch
  DevBuf i_tok, i_lit, i_stat, i_tab, i_tabcnt, i_fast, i_ord;  // inflate pre-decode workspace
  DevBuf i_split;  // [1] u64: messages the split-lane decode took (wsg_inflate_split_count)
  DevBuf i_tok2, i_lit2;  // the split's tail regions
  // permessage-deflate compression workspace (deflate.hip, DeflArgs)
  DevBuf d_flags, d_fout, d_fsym, d_ff, d_fs, d_sums, d_S, d_link, d_res, d_tres, d_strips, d_ftail, d_chunks, d_sym, d_tw, d_ssym,
      d_blocks;
  int defl_serial = 0;               // WSG_TUNE_DEFLATE_SERIAL 1: zlib's loop per session at every level (tests)
  int64_t stage_fail = 0;            // WSG_TUNE_STAGE_FAIL n: the n-th stage step from now fails (tests)
  int defl_lds = 1;                  // WSG_TUNE_DEFLATE_LDS 0: the match search in global memory only
  // measurement / test switches (wsg_set_tuning; the defaults are the product)
  int infl_tokens = 1;               // WSG_TUNE_INFLATE_TOKENS 0: no lane pre-decode (serial decoder only)
  uint32_t infl_lanes = 262144;      // WSG_TUNE_INFLATE_LANES: k_infl_tok lanes at most
  uint32_t infl_tabs = 32768;        // HBM table blocks for the lanes that need them (WSG_TUNE_INFLATE_TABS)
  int infl_fast = 1;                 // WSG_TUNE_INFLATE_FAST 0: no parallel token replay; 2: it alone (tests)
  int infl_lds = 1;                  // WSG_TUNE_INFLATE_LDS 0: the pre-decode keeps its tables in HBM
  int infl_order = 1;                // WSG_TUNE_INFLATE_ORDER 0: lanes take frames in batch order
  int infl_split = 0;                // WSG_TUNE_INFLATE_SPLIT 0 (default): never, 1: batches that leave lanes idle, 2: always
                                     //   (measured slower end to end, DESIGN.md §9.1: kept as a switch)
  int fused_scan = 1;                // WSG_TUNE_FUSED_SCAN 0: always launch k_scan
  int agg_units = 2;                 // WSG_TUNE_AGG_UNITS: k_agg_gather units per wave (1, 2 or 4)
  uint32_t agg_grid = 65536;         // WSG_TUNE_AGG_GRID: k_agg_gather waves at most
  uint32_t agg_fold = 0xFFFFFFFFu;   // WSG_TUNE_AGG_FOLD_MAX: plan blocks folded at most (tests: 0 forces k_agg_scan)
  uint64_t tok_frames = 0, tok_payload_len = 0;  // the last ws::inflate_tok_phase's list (its workspace's layout)
  // host-path device buffers
  DevBuf h_wire, h_off, h_sf, h_state, h_payload, h_desc, h_result, h_frames, h_closed, h_wire_off;
  // pipelined host path: copy-in / copy-out streams and two staging slots
  hipStream_t s_in = nullptr, s_out = nullptr;
  HostSlot slot[2];
  int next_slot = 0;
  hipEvent_t ev_prev_state = nullptr;  // state download of the previous async batch
  uint8_t* last_async_payload = nullptr;  // device payload of the last async batch (batcher stages)
  // timing
  int timing = 0;  // 0 off, 1 every kernel, 2 the streaming kernels only (WSG_TIMING_*)
  uint32_t timing_every = 1;  // mode 2: bracket one launch in timing_every of a streaming kernel
  uint64_t timing_seen[K_COUNT] = {};
  std::vector<EventPair> pending;
  std::vector<hipEvent_t> free_events;
  double ms[K_COUNT] = {};
  uint64_t count[K_COUNT] = {};
};

static int set_err(wsg_ctx* c, int code, const char* fmt, ...) {
  if (c) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    c->err = buf;
  }
  return code;
}

#define HIP_TRY(c, expr)                                                                        \
  do {                                                                                          \
    hipError_t _e = (expr);                                                                     \
    if (_e != hipSuccess) return set_err((c), WSG_API_EHIP, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

static hipEvent_t get_event(wsg_ctx* c) {
  if (!c->free_events.empty()) {
    hipEvent_t e = c->free_events.back();
    c->free_events.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

static void drain_timing(wsg_ctx* c) {
  for (auto& p : c->pending) {
    (void)hipEventSynchronize(p.b);
    float t = 0.f;
    if (hipEventElapsedTime(&t, p.a, p.b) == hipSuccess) {
      c->ms[p.kid] += t;
      c->count[p.kid] += 1;
    }
    c->free_events.push_back(p.a);
    c->free_events.push_back(p.b);
  }
  c->pending.clear();
}

template <typename F>
static void timed(wsg_ctx* c, int kid, F&& f) {
  // an event pair costs a few microseconds of queue time: mode 2 brackets only the
  // streaming kernels, so a timed step keeps the side kernels back to back
  if (!c->timing || (c->timing == 2 && kid != K_UNMASK && kid != K_ENC_EMIT && kid != K_AGG_GATHER && kid != K_INFLATE && kid != K_HS_ACCEPT && kid != K_HS_VALIDATE && kid != K_INFL_TOK && kid != K_INFL_FAST && kid != K_DEFL_MATCH && kid != K_DEFL_PARSE && kid != K_DEFL_PREP && kid != K_DEFL_SERIAL && kid != K_DEFL_TREES && kid != K_DEFL_MATCH_LDS && kid != K_DEFL_LINKS &&
                                 kid != K_DEFL_EMIT && kid != K_DEFL_HIST)) {
    f();
    return;
  }
  if (c->timing == 2 && (c->timing_seen[kid]++ % c->timing_every) != 0) {
    f();
    return;
  }
  if (c->pending.size() > 4096) drain_timing(c);
  EventPair p{kid, get_event(c), get_event(c)};
  (void)hipEventRecord(p.a, c->stream);
  f();
  (void)hipEventRecord(p.b, c->stream);
  c->pending.push_back(p);
}

namespace ws {
hipError_t ctx_wait_prev_state(wsg_ctx* c) { return c->ev_prev_state ? hipEventSynchronize(c->ev_prev_state) : hipSuccess; }
hipError_t ctx_record_out(wsg_ctx* c, hipEvent_t e) { return hipEventRecord(e, c->s_out ? c->s_out : c->stream); }
hipStream_t ctx_stream(wsg_ctx* c) { return c->stream; }
hipStream_t ctx_out_stream(wsg_ctx* c) { return c->s_out ? c->s_out : c->stream; }
// a context's measurement / test switches (wsg_set_tuning) onto another (a batcher's stage context)
void ctx_copy_tuning(wsg_ctx* dst, const wsg_ctx* src) {
  dst->infl_tokens = src->infl_tokens;
  dst->infl_lanes = src->infl_lanes;
  dst->infl_tabs = src->infl_tabs;
  dst->infl_fast = src->infl_fast;
  dst->infl_lds = src->infl_lds;
  dst->infl_order = src->infl_order;
  dst->infl_split = src->infl_split;
  dst->fused_scan = src->fused_scan;
  dst->agg_units = src->agg_units;
  dst->agg_grid = src->agg_grid;
  dst->agg_fold = src->agg_fold;
  dst->defl_serial = src->defl_serial;
  dst->defl_lds = src->defl_lds;
}
int ctx_device(wsg_ctx* c) { return c->device; }
// the batcher's two-phase inflate applies (the pre-decode on, the split-lane decode off)
bool ctx_inflate_two_phase(const wsg_ctx* c) { return c->infl_tokens && c->infl_split == 0; }
uint8_t* ctx_async_payload(wsg_ctx* c) { return c->last_async_payload; }
bool ctx_stage_fail(wsg_ctx* c) { return c->stage_fail > 0 && --c->stage_fail == 0; }
}  // namespace ws

extern "C" {

int wsg_version(void) { return WSG_ABI_VERSION; }

int wsg_num_kernels(void) { return K_COUNT; }

const char* wsg_kernel_name(int kid) { return (kid >= 0 && kid < K_COUNT) ? kKernelNames[kid] : ""; }

int wsg_open(int device, void* stream, wsg_ctx** out) {
  if (!out) return WSG_API_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return WSG_API_EHIP;
  if (device < 0 || device >= n) return WSG_API_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return WSG_API_EHIP;
  wsg_ctx* c = new wsg_ctx();
  c->device = device;
  if (stream) {
    c->stream = (hipStream_t)stream;
  } else {
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
      delete c;
      return WSG_API_EHIP;
    }
    c->own_stream = true;
  }
  *out = c;
  return WSG_API_OK;
}

int wsg_close(wsg_ctx* c) {
  if (!c) return WSG_API_EINVAL;
  (void)hipSetDevice(c->device);
  if (c->s_in) (void)hipStreamSynchronize(c->s_in);
  (void)hipStreamSynchronize(c->stream);
  if (c->s_out) (void)hipStreamSynchronize(c->s_out);
  drain_timing(c);
  for (auto e : c->free_events) (void)hipEventDestroy(e);
  DevBuf* bufs[] = {&c->rec,     &c->vflag, &c->chunk,    &c->edge,     &c->blk_sum,  &c->blk_max,   &c->sess_err,
                    &c->total,   &c->pieces, &c->slink, &c->esess,   &c->elast_close, &c->epieces, &c->epidx, &c->h_wire, &c->h_off,    &c->h_sf,
                    &c->h_state, &c->h_payload, &c->h_desc, &c->h_result, &c->h_frames, &c->h_closed,
                    &c->h_wire_off};
  for (DevBuf* b : bufs) b->release();
  DevBuf* abufs[] = {&c->a_code, &c->a_last, &c->a_pl, &c->a_cl,
                     &c->a_blk,  &c->a_sess_err, &c->a_pieces, &c->v_desc, &c->i_tok, &c->i_lit,
                     &c->i_stat, &c->i_tab, &c->i_tabcnt, &c->i_fast, &c->i_ord, &c->i_split,
                     &c->i_tok2, &c->i_lit2};
  for (DevBuf* b : abufs) b->release();
  for (HostSlot& hs : c->slot) {
    DevBuf* sb[] = {&hs.wire, &hs.off, &hs.sf, &hs.state, &hs.payload, &hs.desc, &hs.result};
    for (DevBuf* b : sb) b->release();
    hipEvent_t evs[] = {hs.ev_in, hs.ev_k, hs.ev_state, hs.ev_out};
    for (hipEvent_t e : evs)
      if (e) (void)hipEventDestroy(e);
  }
  if (c->s_in) (void)hipStreamDestroy(c->s_in);
  if (c->s_out) (void)hipStreamDestroy(c->s_out);
  if (c->own_stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return WSG_API_OK;
}

int wsg_set_tuning(wsg_ctx* c, int key, int64_t value) {
  if (!c) return WSG_API_EINVAL;
  switch (key) {
    case WSG_TUNE_INFLATE_TOKENS: c->infl_tokens = value != 0; break;
    case WSG_TUNE_INFLATE_FAST: c->infl_fast = (int)value; break;
    case WSG_TUNE_INFLATE_LDS: c->infl_lds = value != 0; break;
    case WSG_TUNE_INFLATE_ORDER: c->infl_order = value != 0; break;
    case WSG_TUNE_INFLATE_LANES: c->infl_lanes = value < 64 ? 64u : (uint32_t)value & ~63u; break;
    case WSG_TUNE_INFLATE_SPLIT:
      if (value < 0 || value > 2) return set_err(c, WSG_API_EINVAL, "INFLATE_SPLIT is 0, 1 or 2");
      c->infl_split = (int)value;
      break;
    case WSG_TUNE_INFLATE_TABS: c->infl_tabs = value < 0 ? 0u : (value > (1 << 22) ? (1u << 22) : (uint32_t)value); break;
    case WSG_TUNE_FUSED_SCAN: c->fused_scan = value != 0; break;
    case WSG_TUNE_AGG_UNITS:
      if (value != 1 && value != 2 && value != 4) return set_err(c, WSG_API_EINVAL, "AGG_UNITS is 1, 2 or 4");
      c->agg_units = (int)value;
      break;
    case WSG_TUNE_AGG_GRID: c->agg_grid = value < 1 ? 1u : (value > (1 << 24) ? (1u << 24) : (uint32_t)value); break;
    case WSG_TUNE_DEFLATE_SERIAL: c->defl_serial = value != 0; break;
    case WSG_TUNE_STAGE_FAIL: c->stage_fail = value < 0 ? 0 : value; break;
    case WSG_TUNE_DEFLATE_LDS: c->defl_lds = value != 0; break;
    case WSG_TUNE_AGG_FOLD_MAX: c->agg_fold = value < 0 ? 0u : (value > 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)value); break;
    default: return set_err(c, WSG_API_EINVAL, "unknown tuning key");
  }
  return WSG_API_OK;
}

int wsg_set_stream(wsg_ctx* c, void* stream) {
  if (!c) return WSG_API_EINVAL;
  if (c->own_stream) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamDestroy(c->stream);
    c->own_stream = false;
  }
  c->stream = (hipStream_t)stream;
  return WSG_API_OK;
}

int wsg_get_stream(wsg_ctx* c, void** stream) {
  if (!c || !stream) return WSG_API_EINVAL;
  *stream = (void*)c->stream;
  return WSG_API_OK;
}

const char* wsg_last_error(wsg_ctx* c) { return c ? c->err.c_str() : "null context"; }

int wsg_sync(wsg_ctx* c) {
  if (!c) return WSG_API_EINVAL;
  if (c->s_in) HIP_TRY(c, hipStreamSynchronize(c->s_in));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (c->s_out) HIP_TRY(c, hipStreamSynchronize(c->s_out));
  return WSG_API_OK;
}

int wsg_set_timing_every(wsg_ctx* c, uint32_t every) {
  if (!c || every == 0) return WSG_API_EINVAL;
  c->timing_every = every;
  for (auto& n : c->timing_seen) n = 0;
  return WSG_API_OK;
}

int wsg_set_timing(wsg_ctx* c, int enable) {
  if (!c) return WSG_API_EINVAL;
  c->timing = enable == 2 ? 2 : (enable != 0 ? 1 : 0);
  return WSG_API_OK;
}

int wsg_get_timing(wsg_ctx* c, double* out_ms, uint64_t* out_count, int max_kernels) {
  if (!c) return WSG_API_EINVAL;
  drain_timing(c);
  for (int i = 0; i < K_COUNT && i < max_kernels; ++i) {
    if (out_ms) out_ms[i] = c->ms[i];
    if (out_count) out_count[i] = c->count[i];
  }
  return K_COUNT;
}

int wsg_reset_timing(wsg_ctx* c) {
  if (!c) return WSG_API_EINVAL;
  drain_timing(c);
  memset(c->ms, 0, sizeof c->ms);
  memset(c->count, 0, sizeof c->count);
  return WSG_API_OK;
}

static int ensure_decode_ws(wsg_ctx* c, uint64_t n_frames, uint32_t n_sessions, uint64_t wire_len) {
  const uint64_t F = n_frames ? n_frames : 1;
  const uint64_t nblk = (F + DBLOCK - 1) / DBLOCK;
  // + PIECES_PER_WAVE: k_piecesN reads its descriptors in groups
  HIP_TRY(c, c->pieces.ensure((piece_bound(wire_len, F) + 8) * sizeof(PieceDesc)));
  // sess_err is kept in its idle state between batches (k_final resets what it
  // reads), so no per-batch memset is needed
  HIP_TRY(c, c->rec.ensure(F * sizeof(FrameRec)));
  HIP_TRY(c, c->vflag.ensure(F));
  HIP_TRY(c, c->slink.ensure(3 * (uint64_t)(n_sessions ? n_sessions : 1) * sizeof(int32_t)));
  HIP_TRY(c, c->edge.ensure(2 * F * sizeof(uint32_t)));
  HIP_TRY(c, c->blk_sum.ensure(nblk * sizeof(uint64_t)));
  HIP_TRY(c, c->blk_max.ensure(4 * ((nblk + 3) & ~3ull) * sizeof(int32_t)));  // rows 16-B aligned (decode.hip blk_stride)
  HIP_TRY(c, c->chunk.ensure((nblk / SCAN_CHUNK + 1) * (sizeof(uint64_t) + 4 * sizeof(int32_t))));
  HIP_TRY(c, c->sess_err.ensure((uint64_t)(n_sessions ? n_sessions : 1) * sizeof(uint64_t), 0xff, c->stream));
  HIP_TRY(c, c->total.ensure(sizeof(uint64_t)));
  return WSG_API_OK;
}

static int ensure_encode_ws(wsg_ctx* c, uint64_t n_frames) {
  const uint64_t F = n_frames ? n_frames : 1;
  const uint64_t nblk = (F + BLOCK - 1) / BLOCK;
  HIP_TRY(c, c->esess.ensure(F * sizeof(uint32_t)));
  HIP_TRY(c, c->elast_close.ensure(F * sizeof(int32_t)));
  HIP_TRY(c, c->blk_sum.ensure(nblk * sizeof(uint64_t)));
  HIP_TRY(c, c->blk_max.ensure(3 * nblk * sizeof(int32_t)));
  return WSG_API_OK;
}

// the lane pre-decode's workspace for a batch of n_frames frames and payload_len
// compressed bytes (grow-only, so a batch within a reservation allocates nothing)
// k_infl_tok's lanes for a batch: a lane a frame, or (the split-lane decode) a pair of
// lanes a frame when the batch would leave the chip's resident lanes (256 CUs x 4
// workgroups of 64, what its LDS allows) half idle, or when tuned to always
static constexpr uint64_t INFL_RESIDENT_LANES = 65536;
static bool infl_pairs(const wsg_ctx* c, uint64_t n_frames) {
  return c->infl_lds && (c->infl_split == 2 || (c->infl_split == 1 && 2 * n_frames <= INFL_RESIDENT_LANES));
}
static uint64_t infl_lane_count(const wsg_ctx* c, uint64_t n_frames) {
  const uint64_t want = infl_pairs(c, n_frames) ? 2 * n_frames : n_frames;
  return want < c->infl_lanes ? ((want + 63) / 64) * 64 : c->infl_lanes;
}

static int ensure_inflate_ws(wsg_ctx* c, uint64_t n_frames, uint64_t payload_len) {
  const uint64_t lanes = infl_lane_count(c, n_frames);
  const uint64_t n_tab = lanes < c->infl_tabs ? lanes : c->infl_tabs;
  HIP_TRY(c, c->i_tok.ensure(infl_tok_words(payload_len, n_frames) * 4));
  HIP_TRY(c, c->i_lit.ensure(infl_lit_bytes(payload_len, n_frames)));
  HIP_TRY(c, c->i_stat.ensure(n_frames * sizeof(InflTokStat)));
  HIP_TRY(c, c->i_tab.ensure(n_tab * infl_tab_bytes()));
  HIP_TRY(c, c->i_tabcnt.ensure(sizeof(uint32_t)));
  if (c->infl_order) HIP_TRY(c, c->i_ord.ensure(infl_ord_words(n_frames) * 4));
  HIP_TRY(c, c->i_split.ensure(sizeof(uint64_t), 0, c->stream));
  if (infl_pairs(c, n_frames)) {
    HIP_TRY(c, c->i_tok2.ensure(infl_tok_words(payload_len, n_frames) * 4));
    HIP_TRY(c, c->i_lit2.ensure(infl_lit_bytes(payload_len, n_frames)));
  }
  return WSG_API_OK;
}

int wsg_reserve_inflate(wsg_ctx* c, uint64_t max_frames, uint32_t max_sessions, uint64_t max_payload_len) {
  if (!c) return WSG_API_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, c->i_fast.ensure(max_sessions ? max_sessions : 1));
  int rc = ensure_inflate_ws(c, max_frames, max_payload_len);
  if (rc) return rc;
  // a smaller batch within the reservation may take the split (2 n_frames <= the resident
  // lanes): its tail regions too
  const uint64_t split_frames = c->infl_split == 2 ? max_frames : std::min<uint64_t>(max_frames, INFL_RESIDENT_LANES / 2);
  if (c->infl_split && c->infl_lds && split_frames) {
    HIP_TRY(c, c->i_tok2.ensure(infl_tok_words(max_payload_len, split_frames) * 4));
    HIP_TRY(c, c->i_lit2.ensure(infl_lit_bytes(max_payload_len, split_frames)));
  }
  return WSG_API_OK;
}

int wsg_inflate_split_count(wsg_ctx* c, uint64_t* count) {
  if (!c || !count) return WSG_API_EINVAL;
  *count = 0;
  if (!c->i_split.p) return WSG_API_OK;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipMemcpyAsync(count, c->i_split.p, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return WSG_API_OK;
}

static int ensure_agg_ws(wsg_ctx* c, uint64_t F, uint32_t n_sessions, uint64_t agg_cap);

}  // extern "C" (reopened below)

namespace ws {
uint64_t ctx_alloc_count() { return g_ctx_allocs.load(); }

// The stage context's workspace for a flush's stages (wsg_batcher_reserve_stages):
// inflate over `payload_len` arena bytes, the validator over the same, the aggregator
// into `agg_cap` bytes, `max_frames` frames and `max_sessions` sessions each.
int ctx_reserve_stages(wsg_ctx* c, uint64_t max_frames, uint32_t max_sessions, uint64_t payload_len,
                       uint64_t agg_cap) {
  if (!c) return WSG_API_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  int rc = wsg_reserve_inflate(c, max_frames, max_sessions, payload_len);
  if (!rc) rc = ensure_decode_ws(c, max_frames, max_sessions, payload_len);
  if (rc) return rc;
  HIP_TRY(c, c->v_desc.ensure((max_frames + 1) * sizeof(wsg_frame_desc)));
  return ensure_agg_ws(c, max_frames ? max_frames : 1, max_sessions, agg_cap);
}
}  // namespace ws

extern "C" {

int wsg_reserve(wsg_ctx* c, uint64_t max_frames, uint32_t max_sessions, uint64_t max_wire_len) {
  if (!c) return WSG_API_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  int rc = ensure_decode_ws(c, max_frames, max_sessions, max_wire_len);
  if (rc) return rc;
  return ensure_encode_ws(c, max_frames);
}

uint64_t wsg_decode_payload_bound(uint64_t wire_len, uint64_t n_frames) { return wire_len + 16 * n_frames + 16; }


int wsg_decode_batch_device(wsg_ctx* c, const wsg_decoder_cfg* cfg, const uint8_t* wire, uint64_t wire_len,
                            const uint64_t* frame_off, uint64_t n_frames, const uint32_t* session_first,
                            uint32_t n_sessions, wsg_session_state* state, uint8_t* payload_out,
                            uint64_t payload_cap, wsg_frame_desc* desc_out, wsg_session_result* result_out) {
  if (!c || !cfg) return WSG_API_EINVAL;
  if (n_sessions == 0) return n_frames ? set_err(c, WSG_API_EINVAL, "frames without sessions") : WSG_API_OK;
  if (n_frames >= (1ull << 30)) return set_err(c, WSG_API_ERANGE, "too many frames in one batch (max 2^30 - 1)");
  if (((uintptr_t)wire & 3) || ((uintptr_t)payload_out & 15))
    return set_err(c, WSG_API_EINVAL, "wire must be 4-B aligned and payload_out 16-B aligned");
  if (payload_cap < wire_len + 16 * n_frames)
    return set_err(c, WSG_API_ERANGE, "payload_cap below wsg_decode_payload_bound()");
  HIP_TRY(c, hipSetDevice(c->device));
  int rc = ensure_decode_ws(c, n_frames, n_sessions, wire_len);
  if (rc) return rc;
  DecodeArgs a;
  a.wire = wire;
  a.wire_len = wire_len;
  a.frame_off = frame_off;
  a.n_frames = n_frames;
  a.session_first = session_first;
  a.n_sessions = n_sessions;
  a.client_mode = cfg->client_mode != 0;
  a.allow_ext = cfg->allow_extensions != 0;
  a.validate = cfg->validate_utf8 != 0;
  a.max_payload = cfg->max_payload_len;
  a.state = state;
  a.payload_out = payload_out;
  a.desc = desc_out;
  a.result = result_out;
  a.rec = (FrameRec*)c->rec.p;
  a.vflag = (uint8_t*)c->vflag.p;
  a.slink = (int32_t*)c->slink.p;
  a.edge = (uint32_t*)c->edge.p;
  a.blk_sum = (uint64_t*)c->blk_sum.p;
  a.blk_max = (int32_t*)c->blk_max.p;
  a.chunk_sum = (uint64_t*)c->chunk.p;
  a.chunk_max = (int32_t*)(a.chunk_sum + (n_frames + DBLOCK - 1) / DBLOCK / SCAN_CHUNK + 1);
  a.sess_err = (uint64_t*)c->sess_err.p;
  a.total = (uint64_t*)c->total.p;
  a.pieces = (PieceDesc*)c->pieces.p;
  a.nblk = (uint32_t)((n_frames + DBLOCK - 1) / DBLOCK);
  a.n_pieces = piece_bound(wire_len, n_frames);
  a.validator_only = 0;
  a.in_desc = nullptr;
  a.sparse = (cfg->flags & WSG_CFG_SPARSE) != 0;
  a.fused_scan = a.nblk <= FUSED_SCAN_MAX_BLOCKS && c->fused_scan;
  if (n_frames) {
    timed(c, K_PARSE, [&] { launch_parse(a, c->stream); });
    if (!a.fused_scan) timed(c, K_SCAN, [&] { launch_scan(a, c->stream); });
    timed(c, K_LINK, [&] { launch_link(a, c->stream); });
    timed(c, K_UNMASK, [&] { launch_pieces(a, c->stream, piece_bound(wire_len, n_frames)); });
  }
  timed(c, K_FINAL, [&] { launch_final(a, c->stream); });
  HIP_TRY(c, hipGetLastError());
  return WSG_API_OK;
}

int wsg_validate_batch_device(wsg_ctx* c, const wsg_frame_desc* desc, uint64_t n_frames,
                              const uint32_t* session_first, uint32_t n_sessions, const uint8_t* payload,
                              uint64_t payload_len, wsg_session_state* state, wsg_session_result* result_out) {
  if (!c) return WSG_API_EINVAL;
  if (n_sessions == 0) return n_frames ? set_err(c, WSG_API_EINVAL, "frames without sessions") : WSG_API_OK;
  if (n_frames >= (1ull << 30)) return set_err(c, WSG_API_ERANGE, "too many frames in one batch (max 2^30 - 1)");
  if ((uintptr_t)payload & 3) return set_err(c, WSG_API_EINVAL, "payload must be 4-B aligned");
  HIP_TRY(c, hipSetDevice(c->device));
  int rc = ensure_decode_ws(c, n_frames, n_sessions, payload_len);
  if (rc) return rc;
  HIP_TRY(c, c->v_desc.ensure((n_frames + 1) * sizeof(wsg_frame_desc)));
  DecodeArgs a;
  a.wire = payload;
  a.wire_len = payload_len;
  a.frame_off = nullptr;
  a.n_frames = n_frames;
  a.session_first = session_first;
  a.n_sessions = n_sessions;
  a.client_mode = 0;
  a.allow_ext = 1;
  a.validate = 1;
  a.max_payload = INT64_MAX;
  a.state = state;
  a.payload_out = nullptr;  // validate only: the piece kernel stores nothing
  a.desc = (wsg_frame_desc*)c->v_desc.p;
  a.result = result_out;
  a.rec = (FrameRec*)c->rec.p;
  a.vflag = (uint8_t*)c->vflag.p;
  a.slink = (int32_t*)c->slink.p;
  a.edge = (uint32_t*)c->edge.p;
  a.blk_sum = (uint64_t*)c->blk_sum.p;
  a.blk_max = (int32_t*)c->blk_max.p;
  a.chunk_sum = (uint64_t*)c->chunk.p;
  a.chunk_max = (int32_t*)(a.chunk_sum + (n_frames + DBLOCK - 1) / DBLOCK / SCAN_CHUNK + 1);
  a.sess_err = (uint64_t*)c->sess_err.p;
  a.total = (uint64_t*)c->total.p;
  a.pieces = (PieceDesc*)c->pieces.p;
  a.nblk = (uint32_t)((n_frames + DBLOCK - 1) / DBLOCK);
  a.n_pieces = piece_bound(payload_len, n_frames);
  a.validator_only = 1;
  a.in_desc = desc;
  a.sparse = 0;
  a.fused_scan = a.nblk <= FUSED_SCAN_MAX_BLOCKS && c->fused_scan;
  if (n_frames) {
    timed(c, K_PARSE, [&] { launch_vparse(a, c->stream); });
    if (!a.fused_scan) timed(c, K_SCAN, [&] { launch_scan(a, c->stream); });
    timed(c, K_LINK, [&] { launch_link(a, c->stream); });
    timed(c, K_UNMASK, [&] { launch_vpieces(a, c->stream, a.n_pieces); });
  }
  timed(c, K_FINAL, [&] { launch_final(a, c->stream); });
  HIP_TRY(c, hipGetLastError());
  return WSG_API_OK;
}

int wsg_validate_batch_host(wsg_ctx* c, const wsg_frame_desc* desc, uint64_t n_frames, const uint32_t* session_first,
                            uint32_t n_sessions, const uint8_t* payload, uint64_t payload_len, wsg_session_state* state,
                            wsg_session_result* result_out) {
  if (!c) return WSG_API_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  const uint64_t S = n_sessions;
  HIP_TRY(c, c->h_desc.ensure((n_frames + 1) * sizeof(wsg_frame_desc)));
  HIP_TRY(c, c->h_sf.ensure((S + 1) * sizeof(uint32_t)));
  HIP_TRY(c, c->h_payload.ensure(payload_len + 32));
  HIP_TRY(c, c->h_state.ensure((S + 1) * sizeof(wsg_session_state)));
  HIP_TRY(c, c->h_result.ensure((S + 1) * sizeof(wsg_session_result)));
  hipStream_t s = c->stream;
  if (n_frames) HIP_TRY(c, hipMemcpyAsync(c->h_desc.p, desc, n_frames * sizeof(wsg_frame_desc), hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->h_sf.p, session_first, (S + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  if (payload_len) HIP_TRY(c, hipMemcpyAsync(c->h_payload.p, payload, payload_len, hipMemcpyHostToDevice, s));
  if (S) HIP_TRY(c, hipMemcpyAsync(c->h_state.p, state, S * sizeof(wsg_session_state), hipMemcpyHostToDevice, s));
  int rc = wsg_validate_batch_device(c, (const wsg_frame_desc*)c->h_desc.p, n_frames, (const uint32_t*)c->h_sf.p,
                                     n_sessions, (const uint8_t*)c->h_payload.p, payload_len,
                                     (wsg_session_state*)c->h_state.p, (wsg_session_result*)c->h_result.p);
  if (rc) return rc;
  if (S) {
    HIP_TRY(c, hipMemcpyAsync(result_out, c->h_result.p, S * sizeof(wsg_session_result), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(state, c->h_state.p, S * sizeof(wsg_session_state), hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(c, hipStreamSynchronize(s));
  return WSG_API_OK;
}

// H2D, decode, D2H on the ctx stream, then wait; exactly the payload bytes used
// are copied back.
static int decode_host_impl(wsg_ctx* c, const wsg_decoder_cfg* cfg, const uint8_t* wire, uint64_t wire_len,
                            const uint64_t* frame_off, uint64_t n_frames, const uint32_t* session_first,
                            uint32_t n_sessions, wsg_session_state* state, uint8_t* payload_out, uint64_t payload_cap,
                            wsg_frame_desc* desc_out, wsg_session_result* result_out) {
  if (!c || !cfg) return WSG_API_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  const uint64_t bound = wire_len + 16 * n_frames + 16;
  HIP_TRY(c, c->h_wire.ensure(wire_len + 32));
  HIP_TRY(c, c->h_off.ensure((n_frames + 1) * sizeof(uint64_t)));
  HIP_TRY(c, c->h_sf.ensure(((uint64_t)n_sessions + 1) * sizeof(uint32_t)));
  HIP_TRY(c, c->h_state.ensure(((uint64_t)n_sessions + 1) * sizeof(wsg_session_state)));
  HIP_TRY(c, c->h_payload.ensure(bound));
  HIP_TRY(c, c->h_desc.ensure((n_frames + 1) * sizeof(wsg_frame_desc)));
  HIP_TRY(c, c->h_result.ensure(((uint64_t)n_sessions + 1) * sizeof(wsg_session_result)));
  hipStream_t s = c->stream;
  if (wire_len) HIP_TRY(c, hipMemcpyAsync(c->h_wire.p, wire, wire_len, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->h_off.p, frame_off, (n_frames + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->h_sf.p, session_first, ((uint64_t)n_sessions + 1) * sizeof(uint32_t),
                            hipMemcpyHostToDevice, s));
  if (n_sessions)
    HIP_TRY(c, hipMemcpyAsync(c->h_state.p, state, (uint64_t)n_sessions * sizeof(wsg_session_state),
                              hipMemcpyHostToDevice, s));
  int rc = wsg_decode_batch_device(c, cfg, (const uint8_t*)c->h_wire.p, wire_len, (const uint64_t*)c->h_off.p,
                                   n_frames, (const uint32_t*)c->h_sf.p, n_sessions,
                                   (wsg_session_state*)c->h_state.p, (uint8_t*)c->h_payload.p, bound,
                                   (wsg_frame_desc*)c->h_desc.p, (wsg_session_result*)c->h_result.p);
  if (rc) return rc;
  if (n_frames) {
    uint64_t total;
    HIP_TRY(c, hipMemcpyAsync(&total, c->total.p, sizeof total, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    if (total > payload_cap)
      return set_err(c, WSG_API_ERANGE, "payload_cap %llu < %llu", (unsigned long long)payload_cap,
                     (unsigned long long)total);
    if (total) HIP_TRY(c, hipMemcpyAsync(payload_out, c->h_payload.p, total, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(desc_out, c->h_desc.p, n_frames * sizeof(wsg_frame_desc), hipMemcpyDeviceToHost, s));
  }
  if (n_sessions) {
    HIP_TRY(c, hipMemcpyAsync(result_out, c->h_result.p, (uint64_t)n_sessions * sizeof(wsg_session_result),
                              hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(state, c->h_state.p, (uint64_t)n_sessions * sizeof(wsg_session_state),
                              hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(c, hipStreamSynchronize(s));
  return WSG_API_OK;
}

int wsg_decode_batch_host(wsg_ctx* c, const wsg_decoder_cfg* cfg, const uint8_t* wire, uint64_t wire_len,
                          const uint64_t* frame_off, uint64_t n_frames, const uint32_t* session_first,
                          uint32_t n_sessions, wsg_session_state* state, uint8_t* payload_out, uint64_t payload_cap,
                          wsg_frame_desc* desc_out, wsg_session_result* result_out) {
  return decode_host_impl(c, cfg, wire, wire_len, frame_off, n_frames, session_first, n_sessions, state, payload_out,
                          payload_cap, desc_out, result_out);
}

// Pipelined host batch: uploads on s_in, kernels on the ctx stream, downloads on
// s_out (each copy direction needs its own stream to overlap), two staging slots
// used alternately.  Event edges:
//   slot reuse   upload(i+2) waits kernels(i); kernels(i+2) waits downloads(i)
//   carry state  state upload(i+1) waits state download(i), so batches that share
//                sessions (and one host state array) chain correctly while the
//                wire upload of batch i+1 still overlaps the kernels of batch i
int wsg_decode_batch_host_async(wsg_ctx* c, const wsg_decoder_cfg* cfg, const uint8_t* wire, uint64_t wire_len,
                                const uint64_t* frame_off, uint64_t n_frames, const uint32_t* session_first,
                                uint32_t n_sessions, wsg_session_state* state, uint8_t* payload_out,
                                uint64_t payload_cap, wsg_frame_desc* desc_out, wsg_session_result* result_out) {
  if (!c || !cfg) return WSG_API_EINVAL;
  if (n_frames && payload_cap < wire_len + 16 * n_frames)
    return set_err(c, WSG_API_ERANGE, "payload_cap below wire_len + 16 * n_frames");
  HIP_TRY(c, hipSetDevice(c->device));
  if (!c->s_in) HIP_TRY(c, hipStreamCreateWithFlags(&c->s_in, hipStreamNonBlocking));
  if (!c->s_out) HIP_TRY(c, hipStreamCreateWithFlags(&c->s_out, hipStreamNonBlocking));
  HostSlot& h = c->slot[c->next_slot];
  c->next_slot ^= 1;
  hipEvent_t* evs[] = {&h.ev_in, &h.ev_k, &h.ev_state, &h.ev_out};
  for (hipEvent_t* e : evs)
    if (!*e) HIP_TRY(c, hipEventCreateWithFlags(e, hipEventDisableTiming));
  const uint64_t bound = wire_len + 16 * n_frames + 16;
  if (h.used) {  // buffers may be re-allocated below: drain this slot's last batch first
    HIP_TRY(c, hipEventSynchronize(h.ev_out));
  }
  HIP_TRY(c, h.wire.ensure(wire_len + 32));
  HIP_TRY(c, h.off.ensure((n_frames + 1) * sizeof(uint64_t)));
  HIP_TRY(c, h.sf.ensure(((uint64_t)n_sessions + 1) * sizeof(uint32_t)));
  HIP_TRY(c, h.state.ensure(((uint64_t)n_sessions + 1) * sizeof(wsg_session_state)));
  HIP_TRY(c, h.payload.ensure(bound));
  HIP_TRY(c, h.desc.ensure((n_frames + 1) * sizeof(wsg_frame_desc)));
  HIP_TRY(c, h.result.ensure(((uint64_t)n_sessions + 1) * sizeof(wsg_session_result)));
  // uploads
  if (wire_len) HIP_TRY(c, hipMemcpyAsync(h.wire.p, wire, wire_len, hipMemcpyHostToDevice, c->s_in));
  HIP_TRY(c, hipMemcpyAsync(h.off.p, frame_off, (n_frames + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, c->s_in));
  HIP_TRY(c, hipMemcpyAsync(h.sf.p, session_first, ((uint64_t)n_sessions + 1) * sizeof(uint32_t),
                            hipMemcpyHostToDevice, c->s_in));
  if (c->ev_prev_state) HIP_TRY(c, hipStreamWaitEvent(c->s_in, c->ev_prev_state, 0));
  if (n_sessions)
    HIP_TRY(c, hipMemcpyAsync(h.state.p, state, (uint64_t)n_sessions * sizeof(wsg_session_state),
                              hipMemcpyHostToDevice, c->s_in));
  HIP_TRY(c, hipEventRecord(h.ev_in, c->s_in));
  // kernels
  HIP_TRY(c, hipStreamWaitEvent(c->stream, h.ev_in, 0));
  int rc = wsg_decode_batch_device(c, cfg, (const uint8_t*)h.wire.p, wire_len, (const uint64_t*)h.off.p, n_frames,
                                   (const uint32_t*)h.sf.p, n_sessions, (wsg_session_state*)h.state.p,
                                   (uint8_t*)h.payload.p, bound, (wsg_frame_desc*)h.desc.p,
                                   (wsg_session_result*)h.result.p);
  if (rc) return rc;
  HIP_TRY(c, hipEventRecord(h.ev_k, c->stream));
  // downloads: the carry state first (the next batch's state upload waits for it)
  HIP_TRY(c, hipStreamWaitEvent(c->s_out, h.ev_k, 0));
  if (n_sessions)
    HIP_TRY(c, hipMemcpyAsync(state, h.state.p, (uint64_t)n_sessions * sizeof(wsg_session_state),
                              hipMemcpyDeviceToHost, c->s_out));
  HIP_TRY(c, hipEventRecord(h.ev_state, c->s_out));
  c->ev_prev_state = h.ev_state;
  if (n_sessions)
    HIP_TRY(c, hipMemcpyAsync(result_out, h.result.p, (uint64_t)n_sessions * sizeof(wsg_session_result),
                              hipMemcpyDeviceToHost, c->s_out));
  if (n_frames) {
    HIP_TRY(c, hipMemcpyAsync(desc_out, h.desc.p, n_frames * sizeof(wsg_frame_desc), hipMemcpyDeviceToHost, c->s_out));
    if (payload_out)
      HIP_TRY(c, hipMemcpyAsync(payload_out, h.payload.p, wire_len + 16 * n_frames, hipMemcpyDeviceToHost, c->s_out));
  }
  c->last_async_payload = (uint8_t*)h.payload.p;
  HIP_TRY(c, hipEventRecord(h.ev_out, c->s_out));
  h.used = true;
  return WSG_API_OK;
}

// FrameDecoder.available(session, byte[], off, len), FrameDecoder.java:357-401,
// with the JVM's int/long arithmetic (the u64 branch can wrap).
int64_t wsg_frame_available(const uint8_t* buf, uint64_t len_u, int32_t* err, int64_t* detail, int64_t* detail2) {
  if (err) *err = 0;
  const int64_t len = (int64_t)len_u;
  int32_t need = 2;
  if (len < need) return 0;
  if (buf[1] & 0x80) {
    need += 4;
    if (len < need) return 0;
  }
  int64_t plen = buf[1] & 0x7f;
  if (plen < 126) {
    need += (int32_t)plen;
  } else if (plen == 126) {
    need += 2;
    if (len < need) return 0;
    need += (int32_t)(((uint32_t)buf[2] << 8) | buf[3]);
  } else {
    need += 8;
    if (len < need) return 0;
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | buf[2 + i];
    plen = (int64_t)v;
    if (plen < 0) {
      if (err) *err = WSG_E_NEG_LEN;
      if (detail) *detail = plen;
      if (detail2) *detail2 = 0;
      return -1;
    }
    if ((int64_t)((uint64_t)plen + (uint64_t)(int64_t)need) > (int64_t)0x7fffffff) {
      if (err) *err = WSG_E_EXT_LEN;
      if (detail) *detail = plen;
      if (detail2) *detail2 = (int64_t)0x7fffffff - need;
      return -1;
    }
    need = (int32_t)(uint32_t)((uint64_t)(int64_t)need + (uint64_t)plen);
  }
  return len > need ? need : len;
}

int32_t wsg_check_header(const wsg_decoder_cfg* cfg, int fragmentation, const uint8_t* buf, uint64_t len,
                         int64_t* detail) {
  Header h;
  if (detail) *detail = 0;
  if (!parse_header(buf, len, h)) return WSG_E_BATCH;
  uint32_t e = rules_pre(h, cfg->client_mode, cfg->allow_extensions);
  if (!e) e = rules_frag(h.opcode, fragmentation != 0);
  if (!e) e = rules_post(h, cfg->max_payload_len);
  if (detail) {
    switch (e) {
      case WSG_E_OPCODE: *detail = h.opcode; break;
      case WSG_E_RSV: *detail = h.rsv; break;
      case WSG_E_CONTROL_LEN:
      case WSG_E_CLOSE_LEN: *detail = h.len7; break;
      case WSG_E_TOO_LONG: *detail = cfg->max_payload_len; break;
      default: break;
    }
  }
  return (int32_t)e;
}

uint64_t wsg_encoded_length(uint32_t len, int client_mode) {
  uint64_t n = len;
  if (len > 0xffffu) n += 8;
  else if (len > 125u) n += 2;
  if (client_mode) n += 4;
  return n + 2;
}

int wsg_encode_batch_device(wsg_ctx* c, int client_mode, const uint8_t* payload, uint64_t payload_len,
                            const wsg_encode_frame* frames, uint64_t n_frames, const uint32_t* session_first,
                            uint32_t n_sessions, uint8_t* closed, uint8_t* wire_out, uint64_t wire_cap,
                            uint64_t* wire_off) {
  if (!c) return WSG_API_EINVAL;
  if (n_sessions == 0) return n_frames ? set_err(c, WSG_API_EINVAL, "frames without sessions") : WSG_API_OK;
  if (n_frames >= 0x7fffffffull) return set_err(c, WSG_API_ERANGE, "too many frames in one batch");
  if ((uintptr_t)wire_out & 15) return set_err(c, WSG_API_EINVAL, "wire_out must be 16-B aligned");
  HIP_TRY(c, hipSetDevice(c->device));
  int rc = ensure_encode_ws(c, n_frames);
  if (rc) return rc;
  EncodeArgs a;
  a.client_mode = client_mode != 0;
  a.payload = payload;
  a.payload_len = payload_len;
  a.frames = frames;
  a.n_frames = n_frames;
  a.session_first = session_first;
  a.n_sessions = n_sessions;
  a.closed = closed;
  a.wire_out = wire_out;
  a.wire_cap = wire_cap;
  a.wire_off = wire_off;
  a.sess = (uint32_t*)c->esess.p;
  a.blk_sum = (uint64_t*)c->blk_sum.p;
  a.blk_max = (int32_t*)c->blk_max.p;
  a.last_close = (int32_t*)c->elast_close.p;
  a.nblk = (uint32_t)((n_frames + BLOCK - 1) / BLOCK);
  // pieces of wire_out: bounded by the caller's capacity (the total is only known on the device)
  a.n_pieces = wire_cap / PIECE + 1;
  a.n_idx = a.n_pieces / 64 + 2;
  if (n_frames) {
    HIP_TRY(c, c->epieces.ensure((a.n_pieces + ENC_PIECES_PER_WAVE) * sizeof(PieceDesc)));
    HIP_TRY(c, c->epidx.ensure(a.n_idx * sizeof(uint32_t)));
  }
  a.pieces = (PieceDesc*)c->epieces.p;
  a.pidx = (uint32_t*)c->epidx.p;
  if (n_frames) {
    timed(c, K_ENC_LEN, [&] { launch_enc_len(a, c->stream); });
    timed(c, K_ENC_SCAN, [&] { launch_enc_scan(a, c->stream); });
    timed(c, K_ENC_DESC, [&] { launch_enc_desc(a, c->stream); });
    timed(c, K_ENC_EMIT, [&] { launch_enc_pieces(a, c->stream); });
    timed(c, K_ENC_FINAL, [&] { launch_enc_final(a, c->stream); });
  } else {
    HIP_TRY(c, hipMemsetAsync(wire_off, 0, sizeof(uint64_t), c->stream));
  }
  HIP_TRY(c, hipGetLastError());
  return WSG_API_OK;
}

int wsg_encode_batch_host(wsg_ctx* c, int client_mode, const uint8_t* payload, uint64_t payload_len,
                          const wsg_encode_frame* frames, uint64_t n_frames, const uint32_t* session_first,
                          uint32_t n_sessions, uint8_t* closed, uint8_t* wire_out, uint64_t wire_cap,
                          uint64_t* wire_off) {
  if (!c) return WSG_API_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  uint64_t need = 0;
  for (uint64_t k = 0; k < n_frames; ++k) need += wsg_encoded_length(frames[k].payload_len, client_mode);
  HIP_TRY(c, c->h_payload.ensure(payload_len + 32));
  HIP_TRY(c, c->h_frames.ensure((n_frames + 1) * sizeof(wsg_encode_frame)));
  HIP_TRY(c, c->h_sf.ensure(((uint64_t)n_sessions + 1) * sizeof(uint32_t)));
  HIP_TRY(c, c->h_closed.ensure((uint64_t)n_sessions + 1));
  HIP_TRY(c, c->h_wire.ensure(need + 32));
  HIP_TRY(c, c->h_wire_off.ensure((n_frames + 1) * sizeof(uint64_t)));
  hipStream_t s = c->stream;
  if (payload_len) HIP_TRY(c, hipMemcpyAsync(c->h_payload.p, payload, payload_len, hipMemcpyHostToDevice, s));
  if (n_frames)
    HIP_TRY(c, hipMemcpyAsync(c->h_frames.p, frames, n_frames * sizeof(wsg_encode_frame), hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->h_sf.p, session_first, ((uint64_t)n_sessions + 1) * sizeof(uint32_t),
                            hipMemcpyHostToDevice, s));
  if (n_sessions) HIP_TRY(c, hipMemcpyAsync(c->h_closed.p, closed, n_sessions, hipMemcpyHostToDevice, s));
  int rc = wsg_encode_batch_device(c, client_mode, (const uint8_t*)c->h_payload.p, payload_len,
                                   (const wsg_encode_frame*)c->h_frames.p, n_frames, (const uint32_t*)c->h_sf.p,
                                   n_sessions, (uint8_t*)c->h_closed.p, (uint8_t*)c->h_wire.p, need + 32,
                                   (uint64_t*)c->h_wire_off.p);
  if (rc) return rc;
  HIP_TRY(c, hipMemcpyAsync(wire_off, c->h_wire_off.p, (n_frames + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  const uint64_t total = wire_off[n_frames];
  if (total > wire_cap) return set_err(c, WSG_API_ERANGE, "wire_cap too small");
  if (total) HIP_TRY(c, hipMemcpyAsync(wire_out, c->h_wire.p, total, hipMemcpyDeviceToHost, s));
  if (n_sessions) HIP_TRY(c, hipMemcpyAsync(closed, c->h_closed.p, n_sessions, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  return WSG_API_OK;
}

// the aggregator's workspace for F frames, S sessions and agg_cap output bytes
static int ensure_agg_ws(wsg_ctx* c, uint64_t F, uint32_t n_sessions, uint64_t agg_cap) {
  const uint64_t nblk = (F + ABLOCK - 1) / ABLOCK;
  HIP_TRY(c, c->a_code.ensure(F * 2 * sizeof(uint32_t)));
  HIP_TRY(c, c->a_last.ensure(F * 2 * sizeof(int32_t)));
  HIP_TRY(c, c->a_pl.ensure(F * sizeof(uint64_t)));
  HIP_TRY(c, c->a_cl.ensure(F * sizeof(uint64_t) + sizeof(uint64_t)));
  HIP_TRY(c, c->a_blk.ensure(nblk * (4 * sizeof(uint64_t) + 2 * sizeof(int32_t))));
  HIP_TRY(c, c->a_sess_err.ensure((uint64_t)(n_sessions ? n_sessions : 1) * sizeof(uint64_t), 0xff, c->stream));
  HIP_TRY(c, c->a_pieces.ensure((agg_cap / PIECE + 2 * F + 2 + 1) * sizeof(PieceDesc)));
  return WSG_API_OK;
}

int wsg_aggregate_batch_device(wsg_ctx* c, int64_t max_aggregated_len, const wsg_frame_desc* desc,
                               uint64_t n_frames, const uint32_t* session_first, uint32_t n_sessions,
                               const wsg_session_result* dec_result, const uint8_t* payload, uint64_t payload_len,
                               wsg_agg_state* state, uint8_t* agg_out, uint64_t agg_cap, wsg_frame_desc* out_desc,
                               wsg_session_result* out_result, uint64_t* agg_total) {
  if (!c) return WSG_API_EINVAL;
  if (n_sessions == 0) return n_frames ? set_err(c, WSG_API_EINVAL, "frames without sessions") : WSG_API_OK;
  if (n_frames >= (1ull << 30)) return set_err(c, WSG_API_ERANGE, "too many frames in one batch (max 2^30 - 1)");
  if (((uintptr_t)payload & 15) || ((uintptr_t)agg_out & 15))
    return set_err(c, WSG_API_EINVAL, "payload and agg_out must be 16-B aligned");
  HIP_TRY(c, hipSetDevice(c->device));
  const uint64_t F = n_frames ? n_frames : 1;
  const uint64_t nblk = (F + ABLOCK - 1) / ABLOCK;
  AggArgs a;
  a.max_len = max_aggregated_len;
  a.desc = desc;
  a.n_frames = n_frames;
  a.session_first = session_first;
  a.n_sessions = n_sessions;
  a.dec_result = dec_result;
  a.payload = payload;
  a.state = state;
  a.agg_out = agg_out;
  a.agg_cap = agg_cap;
  a.out_desc = out_desc;
  a.out_result = out_result;
  a.agg_total = agg_total;
  a.nblk = (uint32_t)((n_frames + ABLOCK - 1) / ABLOCK);
  // gather units: a member of m bytes has ceil((m + 15) / 1 KiB); those holding bytes below
  // agg_cap number at most agg_cap / 1 KiB + 2 per member before them
  a.n_pieces = agg_cap / PIECE + 2 * F + 2;
  a.fold_max = std::min(c->agg_fold, agg_fold_bound());
  {
    const int rc = ensure_agg_ws(c, F, n_sessions, agg_cap);
    if (rc) return rc;
  }
  a.code = (uint32_t*)c->a_code.p;
  a.sess = a.code + F;
  a.last = (int32_t*)c->a_last.p;
  a.pl = (uint64_t*)c->a_pl.p;
  a.cl = (uint64_t*)c->a_cl.p;
  a.n_units = a.cl + F;
  a.blk_sum = (uint64_t*)c->a_blk.p;
  a.blk_cnt = a.blk_sum + nblk;
  a.pre_sum = a.blk_cnt + nblk;
  a.pre_cnt = a.pre_sum + nblk;
  a.blk_max = (int32_t*)(a.pre_cnt + nblk);
  a.sess_err = (uint64_t*)c->a_sess_err.p;
  a.pieces = (PieceDesc*)c->a_pieces.p;
  if (!n_frames) HIP_TRY(c, hipMemsetAsync(agg_total, 0, sizeof(uint64_t), c->stream));
  timed(c, K_AGG, [&] { launch_agg_plan(a, c->stream); });
  timed(c, K_AGG_GATHER, [&] { launch_agg_gather(a, c->stream, payload_len, c->agg_units, c->agg_grid); });
  HIP_TRY(c, hipGetLastError());
  return WSG_API_OK;
}

int wsg_aggregate_batch_host(wsg_ctx* c, int64_t max_aggregated_len, const wsg_frame_desc* desc, uint64_t n_frames,
                             const uint32_t* session_first, uint32_t n_sessions, const wsg_session_result* dec_result,
                             const uint8_t* payload, uint64_t payload_len, wsg_agg_state* state, uint8_t* agg_out,
                             uint64_t agg_cap, wsg_frame_desc* out_desc, wsg_session_result* out_result,
                             uint64_t* agg_total) {
  if (!c || !agg_total) return WSG_API_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  const uint64_t S = n_sessions;
  DevBuf d_desc, d_sf, d_res, d_pay, d_state, d_agg, d_odesc, d_ores, d_tot;
  struct Guard {
    DevBuf* b[9];
    ~Guard() { for (DevBuf* x : b) x->release(); }
  } g{{&d_desc, &d_sf, &d_res, &d_pay, &d_state, &d_agg, &d_odesc, &d_ores, &d_tot}};
  HIP_TRY(c, d_desc.ensure((n_frames + 1) * sizeof(wsg_frame_desc)));
  HIP_TRY(c, d_sf.ensure((S + 1) * sizeof(uint32_t)));
  HIP_TRY(c, d_res.ensure((S + 1) * sizeof(wsg_session_result)));
  HIP_TRY(c, d_pay.ensure(payload_len + 32));
  HIP_TRY(c, d_state.ensure((S + 1) * sizeof(wsg_agg_state)));
  HIP_TRY(c, d_agg.ensure(agg_cap + 32));
  HIP_TRY(c, d_odesc.ensure((n_frames + S + 1) * sizeof(wsg_frame_desc)));
  HIP_TRY(c, d_ores.ensure((S + 1) * sizeof(wsg_session_result)));
  HIP_TRY(c, d_tot.ensure(sizeof(uint64_t)));
  hipStream_t s = c->stream;
  if (n_frames) HIP_TRY(c, hipMemcpyAsync(d_desc.p, desc, n_frames * sizeof(wsg_frame_desc), hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(d_sf.p, session_first, (S + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  if (S) {
    HIP_TRY(c, hipMemcpyAsync(d_res.p, dec_result, S * sizeof(wsg_session_result), hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(d_state.p, state, S * sizeof(wsg_agg_state), hipMemcpyHostToDevice, s));
  }
  if (payload_len) HIP_TRY(c, hipMemcpyAsync(d_pay.p, payload, payload_len, hipMemcpyHostToDevice, s));
  int rc = wsg_aggregate_batch_device(c, max_aggregated_len, (const wsg_frame_desc*)d_desc.p, n_frames,
                                      (const uint32_t*)d_sf.p, n_sessions, (const wsg_session_result*)d_res.p,
                                      (const uint8_t*)d_pay.p, payload_len, (wsg_agg_state*)d_state.p,
                                      (uint8_t*)d_agg.p, agg_cap, (wsg_frame_desc*)d_odesc.p,
                                      (wsg_session_result*)d_ores.p, (uint64_t*)d_tot.p);
  if (rc) return rc;
  HIP_TRY(c, hipMemcpyAsync(agg_total, d_tot.p, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  const uint64_t used = *agg_total < agg_cap ? *agg_total : agg_cap;
  if (used) HIP_TRY(c, hipMemcpyAsync(agg_out, d_agg.p, used, hipMemcpyDeviceToHost, s));
  if (n_frames + S)
    HIP_TRY(c, hipMemcpyAsync(out_desc, d_odesc.p, (n_frames + S) * sizeof(wsg_frame_desc), hipMemcpyDeviceToHost, s));
  if (S) {
    HIP_TRY(c, hipMemcpyAsync(out_result, d_ores.p, S * sizeof(wsg_session_result), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(state, d_state.p, S * sizeof(wsg_agg_state), hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(c, hipStreamSynchronize(s));
  if (*agg_total > agg_cap) return set_err(c, WSG_API_ERANGE, "agg_cap %llu < %llu", (unsigned long long)agg_cap,
                                           (unsigned long long)*agg_total);
  return WSG_API_OK;
}

}  // extern "C" (reopened below)

// The arguments of an inflate launch sequence with no pre-decode attached.
static InflArgs infl_args(wsg_ctx* c, int no_context, const wsg_frame_desc* desc, uint64_t n_frames,
                          const uint32_t* session_first, uint32_t n_sessions, const uint8_t* payload,
                          uint64_t payload_len, wsg_inflate_state* state, uint8_t* window, uint8_t* out,
                          const uint64_t* out_off, wsg_frame_desc* out_desc, wsg_session_result* out_result,
                          uint32_t* replay_from) {
  InflArgs a;
  a.no_context = no_context != 0;
  a.desc = desc;
  a.n_frames = n_frames;
  a.session_first = session_first;
  a.n_sessions = n_sessions;
  a.payload = payload;
  a.payload_len = payload_len;
  a.state = state;
  a.window = window;
  a.out = out;
  a.out_off = out_off;
  a.out_desc = out_desc;
  a.result = out_result;
  a.replay_from = replay_from;
  a.tok = nullptr;
  a.lit = nullptr;
  a.lit_len = 0;
  a.tstat = nullptr;
  a.tab = nullptr;
  a.n_tab = 0;
  a.tab_cnt = nullptr;
  a.n_lanes = 0;
  a.fast_done = nullptr;
  a.order = nullptr;
  a.ord_cnt = nullptr;
  a.tok_lds = c->infl_lds;
  a.split = 0;
  a.split_cnt = nullptr;
  a.tok2 = nullptr;
  a.lit2 = nullptr;
  a.tmap = nullptr;
  return a;
}

// The pre-decode's workspace on c for a list of n_frames frames over payload_len bytes.
static int infl_tok_args(wsg_ctx* c, InflArgs& a, uint64_t n_frames, uint64_t payload_len) {
  const uint32_t lanes = (uint32_t)infl_lane_count(c, n_frames);
  const int rc = ensure_inflate_ws(c, n_frames, payload_len);
  if (rc) return rc;
  a.tok = (uint32_t*)c->i_tok.p;
  a.lit = (uint8_t*)c->i_lit.p;
  a.lit_len = infl_lit_bytes(payload_len, n_frames);
  a.tstat = (InflTokStat*)c->i_stat.p;
  a.tab = (uint8_t*)c->i_tab.p;
  a.n_tab = lanes < c->infl_tabs ? lanes : c->infl_tabs;
  a.tab_cnt = (uint32_t*)c->i_tabcnt.p;
  a.n_lanes = lanes;
  a.split = infl_pairs(c, n_frames) ? 1 : 0;
  a.tok2 = (uint32_t*)c->i_tok2.p;
  a.lit2 = (uint8_t*)c->i_lit2.p;
  a.split_cnt = (unsigned long long*)c->i_split.p;
  a.order = nullptr;
  a.ord_cnt = nullptr;
  if (c->infl_order) {
    a.order = (uint32_t*)c->i_ord.p;
    a.ord_cnt = a.order + n_frames;
  }
  return WSG_API_OK;
}

namespace ws {
int inflate_tok_phase(wsg_ctx* c, const wsg_frame_desc* desc, uint64_t n_frames, const uint32_t* session_first,
                      uint32_t n_sessions, const uint8_t* payload, uint64_t payload_len) {
  if (!c) return WSG_API_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  c->tok_frames = n_frames;
  c->tok_payload_len = payload_len;
  if (!n_frames || !c->infl_tokens) return WSG_API_OK;
  InflArgs a = infl_args(c, 0, desc, n_frames, session_first, n_sessions, payload, payload_len, nullptr, nullptr,
                         nullptr, nullptr, nullptr, nullptr, nullptr);
  const int rc = infl_tok_args(c, a, n_frames, payload_len);
  if (rc) return rc;
  HIP_TRY(c, hipMemsetAsync(c->i_tabcnt.p, 0, sizeof(uint32_t), c->stream));
  timed(c, K_INFL_TOK, [&] { launch_infl_tok(a, c->stream); });
  HIP_TRY(c, hipGetLastError());
  return WSG_API_OK;
}

int inflate_replay_phase(wsg_ctx* c, wsg_ctx* tokc, const uint32_t* tmap, int no_context, const wsg_frame_desc* desc,
                         uint64_t n_frames, const uint32_t* session_first, uint32_t n_sessions, const uint8_t* payload,
                         uint64_t payload_len, wsg_inflate_state* state, uint8_t* window, uint8_t* out,
                         const uint64_t* out_off, wsg_frame_desc* out_desc, wsg_session_result* out_result,
                         uint32_t* replay_from) {
  if (!c || !tokc) return WSG_API_EINVAL;
  if (n_sessions == 0) return n_frames ? set_err(c, WSG_API_EINVAL, "frames without sessions") : WSG_API_OK;
  HIP_TRY(c, hipSetDevice(c->device));
  InflArgs a = infl_args(c, no_context, desc, n_frames, session_first, n_sessions, payload, payload_len, state, window,
                         out, out_off, out_desc, out_result, replay_from);
  if (tokc->infl_tokens && tokc->tok_frames && n_frames) {  // the pre-decode tokc ran (its layout)
    a.tok = (uint32_t*)tokc->i_tok.p;
    a.lit = (uint8_t*)tokc->i_lit.p;
    a.lit_len = infl_lit_bytes(tokc->tok_payload_len, tokc->tok_frames);
    a.tstat = (InflTokStat*)tokc->i_stat.p;
    a.tmap = tmap;
    if (c->infl_fast) {
      HIP_TRY(c, c->i_fast.ensure(n_sessions));
      a.fast_done = (uint8_t*)c->i_fast.p;
      timed(c, K_INFL_FAST, [&] { launch_infl_fast(a, c->stream); });
    }
  }
  if (!(c->infl_fast == 2 && a.fast_done)) timed(c, K_INFLATE, [&] { launch_inflate(a, c->stream); });
  HIP_TRY(c, hipGetLastError());
  return WSG_API_OK;
}
}  // namespace ws

namespace ws {
// ---------------------------------------------------------------- permessage-deflate encode
static inline uint64_t r16h(uint64_t x) { return (x + 15) & ~15ull; }

void deflate_bounds_add(DeflBounds& b, uint32_t len) {
  b.tot[0] += len;
  b.tot[1] += r16h(len + ((len + 7) >> 3) + ((len + 63) >> 6) + 15);   // ZlibEncoder.deflateBound (java_bound)
  b.tot[2] += (len + 3) & ~3u;
  b.tot[3] += (len > 2 ? (len - 2 + DEFL_CH - 1) / DEFL_CH : 0) + 1;
  b.tot[4] += defl_blk_cap(len);
}
void deflate_bounds_session(DeflBounds& b) { b.tot[0] += r16h(DEFL_HIST + DEFL_PAD) + 16; }

// wsg_deflate_batch_device; with `bounds` the workspace is sized from them and nothing is read
// back (the launches stay asynchronous), else from the plan's totals (one synchronisation)
int deflate_launch(wsg_ctx* c, int level, int no_context, const wsg_frame_desc* desc, uint64_t n_frames,
                   const uint32_t* session_first, uint32_t n_sessions, const uint8_t* payload,
                   wsg_deflate_state* state, uint8_t* session_mem, uint8_t* out, uint64_t out_cap,
                   wsg_frame_desc* out_desc, const DeflBounds* bounds, uint64_t* out_total) {
  if (!c) return WSG_API_EINVAL;
  if (level < 0 || level > 9) return set_err(c, WSG_API_EINVAL, "compression level is out of range");
  if (out_total) *out_total = 0;
  if (n_sessions == 0) return n_frames ? set_err(c, WSG_API_EINVAL, "frames without sessions") : WSG_API_OK;
  if (n_frames >= (1ull << 31)) return set_err(c, WSG_API_ERANGE, "too many frames in one batch (max 2^31 - 1)");
  HIP_TRY(c, hipSetDevice(c->device));
  const uint64_t S = n_sessions, F = n_frames ? n_frames : 1;
  HIP_TRY(c, c->d_flags.ensure(F * sizeof(uint32_t)));
  HIP_TRY(c, c->d_fout.ensure(F * sizeof(uint64_t)));
  HIP_TRY(c, c->d_fsym.ensure(F * sizeof(uint64_t)));
  HIP_TRY(c, c->d_ff.ensure(F * sizeof(DeflFrame)));
  HIP_TRY(c, c->d_fs.ensure(S * sizeof(DeflSess)));
  HIP_TRY(c, c->d_sums.ensure(5 * (S + 1) * sizeof(uint64_t)));
  HIP_TRY(c, c->d_ftail.ensure(F));
  DeflArgs a{};
  a.level = level;
  a.no_context = no_context ? 1 : 0;
  a.serial = (level >= 1 && level <= 3) || (level >= 4 && c->defl_serial) ? 1 : 0;
  a.match_lds = c->defl_lds;
  a.desc = desc;
  a.n_frames = n_frames;
  a.session_first = session_first;
  a.n_sessions = n_sessions;
  a.payload = payload;
  a.state = state;
  a.smem = session_mem;
  a.out = out;
  a.out_cap = out_cap;
  a.out_desc = out_desc;
  a.fflags = (uint32_t*)c->d_flags.p;
  a.fout = (uint64_t*)c->d_fout.p;
  a.fsym = (uint64_t*)c->d_fsym.p;
  a.ff = (DeflFrame*)c->d_ff.p;
  a.fs = (DeflSess*)c->d_fs.p;
  a.sums = (uint64_t*)c->d_sums.p;
  a.ftail = (uint8_t*)c->d_ftail.p;
  timed(c, K_DEFL_PLAN, [&] { launch_defl_plan(a, c->stream); });
  uint64_t tot[5];
  if (bounds) {
    for (int i = 0; i < 5; i++) tot[i] = bounds->tot[i];
  } else {  // the regions' totals decide the workspace: read them back
    for (int i = 0; i < 5; i++)
      HIP_TRY(c, hipMemcpyAsync(&tot[i], a.sums + (uint64_t)i * (S + 1) + S, sizeof(uint64_t), hipMemcpyDeviceToHost,
                                c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  if (tot[1] > out_cap)
    return set_err(c, WSG_API_ERANGE, "out_cap %llu below the batch's %llu slot bytes", (unsigned long long)out_cap,
                   (unsigned long long)tot[1]);
  if (out_total) *out_total = tot[1];
  const size_t twb = defl_treework_bytes();
  if (a.serial) {
    HIP_TRY(c, c->d_ssym.ensure(S * zd_lit_bufsize() * sizeof(uint32_t)));
    HIP_TRY(c, c->d_tw.ensure(S * twb));
    a.ssym = (uint32_t*)c->d_ssym.p;
    a.tw = c->d_tw.p;
    timed(c, K_DEFL_SERIAL, [&] { launch_defl_serial(a, c->stream); });
    return WSG_API_OK;
  }
  // a parse lane a frame (the lanes are latency-bound: 65536 of them were one wave a SIMD)
  a.n_lanes = (uint32_t)(F < (1u << 22) ? F : (1u << 22));
  if (level >= 4) {
    HIP_TRY(c, c->d_S.ensure(tot[0] + 64));
    HIP_TRY(c, c->d_link.ensure((tot[0] + 64) * sizeof(uint16_t)));
    HIP_TRY(c, c->d_res.ensure((tot[0] + 64) * 2 * sizeof(uint32_t)));
    HIP_TRY(c, c->d_tres.ensure(F * DEFL_TAILN * 2 * sizeof(uint32_t)));
    HIP_TRY(c, c->d_strips.ensure(F * 2 * zd_strip()));
    HIP_TRY(c, c->d_chunks.ensure((tot[3] + 1) * sizeof(uint64_t)));
    HIP_TRY(c, c->d_sym.ensure((tot[2] + 4) * sizeof(uint32_t)));
    HIP_TRY(c, c->d_blocks.ensure((tot[4] + 1) * sizeof(DeflBlock)));
    a.S = (uint8_t*)c->d_S.p;
    a.link = (uint16_t*)c->d_link.p;
    a.res = (uint32_t*)c->d_res.p;
    a.tres = (uint32_t*)c->d_tres.p;
    a.strips = (uint8_t*)c->d_strips.p;
    a.chunks = (uint64_t*)c->d_chunks.p;
    a.chunk_cap = tot[3];
    a.sym = (uint32_t*)c->d_sym.p;
    a.blocks = (DeflBlock*)c->d_blocks.p;
    timed(c, K_DEFL_PREP, [&] { launch_defl_prep(a, c->stream); });
    timed(c, K_DEFL_LINKS, [&] { launch_defl_links(a, c->stream); });
    if (tot[3]) {
      if (a.match_lds) timed(c, K_DEFL_MATCH_LDS, [&] { launch_defl_match_lds(a, c->stream); });
      timed(c, K_DEFL_MATCH, [&] { launch_defl_match(a, c->stream); });
    }
  }
  timed(c, K_DEFL_PARSE, [&] { launch_defl_parse(a, c->stream); });
  if (level >= 4) {
    timed(c, K_DEFL_HIST, [&] { launch_defl_hist(a, c->stream, tot[4]); });
    timed(c, K_DEFL_TREES, [&] { launch_defl_trees(a, c->stream, tot[4]); });
  }
  timed(c, K_DEFL_EMIT, [&] { launch_defl_emit(a, c->stream); });
  timed(c, K_DEFL_FINAL, [&] { launch_defl_final(a, c->stream); });
  HIP_TRY(c, hipGetLastError());
  return WSG_API_OK;
}
}  // namespace ws

extern "C" {

int wsg_deflate_batch_device(wsg_ctx* c, int level, int no_context, const wsg_frame_desc* desc, uint64_t n_frames,
                             const uint32_t* session_first, uint32_t n_sessions, const uint8_t* payload,
                             uint64_t payload_len, wsg_deflate_state* state, uint8_t* session_mem, uint8_t* out,
                             uint64_t out_cap, wsg_frame_desc* out_desc, uint64_t* out_total) {
  if (!c || !out_total) return WSG_API_EINVAL;
  (void)payload_len;
  return ws::deflate_launch(c, level, no_context, desc, n_frames, session_first, n_sessions, payload, state,
                            session_mem, out, out_cap, out_desc, nullptr, out_total);
}

int wsg_deflate_batch_host(wsg_ctx* c, int level, int no_context, const wsg_frame_desc* desc, uint64_t n_frames,
                           const uint32_t* session_first, uint32_t n_sessions, const uint8_t* payload,
                           uint64_t payload_len, wsg_deflate_state* state, uint8_t* session_mem, uint8_t* out,
                           uint64_t out_cap, wsg_frame_desc* out_desc, uint64_t* out_total) {
  if (!c || !out_total) return WSG_API_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  const uint64_t S = n_sessions, F = n_frames;
  DevBuf d_desc, d_sf, d_pay, d_state, d_mem, d_out, d_odesc;
  struct Guard {
    DevBuf* b[7];
    ~Guard() { for (DevBuf* x : b) x->release(); }
  } g{{&d_desc, &d_sf, &d_pay, &d_state, &d_mem, &d_out, &d_odesc}};
  HIP_TRY(c, d_desc.ensure((F + 1) * sizeof(wsg_frame_desc)));
  HIP_TRY(c, d_sf.ensure((S + 1) * sizeof(uint32_t)));
  HIP_TRY(c, d_pay.ensure(payload_len + 32));
  HIP_TRY(c, d_state.ensure((S + 1) * sizeof(wsg_deflate_state)));
  HIP_TRY(c, d_mem.ensure((S + 1) * (uint64_t)WSG_DEFLATE_SESSION_BYTES));
  HIP_TRY(c, d_out.ensure(out_cap + 32));
  HIP_TRY(c, d_odesc.ensure((F + 1) * sizeof(wsg_frame_desc)));
  hipStream_t s = c->stream;
  if (F) HIP_TRY(c, hipMemcpyAsync(d_desc.p, desc, F * sizeof(wsg_frame_desc), hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(d_sf.p, session_first, (S + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  if (payload_len) HIP_TRY(c, hipMemcpyAsync(d_pay.p, payload, payload_len, hipMemcpyHostToDevice, s));
  if (S) {
    HIP_TRY(c, hipMemcpyAsync(d_state.p, state, S * sizeof(wsg_deflate_state), hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(d_mem.p, session_mem, S * (uint64_t)WSG_DEFLATE_SESSION_BYTES, hipMemcpyHostToDevice, s));
  }
  int rc = wsg_deflate_batch_device(c, level, no_context, (const wsg_frame_desc*)d_desc.p, F, (const uint32_t*)d_sf.p,
                                    n_sessions, (const uint8_t*)d_pay.p, payload_len, (wsg_deflate_state*)d_state.p,
                                    (uint8_t*)d_mem.p, (uint8_t*)d_out.p, out_cap, (wsg_frame_desc*)d_odesc.p,
                                    out_total);
  if (rc) return rc;
  if (*out_total) HIP_TRY(c, hipMemcpyAsync(out, d_out.p, *out_total, hipMemcpyDeviceToHost, s));
  if (F) HIP_TRY(c, hipMemcpyAsync(out_desc, d_odesc.p, F * sizeof(wsg_frame_desc), hipMemcpyDeviceToHost, s));
  if (S) {
    HIP_TRY(c, hipMemcpyAsync(state, d_state.p, S * sizeof(wsg_deflate_state), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(session_mem, d_mem.p, S * (uint64_t)WSG_DEFLATE_SESSION_BYTES, hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(c, hipStreamSynchronize(s));
  return WSG_API_OK;
}

int wsg_inflate_batch_device(wsg_ctx* c, int no_context, const wsg_frame_desc* desc, uint64_t n_frames,
                             const uint32_t* session_first, uint32_t n_sessions, const uint8_t* payload,
                             uint64_t payload_len, wsg_inflate_state* state, uint8_t* window, uint8_t* out,
                             const uint64_t* out_off, wsg_frame_desc* out_desc, wsg_session_result* out_result,
                             uint32_t* replay_from) {
  if (!c) return WSG_API_EINVAL;
  if (n_sessions == 0) return n_frames ? set_err(c, WSG_API_EINVAL, "frames without sessions") : WSG_API_OK;
  HIP_TRY(c, hipSetDevice(c->device));
  InflArgs a = infl_args(c, no_context, desc, n_frames, session_first, n_sessions, payload, payload_len, state, window,
                         out, out_off, out_desc, out_result, replay_from);
  if (c->infl_tokens && n_frames) {
    const int rc = infl_tok_args(c, a, n_frames, payload_len);
    if (rc) return rc;
    HIP_TRY(c, hipMemsetAsync(c->i_tabcnt.p, 0, sizeof(uint32_t), c->stream));
    timed(c, K_INFL_TOK, [&] { launch_infl_tok(a, c->stream); });
    if (c->infl_fast) {
      HIP_TRY(c, c->i_fast.ensure(n_sessions));  // (sessions: not covered by wsg_reserve_inflate)
      a.fast_done = (uint8_t*)c->i_fast.p;
      timed(c, K_INFL_FAST, [&] { launch_infl_fast(a, c->stream); });
    }
  }
  // (WSG_INFLATE_FAST=2, tests only: no serial pass, so a session the fast replay did not
  // take is left unprocessed and shows)
  if (!(c->infl_fast == 2 && a.fast_done)) timed(c, K_INFLATE, [&] { launch_inflate(a, c->stream); });
  HIP_TRY(c, hipGetLastError());
  return WSG_API_OK;
}

int wsg_inflate_batch_host(wsg_ctx* c, int no_context, const wsg_frame_desc* desc, uint64_t n_frames,
                           const uint32_t* session_first, uint32_t n_sessions, const uint8_t* payload,
                           uint64_t payload_len, wsg_inflate_state* state, uint8_t* window, uint8_t* out,
                           const uint64_t* out_off, wsg_frame_desc* out_desc, wsg_session_result* out_result,
                           uint32_t* replay_from) {
  if (!c) return WSG_API_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  const uint64_t S = n_sessions, F = n_frames;
  const uint64_t out_len = S ? out_off[S] : 0;
  DevBuf d_desc, d_sf, d_pay, d_state, d_win, d_out, d_off, d_odesc, d_res, d_rf;
  struct Guard {
    DevBuf* b[10];
    ~Guard() { for (DevBuf* x : b) x->release(); }
  } g{{&d_desc, &d_sf, &d_pay, &d_state, &d_win, &d_out, &d_off, &d_odesc, &d_res, &d_rf}};
  HIP_TRY(c, d_desc.ensure((F + 1) * sizeof(wsg_frame_desc)));
  HIP_TRY(c, d_sf.ensure((S + 1) * sizeof(uint32_t)));
  HIP_TRY(c, d_pay.ensure(payload_len + 32));
  HIP_TRY(c, d_state.ensure((S + 1) * sizeof(wsg_inflate_state)));
  HIP_TRY(c, d_win.ensure((S + 1) * WSG_INFLATE_WINDOW));
  HIP_TRY(c, d_out.ensure(out_len + 32));
  HIP_TRY(c, d_off.ensure((S + 1) * sizeof(uint64_t)));
  HIP_TRY(c, d_odesc.ensure((F + 1) * sizeof(wsg_frame_desc)));
  HIP_TRY(c, d_res.ensure((S + 1) * sizeof(wsg_session_result)));
  HIP_TRY(c, d_rf.ensure((S + 1) * sizeof(uint32_t)));
  hipStream_t s = c->stream;
  if (F) HIP_TRY(c, hipMemcpyAsync(d_desc.p, desc, F * sizeof(wsg_frame_desc), hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(d_sf.p, session_first, (S + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  if (payload_len) HIP_TRY(c, hipMemcpyAsync(d_pay.p, payload, payload_len, hipMemcpyHostToDevice, s));
  if (S) {
    HIP_TRY(c, hipMemcpyAsync(d_state.p, state, S * sizeof(wsg_inflate_state), hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(d_win.p, window, S * WSG_INFLATE_WINDOW, hipMemcpyHostToDevice, s));
  }
  HIP_TRY(c, hipMemcpyAsync(d_off.p, out_off, (S + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  int rc = wsg_inflate_batch_device(c, no_context, (const wsg_frame_desc*)d_desc.p, F, (const uint32_t*)d_sf.p,
                                    n_sessions, (const uint8_t*)d_pay.p, payload_len, (wsg_inflate_state*)d_state.p,
                                    (uint8_t*)d_win.p, (uint8_t*)d_out.p, (const uint64_t*)d_off.p,
                                    (wsg_frame_desc*)d_odesc.p, (wsg_session_result*)d_res.p, (uint32_t*)d_rf.p);
  if (rc) return rc;
  if (out_len) HIP_TRY(c, hipMemcpyAsync(out, d_out.p, out_len, hipMemcpyDeviceToHost, s));
  if (F) HIP_TRY(c, hipMemcpyAsync(out_desc, d_odesc.p, F * sizeof(wsg_frame_desc), hipMemcpyDeviceToHost, s));
  if (S) {
    HIP_TRY(c, hipMemcpyAsync(out_result, d_res.p, S * sizeof(wsg_session_result), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(state, d_state.p, S * sizeof(wsg_inflate_state), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(window, d_win.p, S * WSG_INFLATE_WINDOW, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(replay_from, d_rf.p, S * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(c, hipStreamSynchronize(s));
  return WSG_API_OK;
}

// ---- opening handshake (server side), SURVEY §8f rank 4 ----

int wsg_handshake_available(const uint8_t* data, uint64_t len) {
  if (!data && len) return WSG_API_EINVAL;
  int capped = 0;
  int64_t lines_end = 0;
  return ws::hs_frame_len(data, (int64_t)len, &capped, &lines_end);
}

int wsg_handshake_accept_batch_device(wsg_ctx* c, const wsg_hs_config* cfg, const uint8_t* req,
                                      const uint64_t* req_off, uint32_t n, uint8_t* resp, wsg_hs_result* result) {
  if (!c || !cfg) return WSG_API_EINVAL;
  if (!n) return WSG_API_OK;
  if (!req || !req_off || !resp || !result) return set_err(c, WSG_API_EINVAL, "null batch pointer");
  if (((uintptr_t)req & 15) || ((uintptr_t)resp & 15))
    return set_err(c, WSG_API_EINVAL, "req and resp must be 16-B aligned");
  HIP_TRY(c, hipSetDevice(c->device));
  timed(c, K_HS_ACCEPT, [&] { ws::launch_hs_accept(*cfg, req, req_off, n, resp, result, c->stream); });
  HIP_TRY(c, hipGetLastError());
  return WSG_API_OK;
}

int wsg_handshake_accept_batch_host(wsg_ctx* c, const wsg_hs_config* cfg, const uint8_t* req,
                                    const uint64_t* req_off, uint32_t n, uint8_t* resp, wsg_hs_result* result) {
  if (!c || !cfg) return WSG_API_EINVAL;
  if (!n) return WSG_API_OK;
  if (!req_off || !resp || !result) return set_err(c, WSG_API_EINVAL, "null batch pointer");
  for (uint32_t i = 0; i < n; ++i)
    if (req_off[i + 1] < req_off[i]) return set_err(c, WSG_API_EINVAL, "req_off not ascending at %u", i);
  if (req_off[0] != 0) return set_err(c, WSG_API_EINVAL, "req_off[0] must be 0");
  HIP_TRY(c, hipSetDevice(c->device));
  const uint64_t len = req_off[n];
  DevBuf d_req, d_off, d_resp, d_res;
  struct Guard {
    DevBuf* b[4];
    ~Guard() { for (DevBuf* x : b) x->release(); }
  } g{{&d_req, &d_off, &d_resp, &d_res}};
  HIP_TRY(c, d_req.ensure(len + 16));
  HIP_TRY(c, d_off.ensure(((uint64_t)n + 1) * sizeof(uint64_t)));
  HIP_TRY(c, d_resp.ensure((uint64_t)n * WSG_HS_RESP_STRIDE));
  HIP_TRY(c, d_res.ensure((uint64_t)n * sizeof(wsg_hs_result)));
  hipStream_t s = c->stream;
  if (len) HIP_TRY(c, hipMemcpyAsync(d_req.p, req, len, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(d_off.p, req_off, ((uint64_t)n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  int rc = wsg_handshake_accept_batch_device(c, cfg, (const uint8_t*)d_req.p, (const uint64_t*)d_off.p, n,
                                             (uint8_t*)d_resp.p, (wsg_hs_result*)d_res.p);
  if (rc) return rc;
  HIP_TRY(c, hipMemcpyAsync(resp, d_resp.p, (uint64_t)n * WSG_HS_RESP_STRIDE, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(result, d_res.p, (uint64_t)n * sizeof(wsg_hs_result), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  return WSG_API_OK;
}

// ---- opening handshake (client side): validate the servers' responses ----

int wsg_handshake_validate_batch_device(wsg_ctx* c, const wsg_hs_config* cfg, const uint8_t* resp,
                                        const uint64_t* resp_off, const uint8_t* keys, uint32_t n,
                                        uint8_t* expected_out, wsg_hs_result* result) {
  if (!c || !cfg) return WSG_API_EINVAL;
  if (!n) return WSG_API_OK;
  if (!resp || !resp_off || !keys || !expected_out || !result) return set_err(c, WSG_API_EINVAL, "null batch pointer");
  if (((uintptr_t)resp & 15) || ((uintptr_t)expected_out & 15) || ((uintptr_t)keys & 3))
    return set_err(c, WSG_API_EINVAL, "resp and expected_out must be 16-B aligned, keys 4-B aligned");
  HIP_TRY(c, hipSetDevice(c->device));
  timed(c, K_HS_VALIDATE,
        [&] { ws::launch_hs_validate(*cfg, resp, resp_off, keys, n, expected_out, result, c->stream); });
  HIP_TRY(c, hipGetLastError());
  return WSG_API_OK;
}

int wsg_handshake_validate_batch_host(wsg_ctx* c, const wsg_hs_config* cfg, const uint8_t* resp,
                                      const uint64_t* resp_off, const uint8_t* keys, uint32_t n,
                                      uint8_t* expected_out, wsg_hs_result* result) {
  if (!c || !cfg) return WSG_API_EINVAL;
  if (!n) return WSG_API_OK;
  if (!resp_off || !keys || !expected_out || !result) return set_err(c, WSG_API_EINVAL, "null batch pointer");
  for (uint32_t i = 0; i < n; ++i)
    if (resp_off[i + 1] < resp_off[i]) return set_err(c, WSG_API_EINVAL, "resp_off not ascending at %u", i);
  if (resp_off[0] != 0) return set_err(c, WSG_API_EINVAL, "resp_off[0] must be 0");
  HIP_TRY(c, hipSetDevice(c->device));
  const uint64_t len = resp_off[n];
  DevBuf d_resp, d_off, d_keys, d_exp, d_res;
  struct Guard {
    DevBuf* b[5];
    ~Guard() { for (DevBuf* x : b) x->release(); }
  } g{{&d_resp, &d_off, &d_keys, &d_exp, &d_res}};
  HIP_TRY(c, d_resp.ensure(len + 16));
  HIP_TRY(c, d_off.ensure(((uint64_t)n + 1) * sizeof(uint64_t)));
  HIP_TRY(c, d_keys.ensure((uint64_t)n * 24));
  HIP_TRY(c, d_exp.ensure((uint64_t)n * WSG_HS_EXPECTED_STRIDE));
  HIP_TRY(c, d_res.ensure((uint64_t)n * sizeof(wsg_hs_result)));
  hipStream_t s = c->stream;
  if (len) HIP_TRY(c, hipMemcpyAsync(d_resp.p, resp, len, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(d_off.p, resp_off, ((uint64_t)n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(d_keys.p, keys, (uint64_t)n * 24, hipMemcpyHostToDevice, s));
  int rc = wsg_handshake_validate_batch_device(c, cfg, (const uint8_t*)d_resp.p, (const uint64_t*)d_off.p,
                                               (const uint8_t*)d_keys.p, n, (uint8_t*)d_exp.p,
                                               (wsg_hs_result*)d_res.p);
  if (rc) return rc;
  HIP_TRY(c, hipMemcpyAsync(expected_out, d_exp.p, (uint64_t)n * WSG_HS_EXPECTED_STRIDE, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(result, d_res.p, (uint64_t)n * sizeof(wsg_hs_result), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  return WSG_API_OK;
}

}  // extern "C"
