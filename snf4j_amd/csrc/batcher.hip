// batcher.hip — the host side of the drop-in boundary:
// the cross-session batcher a JNI shim drives, and a pinned-host buffer pool in
// the role of snf4j's IByteBufferAllocator (IByteBufferAllocator.java:38-149).
//
// The reference decodes inside each session's read loop: StreamSession
// .consumeBuffer (StreamSession.java:798-854) asks FrameDecoder.available()
// (FrameDecoder.java:357-401) how many bytes form the next frame and hands that
// many to decode().  Here every session's socket bytes are fed to one batcher;
// it runs the same delimiting per session on the host (available(), then the
// header-only rules as soon as a header is complete, as FrameDecoder.decode does
// before the payload arrives, :197-256), keeps complete frames in the session's
// input buffer with the partial one after them, and flush() gathers all
// sessions' complete frames into pinned staging (threads over byte-balanced
// slices of the sessions) and decodes them in ONE device batch
// (wsg_decode_batch_host_async).  Per-session decoder state (fragmentation,
// UTF-8 carry, closed) persists across flushes.
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "wsgpu_internal.h"

namespace {

struct PinnedBuf {
  uint8_t* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= n && p) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    const size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
    hipError_t e = hipHostMalloc((void**)&p, want, hipHostMallocDefault);
    if (e == hipSuccess) n = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
  }
};

struct SessIn {
  std::vector<uint8_t> buf;    // complete frames [0, complete), then the partial frame's bytes
  size_t complete = 0;         // bytes of complete frames
  std::vector<uint32_t> lens;  // lengths of the complete frames
  bool frag = false;           // FrameDecoder.fragmentation as of the complete frames
  int32_t host_err = 0;        // header error seen on the host (its frame may never complete)
  int64_t d1 = 0;
};

uint32_t hdr_len(const uint8_t* p) {
  const uint32_t l7 = p[1] & 0x7fu;
  return 2u + ((p[1] & 0x80u) ? 4u : 0u) + (l7 == 126 ? 2u : (l7 == 127 ? 8u : 0u));
}

uint64_t frame_total(const uint8_t* p) {
  const uint32_t l7 = p[1] & 0x7fu;
  uint64_t len = l7;
  if (l7 == 126) {
    len = ((uint64_t)p[2] << 8) | p[3];
  } else if (l7 == 127) {
    len = 0;
    for (int i = 0; i < 8; ++i) len = (len << 8) | p[2 + i];
  }
  return hdr_len(p) + len;
}

}  // namespace

struct wsg_batcher {
  wsg_ctx* ctx = nullptr;
  wsg_decoder_cfg cfg{};
  uint32_t n = 0;
  std::vector<SessIn> s;
  std::vector<wsg_session_state> state;
  PinnedBuf wire, off, sf, st, payload, desc, result;
  uint32_t threads = 8;
  std::string err;
};

static int bset(wsg_batcher* b, int code, const char* msg) {
  if (b) b->err = msg ? msg : "";
  return code;
}

#define B_TRY(b, expr)                                                           \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    if (_e != hipSuccess) return bset((b), WSG_API_EHIP, hipGetErrorString(_e)); \
  } while (0)

extern "C" {

int wsg_batcher_open(wsg_ctx* ctx, const wsg_decoder_cfg* cfg, uint32_t n_sessions, wsg_batcher** out) {
  if (!ctx || !cfg || !out) return WSG_API_EINVAL;
  wsg_batcher* b = new wsg_batcher();
  b->ctx = ctx;
  b->cfg = *cfg;
  b->n = n_sessions;
  b->s.resize(n_sessions);
  b->state.assign(n_sessions, wsg_session_state{});
  const unsigned hw = std::thread::hardware_concurrency();
  b->threads = hw ? std::min(16u, hw) : 8u;
  *out = b;
  return WSG_API_OK;
}

int wsg_batcher_close(wsg_batcher* b) {
  if (!b) return WSG_API_EINVAL;
  (void)wsg_sync(b->ctx);
  PinnedBuf* bufs[] = {&b->wire, &b->off, &b->sf, &b->st, &b->payload, &b->desc, &b->result};
  for (PinnedBuf* p : bufs) p->release();
  delete b;
  return WSG_API_OK;
}

const char* wsg_batcher_last_error(wsg_batcher* b) { return b ? b->err.c_str() : "null batcher"; }

int wsg_batcher_feed(wsg_batcher* b, uint32_t sid, const uint8_t* data, uint64_t len) {
  if (!b || sid >= b->n || (len && !data)) return WSG_API_EINVAL;
  SessIn& x = b->s[sid];
  if (b->state[sid].closed || x.host_err) return WSG_API_OK;  // FrameDecoder.closed: input is swallowed
  if (x.buf.capacity() < x.buf.size() + len) x.buf.reserve(std::max(x.buf.size() + len, 2 * x.buf.capacity()));
  x.buf.insert(x.buf.end(), data, data + len);
  size_t pos = x.complete;
  for (;;) {
    const uint64_t rem = x.buf.size() - pos;
    uint8_t hdr[16] = {0};  // available() and the header rules read <= 14 bytes
    memcpy(hdr, x.buf.data() + pos, rem < 14 ? rem : 14);
    int32_t e = 0;
    int64_t d1 = 0, d2 = 0;
    const int64_t r = wsg_frame_available(hdr, rem, &e, &d1, &d2);  // FrameDecoder.available
    if (r < 0) {  // the u64 length errors (:388-394)
      x.host_err = e;
      x.d1 = d1;
      break;
    }
    if (r == 0) break;  // header incomplete
    const uint32_t hl = hdr_len(hdr);
    const int32_t he = wsg_check_header(&b->cfg, x.frag ? 1 : 0, hdr, hl, &d1);
    if (he && he != WSG_E_BATCH) {  // a header rule fails now (:197-256)
      x.host_err = he;
      x.d1 = d1;
      break;
    }
    const uint64_t total = frame_total(hdr);
    if (rem < total) break;  // partial frame: stays on the host (FrameDecoder.java:276-283)
    const uint32_t op = hdr[0] & 15u;
    if (op <= WSG_OP_BINARY) x.frag = !(hdr[0] & 0x80u);
    x.lens.push_back((uint32_t)total);
    pos += total;
  }
  x.complete = pos;
  return WSG_API_OK;
}

int wsg_batcher_flush(wsg_batcher* b, wsg_batch_view* out) {
  if (!b || !out) return WSG_API_EINVAL;
  const uint32_t S = b->n;
  std::vector<uint64_t> sbytes(S + 1, 0);
  std::vector<uint32_t> sfr(S + 1, 0);
  for (uint32_t i = 0; i < S; ++i) {
    sbytes[i + 1] = sbytes[i] + b->s[i].complete;
    sfr[i + 1] = sfr[i] + (uint32_t)b->s[i].lens.size();
  }
  const uint64_t W = sbytes[S], F = sfr[S];
  B_TRY(b, b->wire.ensure(W + 64));
  B_TRY(b, b->off.ensure((F + 1) * sizeof(uint64_t)));
  B_TRY(b, b->sf.ensure((S + 1) * sizeof(uint32_t)));
  B_TRY(b, b->st.ensure((S + 1) * sizeof(wsg_session_state)));
  const uint64_t pcap = W + 16 * F + 16;
  B_TRY(b, b->payload.ensure(pcap));
  B_TRY(b, b->desc.ensure((F + 1) * sizeof(wsg_frame_desc)));
  B_TRY(b, b->result.ensure((S + 1) * sizeof(wsg_session_result)));
  uint64_t* off = (uint64_t*)b->off.p;
  uint32_t* sf = (uint32_t*)b->sf.p;
  memcpy(sf, sfr.data(), (S + 1) * sizeof(uint32_t));
  if (S) memcpy(b->st.p, b->state.data(), S * sizeof(wsg_session_state));
  // gather the complete frames into pinned staging: byte-balanced slices of the
  // sessions, one thread each (a single thread below 8 MiB)
  auto work = [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; ++i) {
      SessIn& x = b->s[i];
      if (x.complete) memcpy(b->wire.p + sbytes[i], x.buf.data(), x.complete);
      uint64_t o = sbytes[i];
      uint32_t k = sfr[i];
      for (uint32_t l : x.lens) {
        off[k++] = o;
        o += l;
      }
    }
  };
  const uint32_t T = (W < (8u << 20) || S < 2) ? 1u : std::min<uint32_t>(b->threads, S);
  if (T <= 1) {
    work(0, S);
  } else {
    std::vector<std::thread> pool;
    uint32_t lo = 0;
    for (uint32_t t = 0; t < T && lo < S; ++t) {
      uint32_t hi = lo + 1;
      if (t + 1 == T) {
        hi = S;
      } else {
        const uint64_t target = W * (t + 1) / T;
        while (hi < S && sbytes[hi + 1] <= target) ++hi;
      }
      pool.emplace_back(work, lo, hi);
      lo = hi;
    }
    for (auto& th : pool) th.join();
  }
  off[F] = W;
  int rc = wsg_decode_batch_host_async(b->ctx, &b->cfg, b->wire.p, W, off, F, sf, S, (wsg_session_state*)b->st.p,
                                       b->payload.p, pcap, (wsg_frame_desc*)b->desc.p,
                                       (wsg_session_result*)b->result.p);
  if (rc) return bset(b, rc, wsg_last_error(b->ctx));
  rc = wsg_sync(b->ctx);
  if (rc) return bset(b, rc, wsg_last_error(b->ctx));
  if (S) memcpy(b->state.data(), b->st.p, S * sizeof(wsg_session_state));
  // consume the decoded frames; merge the host-detected header errors of the
  // sessions the device did not fail first (their frame may never complete)
  wsg_session_result* res = (wsg_session_result*)b->result.p;
  for (uint32_t i = 0; i < S; ++i) {
    SessIn& x = b->s[i];
    if (x.complete) {
      x.buf.erase(x.buf.begin(), x.buf.begin() + (ptrdiff_t)x.complete);
      x.complete = 0;
      x.lens.clear();
    }
    if (!res[i].error && x.host_err && !b->state[i].closed) {
      res[i].error = (uint16_t)x.host_err;
      res[i].close_code = WSG_CLOSE_PROTOCOL_ERROR;  // every header / length rule closes with 1002
      res[i].detail = x.d1;
      b->state[i].closed = 1;
    }
    if (b->state[i].closed) {
      std::vector<uint8_t>().swap(x.buf);  // a closed session swallows further input
      x.host_err = 0;
    }
  }
  out->n_frames = F;
  out->n_sessions = S;
  out->wire_bytes = W;
  out->session_first = sf;
  out->desc = (const wsg_frame_desc*)b->desc.p;
  out->payload = b->payload.p;
  out->result = res;
  return WSG_API_OK;
}

int wsg_batcher_session_state(wsg_batcher* b, uint32_t sid, wsg_session_state* st) {
  if (!b || sid >= b->n || !st) return WSG_API_EINVAL;
  *st = b->state[sid];
  return WSG_API_OK;
}

// A session slot handed to a new session: a fresh FrameDecoder (FrameDecoder.java:
// 43-63: no partial frame, fragmentation and closed cleared) and a fresh
// FrameUtf8Validator (no context, FrameUtf8Validator.java:42).  Bytes fed but not
// flushed are dropped with the old session.
int wsg_batcher_session_reset(wsg_batcher* b, uint32_t sid) {
  if (!b || sid >= b->n) return WSG_API_EINVAL;
  SessIn& x = b->s[sid];
  std::vector<uint8_t>().swap(x.buf);
  std::vector<uint32_t>().swap(x.lens);
  x.complete = 0;
  x.frag = false;
  x.host_err = 0;
  x.d1 = 0;
  b->state[sid] = wsg_session_state{};
  return WSG_API_OK;
}

// ------------------------------------------------------------------ encode batcher
// FrameEncoder.encode (FrameEncoder.java:69-120) for every session of a selector
// loop in one device batch per loop iteration.  add() copies a frame's payload
// into a pinned arena in arrival order and keeps a 24-B record; flush() orders the
// records by session (a stable counting sort: a session's frames keep their order,
// their payloads stay where they landed, wsg_encode_frame.payload_off points at
// them) and encodes them in one wsg_encode_batch_host call.  The close latch
// (:71-76) is per session and persists across flushes.
struct wsg_enc_batcher {
  wsg_ctx* ctx = nullptr;
  int client = 0;
  uint32_t n = 0;
  std::vector<uint8_t> closed;           // FrameEncoder.closed per session
  std::vector<uint32_t> rec_sid;         // session of each queued frame, arrival order
  std::vector<wsg_encode_frame> rec;     // queued frames, arrival order
  std::vector<uint32_t> count;           // queued frames per session
  PinnedBuf arena, frames, sf, cl, wire, off;
  uint64_t arena_len = 0;
  std::string err;
};

static int eset(wsg_enc_batcher* b, int code, const char* msg) {
  if (b) b->err = msg ? msg : "";
  return code;
}

int wsg_enc_batcher_open(wsg_ctx* ctx, int client_mode, uint32_t n_sessions, wsg_enc_batcher** out) {
  if (!ctx || !out) return WSG_API_EINVAL;
  wsg_enc_batcher* b = new wsg_enc_batcher();
  b->ctx = ctx;
  b->client = client_mode ? 1 : 0;
  b->n = n_sessions;
  b->closed.assign(n_sessions, 0);
  b->count.assign(n_sessions, 0);
  *out = b;
  return WSG_API_OK;
}

int wsg_enc_batcher_close(wsg_enc_batcher* b) {
  if (!b) return WSG_API_EINVAL;
  (void)wsg_sync(b->ctx);
  PinnedBuf* bufs[] = {&b->arena, &b->frames, &b->sf, &b->cl, &b->wire, &b->off};
  for (PinnedBuf* p : bufs) p->release();
  delete b;
  return WSG_API_OK;
}

const char* wsg_enc_batcher_last_error(wsg_enc_batcher* b) { return b ? b->err.c_str() : "null batcher"; }

int wsg_enc_batcher_add(wsg_enc_batcher* b, uint32_t sid, uint8_t opcode, uint8_t flags, const uint8_t* mask,
                        const uint8_t* payload, uint32_t len) {
  if (!b || sid >= b->n || (len && !payload)) return WSG_API_EINVAL;
  if (b->closed[sid]) return WSG_API_OK;  // FrameEncoder.java:71-76: nothing after a CLOSE (latched earlier)
  const uint64_t at = (b->arena_len + 15) & ~15ull;
  if (at + len + 16 > b->arena.n) {  // grow, keeping what is queued (pinned: the H2D source)
    PinnedBuf g;
    if (g.ensure(std::max<uint64_t>(at + len + 16, 2 * b->arena.n)) != hipSuccess)
      return eset(b, WSG_API_ENOMEM, "pinned arena");
    if (b->arena_len) memcpy(g.p, b->arena.p, b->arena_len);
    b->arena.release();
    b->arena = g;
  }
  if (len) memcpy(b->arena.p + at, payload, len);
  b->arena_len = at + len;
  wsg_encode_frame f{};
  f.payload_off = at;
  f.payload_len = len;
  f.opcode = opcode;
  f.flags = flags;
  if (mask) memcpy(f.mask, mask, 4);
  b->rec.push_back(f);
  b->rec_sid.push_back(sid);
  ++b->count[sid];
  return WSG_API_OK;
}

int wsg_enc_batcher_flush(wsg_enc_batcher* b, wsg_enc_view* out) {
  if (!b || !out) return WSG_API_EINVAL;
  const uint32_t S = b->n;
  const uint64_t F = b->rec.size();
  B_TRY(b, b->frames.ensure((F + 1) * sizeof(wsg_encode_frame)));
  B_TRY(b, b->sf.ensure((S + 1) * sizeof(uint32_t)));
  B_TRY(b, b->cl.ensure(S + 1));
  B_TRY(b, b->off.ensure((F + 1) * sizeof(uint64_t)));
  uint32_t* sf = (uint32_t*)b->sf.p;
  sf[0] = 0;
  for (uint32_t i = 0; i < S; ++i) sf[i + 1] = sf[i] + b->count[i];
  {  // stable counting sort of the records by session
    std::vector<uint32_t> pos(sf, sf + S);
    wsg_encode_frame* fr = (wsg_encode_frame*)b->frames.p;
    for (uint64_t k = 0; k < F; ++k) fr[pos[b->rec_sid[k]]++] = b->rec[k];
  }
  uint64_t need = 0;
  for (uint64_t k = 0; k < F; ++k) need += wsg_encoded_length(b->rec[k].payload_len, b->client);
  B_TRY(b, b->wire.ensure(need + 32));
  if (S) memcpy(b->cl.p, b->closed.data(), S);
  int rc = wsg_encode_batch_host(b->ctx, b->client, b->arena.p, b->arena_len, (const wsg_encode_frame*)b->frames.p, F,
                                 sf, S, b->cl.p, b->wire.p, b->wire.n, (uint64_t*)b->off.p);
  if (rc) return eset(b, rc, wsg_last_error(b->ctx));
  if (S) memcpy(b->closed.data(), b->cl.p, S);
  if (!F) ((uint64_t*)b->off.p)[0] = 0;
  b->rec.clear();
  b->rec_sid.clear();
  std::fill(b->count.begin(), b->count.end(), 0u);
  b->arena_len = 0;
  out->n_frames = F;
  out->wire_bytes = ((const uint64_t*)b->off.p)[F];
  out->n_sessions = S;
  out->reserved = 0;
  out->session_first = sf;
  out->wire_off = (const uint64_t*)b->off.p;
  out->wire = b->wire.p;
  return WSG_API_OK;
}

int wsg_enc_batcher_session_reset(wsg_enc_batcher* b, uint32_t sid) {
  if (!b || sid >= b->n) return WSG_API_EINVAL;
  if (b->count[sid]) {  // drop the slot's queued frames (their arena bytes stay until the flush)
    uint64_t j = 0;
    for (uint64_t k = 0; k < b->rec.size(); ++k)
      if (b->rec_sid[k] != sid) {
        b->rec[j] = b->rec[k];
        b->rec_sid[j++] = b->rec_sid[k];
      }
    b->rec.resize(j);
    b->rec_sid.resize(j);
    b->count[sid] = 0;
  }
  b->closed[sid] = 0;
  return WSG_API_OK;
}

// ------------------------------------------------------------------ pinned pool
// IByteBufferAllocator in the native layer: pinned (page-locked) host buffers in
// power-of-two size classes, recycled on release, so socket reads land where the
// DMA engines read at full PCIe rate (the JNI shim wraps them with NewDirectByteBuffer).
static std::mutex g_pool_mu;
static std::map<size_t, std::vector<void*>> g_pool_free;
static std::map<void*, size_t> g_pool_size;

static size_t size_class(uint64_t n) {
  size_t c = 4096;
  while (c < n) c <<= 1;
  return c;
}

void* wsg_host_alloc(uint64_t capacity) {
  const size_t c = size_class(capacity);
  std::lock_guard<std::mutex> g(g_pool_mu);
  auto& fl = g_pool_free[c];
  if (!fl.empty()) {
    void* p = fl.back();
    fl.pop_back();
    return p;
  }
  void* p = nullptr;
  if (hipHostMalloc(&p, c, hipHostMallocDefault) != hipSuccess) return nullptr;
  g_pool_size[p] = c;
  return p;
}

int wsg_host_release(void* p) {
  if (!p) return WSG_API_EINVAL;
  std::lock_guard<std::mutex> g(g_pool_mu);
  auto it = g_pool_size.find(p);
  if (it == g_pool_size.end()) return WSG_API_EINVAL;  // not from this pool
  g_pool_free[it->second].push_back(p);
  return WSG_API_OK;
}

uint64_t wsg_host_capacity(const void* p) {
  std::lock_guard<std::mutex> g(g_pool_mu);
  auto it = g_pool_size.find(const_cast<void*>(p));
  return it == g_pool_size.end() ? 0 : it->second;
}

int wsg_host_trim(void) {
  std::lock_guard<std::mutex> g(g_pool_mu);
  for (auto& kv : g_pool_free) {
    for (void* p : kv.second) {
      g_pool_size.erase(p);
      (void)hipHostFree(p);
    }
    kv.second.clear();
  }
  return WSG_API_OK;
}

}  // extern "C"
