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
