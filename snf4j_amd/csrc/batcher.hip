// batcher.hip — the host side of the drop-in boundary:
// the cross-session batchers a JNI shim drives, and a pinned-host buffer pool in
// the role of snf4j's IByteBufferAllocator (IByteBufferAllocator.java:38-149).
//
// The reference decodes inside each session's read loop: StreamSession
// .consumeBuffer (StreamSession.java:798-854) asks FrameDecoder.available()
// (FrameDecoder.java:357-401) how many bytes form the next frame and hands that
// many to decode().  Here every session's socket bytes are fed to one batcher:
// a feed copies each session's reads (after its carried partial frame) into a
// region of the open batch's pinned arena and delimits the frames there
// (available(), then the header-only rules as soon as a header is complete, as
// FrameDecoder.decode does before the payload arrives, :197-256); complete
// frames stay where they landed (WSG_CFG_SPARSE), the partial tail is carried.
// flush_async submits the arena as one device batch (wsg_decode_batch_host_async:
// H2D, decode, D2H) without gathering anything; up to two batches are in flight
// while the next one is fed.  Per-session decoder state (fragmentation, UTF-8
// carry, closed) chains through the batches on the device.  The stages after the
// decoder (inflate, validator, aggregator) run on the device over the decoded
// payloads, on a context of their own, with their per-session carry device-resident;
// one gather writes what the handler receives into pinned memory while the next
// flush's stages run.  The cross-session encode batcher (pipelined the same way)
// and the loop -> device policy are here too.
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "wsgpu_internal.h"

#if !defined(__HIP_DEVICE_COMPILE__)
#include <immintrin.h>
#endif

// -DWSG_STAGE_PROF (a measurement build, scripts/build_variant.sh): host time of each
// stage-chain phase, summed per batcher and printed at close.
#ifdef WSG_STAGE_PROF
#include <chrono>
#include <cstdio>
static double g_sp[20];
static const char* g_sp_name[20] = {"compute", "inflate.input", "inflate.kernels+sync", "inflate.results",
                                    "launch.validator", "aggregate", "fin.list", "gather.launch", "finish.sync", "wait.total",
                                    "precompute", "gather.pay_ensure", "gather.upload", "inflate.x", "launch.replay",
                                    "launch.downloads", "upload.memcpy", "upload.h2d", "begin", "fin.build"};
struct SpT {
  int i;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  explicit SpT(int k) : i(k) {}
  ~SpT() { g_sp[i] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count(); }
};
#define SP(k) SpT sp_##k(k)
#else
#define SP(k) (void)0
#endif


namespace {

// Host allocations a batcher made (pinned and device): after wsg_batcher_reserve /
// wsg_enc_batcher_reserve a flush within the reserved sizes makes none.
std::atomic<uint64_t> g_batcher_allocs{0};

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
    g_batcher_allocs.fetch_add(1, std::memory_order_relaxed);
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
  }
};

struct SessIn {
  std::vector<uint8_t> buf;    // the partial frame's bytes, carried to the session's next read
  bool frag = false;           // FrameDecoder.fragmentation as of the frames fed so far
  int32_t host_err = 0;        // header error seen on the host (its frame may never complete)
  int64_t d1 = 0, d2 = 0;
  bool host_closed = false;    // the session failed: further input is swallowed
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

// A persistent pool for the batcher's host work (feeds, the flush gather): creating
// threads per call cost ~30 us each, per round.  run(T, fn) runs fn(0..T-1) on the
// pool and the calling thread and returns when all are done.
// The flushes in flight (the header's WSG_BATCHER_MAX_INFLIGHT; A/B builds may
// override it, with bench.py's WSG_BENCH_INFLIGHT to match) and the two-phase inflate's
// pre-decode contexts (flush t pre-decodes on context t % kTokCtx).
#ifdef WSG_AB_INFLIGHT
static constexpr int kInflight = WSG_AB_INFLIGHT;
#else
static constexpr int kInflight = WSG_BATCHER_MAX_INFLIGHT;
#endif
#ifdef WSG_AB_TOKCTX
static constexpr int kTokCtx = WSG_AB_TOKCTX;
#else
static constexpr int kTokCtx = 3;
#endif

class Pool {
 public:
  explicit Pool(uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) w_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : w_) t.join();
  }
  uint32_t size() const { return (uint32_t)w_.size() + 1; }
  // fn(0..T-1) over the workers and the caller; `side`, if any, runs on the caller
  // first, while the workers start on the jobs
  void run(uint32_t T, const std::function<void(uint32_t)>& fn, const std::function<void()>* side = nullptr) {
    if (T <= 1 || w_.empty()) {
      if (side) (*side)();
      for (uint32_t t = 0; t < T; ++t) fn(t);
      return;
    }
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &fn;
      njobs_ = T;
      next_.store(0);
      left_ = T;
      ++gen_;
    }
    cv_.notify_all();
    if (side) (*side)();
    work();
    std::unique_lock<std::mutex> l(m_);
    done_.wait(l, [this] { return left_ == 0; });
    job_ = nullptr;
  }

 private:
  void work() {
    for (;;) {
      const uint32_t t = next_.fetch_add(1);
      if (t >= njobs_) return;
      (*job_)(t);
      std::lock_guard<std::mutex> g(m_);
      if (--left_ == 0) done_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
    }
  }
  std::vector<std::thread> w_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(uint32_t)>* job_ = nullptr;
  uint32_t njobs_ = 0, left_ = 0;
  std::atomic<uint32_t> next_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// Completion signal for a thread other than the one driving a batcher (wsg_batcher_await,
// wsg_enc_batcher_await): a host function queued on the download stream behind each
// flush raises `done` to that flush's ticket.  The argument is allocated per flush and
// holds the signal by shared_ptr, so a late callback never touches a freed batcher.
struct Notify {
  std::mutex m;
  std::condition_variable cv;
  uint64_t done = 0;
};
struct NotifyArg {
  std::shared_ptr<Notify> n;
  uint64_t ticket;
};
void notify_cb(void* p) {
  NotifyArg* a = (NotifyArg*)p;
  {
    std::lock_guard<std::mutex> g(a->n->m);
    if (a->ticket > a->n->done) a->n->done = a->ticket;
  }
  a->n->cv.notify_all();
  delete a;
}
hipError_t notify_after(hipStream_t s, const std::shared_ptr<Notify>& n, uint64_t ticket) {
  NotifyArg* a = new NotifyArg{n, ticket};
  const hipError_t e = hipLaunchHostFunc(s, notify_cb, a);
  if (e != hipSuccess) delete a;
  return e;
}
int64_t notify_await(Notify& n, uint64_t seen, int64_t timeout_ms) {
  std::unique_lock<std::mutex> l(n.m);
  if (timeout_ms > 0)
    n.cv.wait_for(l, std::chrono::milliseconds(timeout_ms), [&] { return n.done > seen; });
  else if (timeout_ms < 0)
    n.cv.wait(l, [&] { return n.done > seen; });
  return (int64_t)n.done;
}

// ------------------------------------------------------------------ stage chain: device buffers
// A device buffer that only grows.  grow_keep() keeps the first `keep` bytes (a
// stream-ordered copy) when it has to move.
struct DBuf {
  uint8_t* p = nullptr;
  size_t n = 0;
  PinnedBuf up;  // staging of upload() (a DMA from pinned memory, no copy through a runtime bounce buffer)
  hipError_t ensure(size_t bytes) {
    if (bytes <= n && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    const size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
    hipError_t e = hipMalloc((void**)&p, want);
    if (e == hipSuccess) n = want;
    g_batcher_allocs.fetch_add(1, std::memory_order_relaxed);
    return e;
  }
  hipError_t grow_keep(size_t bytes, size_t keep, hipStream_t s) {
    if (bytes <= n && p) return hipSuccess;
    const size_t want = bytes + bytes / 4;
    uint8_t* q = nullptr;
    hipError_t e = hipMalloc((void**)&q, want);
    g_batcher_allocs.fetch_add(1, std::memory_order_relaxed);
    if (e != hipSuccess) return e;
    if (p && keep) {
      e = hipMemcpyAsync(q, p, keep, hipMemcpyDeviceToDevice, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
    }
    if (p) (void)hipFree(p);
    p = q;
    n = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    up.release();
  }
};

typedef unsigned int ws_u32x4 __attribute__((ext_vector_type(4)));

// One copy of the stage chain's output gather: `len` bytes from the stage arena to
// the flush's output region (split so that no copy exceeds COPY_MAX).
struct StageCopy {
  uint64_t src, dst;
  uint32_t len, pad;
};
constexpr uint32_t COPY_MAX = 65536;

// One workgroup per copy.  Output slots are 16-B aligned; a source is 16-B aligned when
// it is a decoder payload slot, byte-aligned when it is inflated output (messages back
// to back): either way the host sees 16-B stores (PCIe writes of whole 16-B chunks; the
// 4-B stores of the unaligned case ran at 31.6 GB/s, profiles/r04_stageprof_final.txt).
#ifdef WSG_AB_GATHER
constexpr uint32_t GATHER_GROUPS = WSG_AB_GATHER;
#else
constexpr uint32_t GATHER_GROUPS = 12;  // workgroups of the output gather: enough to fill PCIe, few enough
                                         // that the next flush's small downloads still get a share of it
#endif

__global__ __launch_bounds__(256) void k_stage_copy(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                    const StageCopy* __restrict__ cp, uint32_t n) {
  for (uint32_t ci = blockIdx.x; ci < n; ci += gridDim.x) {
  const StageCopy c = cp[ci];
  const uint8_t* s = src + c.src;
  uint8_t* d = dst + c.dst;
  const uint32_t t = threadIdx.x;
  const uint64_t al = c.src | c.dst;
  uint32_t done = 0;
  if ((al & 15) == 0) {
    done = c.len & ~15u;
    for (uint32_t i = 16 * t; i < done; i += 16 * 256)
      __builtin_nontemporal_store(__builtin_nontemporal_load((const ws_u32x4*)(s + i)), (ws_u32x4*)(d + i));
  } else if ((c.dst & 15) == 0) {
    // dst aligned, src not (inflated messages lie back to back): each 16-B store is
    // assembled from the two aligned source words around it (v_alignbyte over the
    // word pair; the dword shift is uniform over the copy).  The second word may lie
    // up to 15 B past the source: inside the arena's 64-B tail, and never used.
    done = c.len & ~15u;
    const uint32_t sh = (uint32_t)(c.src & 15), q = sh >> 2, r = sh & 3;
    const ws_u32x4* s16 = (const ws_u32x4*)(s - sh);
    auto run = [&](auto qc) {
      constexpr uint32_t Q = decltype(qc)::value;
      for (uint32_t i = 16 * t; i < done; i += 16 * 256) {
        const ws_u32x4 x = __builtin_nontemporal_load(s16 + i / 16), y = __builtin_nontemporal_load(s16 + i / 16 + 1);
        const uint32_t w[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
        ws_u32x4 o;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) o[j] = __builtin_amdgcn_alignbyte(w[j + Q + 1], w[j + Q], r);
        __builtin_nontemporal_store(o, (ws_u32x4*)(d + i));
      }
    };
    switch (q) {
      case 0: run(std::integral_constant<uint32_t, 0>{}); break;
      case 1: run(std::integral_constant<uint32_t, 1>{}); break;
      case 2: run(std::integral_constant<uint32_t, 2>{}); break;
      default: run(std::integral_constant<uint32_t, 3>{}); break;
    }
  } else if ((al & 3) == 0) {
    done = c.len & ~3u;
    for (uint32_t i = 4 * t; i < done; i += 4 * 256) *(uint32_t*)(d + i) = *(const uint32_t*)(s + i);
  } else {
    // dst aligned, src not: each thread assembles a dword from the source dwords around it
    const uint32_t sh = (uint32_t)(c.src & 3) * 8;
    const uint32_t* s4 = (const uint32_t*)(s - (c.src & 3));
    if ((c.dst & 3) == 0 && c.len >= 8) {
      done = (c.len - 4) & ~3u;  // the last source dword may lie past the source: bytes below
      for (uint32_t i = 4 * t; i < done; i += 4 * 256) {
        const uint32_t lo = s4[i / 4], hi = s4[i / 4 + 1];
        *(uint32_t*)(d + i) = (uint32_t)((((uint64_t)hi << 32) | lo) >> sh);
      }
    }
  }
  for (uint32_t i = done + t; i < c.len; i += 256) d[i] = s[i];
  }
}

// Small device results to pinned host memory by a kernel writing the mapped buffers: a
// runtime D2H of these sizes (16-210 KB) held the calling thread until its stream
// reached it — ≈ 0.5 ms a stage flush of the host's time, the replay and validator's
// duration (profiles/r05_ab/r05an_stageprof.txt, launch.downloads).  Segment
// blockIdx.y, 16-B stores where both ends allow, bytes for the tail.
struct PushSeg {
  const uint8_t* src;
  uint8_t* dst;
  uint64_t bytes;
};
struct PushSegs {
  PushSeg s[4];
  int n;
};
__global__ __launch_bounds__(256) void k_push(PushSegs a) {
  const PushSeg g = a.s[blockIdx.y];
  const uint64_t n16 = g.bytes / 16, stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load((const ws_u32x4*)g.src + i), (ws_u32x4*)g.dst + i);
  if (blockIdx.x == 0)
    for (uint64_t i = 16 * n16 + threadIdx.x; i < g.bytes; i += 256) g.dst[i] = g.src[i];
}

// Fresh stage decoders for the sessions in sids[0..n): one workgroup per session zeroes
// its inflater state and window, validator context and aggregator state.
__global__ __launch_bounds__(256) void k_stage_reset(const uint32_t* __restrict__ sids, wsg_inflate_state* istate,
                                                     uint8_t* iwin, wsg_session_state* vstate, wsg_agg_state* astate) {
  const uint32_t sid = sids[blockIdx.x];
  ws_u32x4* w = (ws_u32x4*)(iwin + (uint64_t)sid * WSG_INFLATE_WINDOW);
  for (uint32_t i = threadIdx.x; i < WSG_INFLATE_WINDOW / 16; i += 256) w[i] = (ws_u32x4){0u, 0u, 0u, 0u};
  if (threadIdx.x == 0) {
    istate[sid] = wsg_inflate_state{};
    vstate[sid] = wsg_session_state{};
    astate[sid] = wsg_agg_state{};
  }
}

// The validator's input, made from inflate's output on the device (no host hop between
// the two stages): output slot k of session s holds a frame the validator must see
// when it is one of the n_delivered frames after the session's replayed ones (which
// stage_inflate keeps); its payload offset moves into the arena (inflated bytes lie at
// `ipos`, passed-through ones where the decoder left them).  Every other slot — a
// replayed frame, a frame after the session's inflate error, every frame of a session
// whose output region overflowed (run again) — becomes an empty final PING, a frame
// FrameUtf8Validator passes without touching its context (FrameUtf8Validator.java:
// 59-98), so the validator's state and its failure index (minus nheld) stay exact.
__global__ __launch_bounds__(256) void k_stage_vprep(const wsg_frame_desc* __restrict__ odesc,
                                                     const uint32_t* __restrict__ sf,
                                                     const uint32_t* __restrict__ nheld,
                                                     const wsg_session_result* __restrict__ ores, uint64_t ipos,
                                                     uint32_t S, uint64_t F, wsg_frame_desc* __restrict__ vdesc) {
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= F) return;
  uint32_t lo = 0, hi = S;  // the session owning slot k: sf[s] <= k < sf[s + 1]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (sf[mid] <= k) lo = mid;
    else hi = mid;
  }
  const uint32_t s = lo;
  const wsg_session_result r = ores[s];
  const uint64_t first = (uint64_t)sf[s] + nheld[s];
  wsg_frame_desc d;
  if (k >= first && k - first < r.n_delivered && r.error != WSG_E_INFLATE_CAPACITY) {
    d = odesc[k];
    if (d.flags & WSG_DESC_INFLATED) d.payload_off += ipos;
    d.flags &= 0xf0u | 0x80u;
  } else {
    d = wsg_frame_desc{};
    d.opcode = WSG_OP_PING;
    d.flags = 0x80u;
  }
  vdesc[k] = d;
}

}  // namespace

// The decoders after "ws-decoder" that run in the same flush (wsg_batcher_set_stages):
// per session, what each stage keeps between batches on the host (the device keeps
// the inflater state and window, the validator context and the aggregator state).
struct StageSess {
  std::vector<wsg_frame_desc> held_desc;  // inflate: frames of a compressed message a batch left open
  std::vector<uint8_t> held_bytes;        //   (their payloads; re-sent with WSG_DESC_REPLAY)
  std::vector<uint8_t> agg_held;          // aggregator: bytes of a message still open (PayloadAggregator)
  bool agg_held_valid = false;
};

// A stage's frames: per session, descriptors whose payload_off is an offset in the
// stage arena (device).
struct StageList {
  std::vector<uint32_t> sf;           // [S + 1]
  std::vector<wsg_frame_desc> desc;
  std::vector<uint32_t> n_ok;         // [S] frames of the session that go on (<= its count)
};

// A flush's output when stages run: what the handler receives, gathered on the device
// (`copies` move stage-arena bytes to 16-B slots of d_pay; `host_parts` are bytes only
// the host holds, an aggregated message's bytes from earlier batches) and downloaded
// on the batcher's download stream, so that the next flush's stages can run meanwhile.
struct StageOut {
  std::vector<uint32_t> sf;
  std::vector<wsg_frame_desc> desc;
  std::vector<wsg_session_result> res;
  std::vector<StageCopy> copies;
  std::vector<std::pair<uint64_t, std::vector<uint8_t>>> host_parts;
  uint64_t len = 0;
  PinnedBuf pay;
  DBuf d_copy;
  hipEvent_t gathered = nullptr, downloaded = nullptr;
  bool staged = false;  // computed, download queued (wsg_batcher_wait collects it)
};

// A flush's stage chain between its start and its collection (stage_begin ->
// stage_compute): the stage input, and the inflate attempt in flight.
struct InflJob {
  bool prepped = false;              // the input built (and, two-phase, its pre-decode launched)
  bool active = false;               // begun: the inflate replay launched
  std::vector<wsg_session_result> res;  // the decode results the input was built from
  int tc = -1;                       // two-phase: the pre-decode's context (b->tctx[tc])
  hipEvent_t tok_done = nullptr;     //   after its pre-decode
  hipEvent_t launched = nullptr;     // after the attempt in flight (its result downloads)
  std::vector<uint32_t> tmap;        //   the attempt's frame -> its index in cur (the pre-decode's list)
  StageList cur;                     // the stage input, then (after inflate) its output
  uint64_t used = 0;                 // the arena's extent so far
  StageList x;                       // the inflate attempt in flight
  bool x_cur = false;                //   (its input is cur as it is: x is not built)
  std::vector<uint32_t> todo, nheld;
  std::vector<uint64_t> cap, held_at, oo;
  uint64_t ipos = 0;
  bool validate = false;
  std::vector<wsg_frame_desc> od;    // output frames, a session's contiguous at od_at[s]
  std::vector<uint64_t> od_at;
  std::vector<uint32_t> od_n;
  bool in_order = true;              // (a session re-run for capacity comes after the others)
};

// One flush's pinned staging and results (two alternate: a flush can be in flight
// while the next one gathers).
struct HostErr {
  uint32_t sid;
  int32_t err;
  int64_t d1, d2;
};
struct FlushSlot {
  // the batch's wire: each feed's bytes of a session land in a region of the arena
  // (its carried partial frame first), so the flush gathers nothing; the complete
  // frames are where they landed (WSG_CFG_SPARSE), a partial tail is a gap
  PinnedBuf arena;
  uint64_t arena_len = 0;
  std::vector<std::vector<uint64_t>> fo;  // [n]: the session's complete frames (arena offsets), in order
  std::vector<uint64_t> fb;               // [n]: their bytes
  PinnedBuf off, sf, payload, desc, result;
  DBuf dpay;                              // with stages: the decoded payloads, kept on the device
  uint64_t pcap = 0;                      //   (their region's size)
  hipEvent_t dpay_done = nullptr;         //   after their copy (the stage stream waits for it)
  StageOut so;                            // the stages' output
  InflJob ij;                             // the stage chain begun (stage_begin)
  uint64_t F = 0, W = 0;
  std::vector<HostErr> host_err;  // header errors found on the host after this batch's frames
  std::vector<uint32_t> resets;   // slots given to a new session while this batch was in flight
  std::vector<int64_t> detail2;   // [n]: the view's detail2
  hipEvent_t done = nullptr;      // after its downloads
  uint64_t ticket = 0;            // its flush number (wsg_batcher_ticket)
};

struct wsg_batcher {
  wsg_ctx* ctx = nullptr;
  wsg_decoder_cfg cfg{};
  uint32_t n = 0;
  std::vector<SessIn> s;
  std::vector<wsg_session_state> state;  // the carry as of the last waited flush (+ host changes)
  PinnedBuf st;                          // the carry the device batches chain through
  FlushSlot fs[kInflight + 1];  // one being fed, up to MAX_INFLIGHT in flight
  int open = 0;                          // the slot feeds land in
  std::deque<int> q;                     // flushes in flight, oldest first
  std::vector<std::pair<uint32_t, int>> patch;  // host changes for the next batch's state: 0 reset, 1 closed
  uint32_t threads = 8;
  std::unique_ptr<Pool> pool;           // threads - 1 workers (the caller is the last one)
  std::string err;
  int stage_rc = 0;        // a deferred stage-chain error (stage_defer), reported by the next wait
  std::string stage_msg;
  // stages after the decoder (wsg_batcher_set_stages), run on the device at wait()
  wsg_stage_cfg stages{};
  bool has_stages = false;
  wsg_ctx* sctx = nullptr;  // the stages' own context (stream + workspace): a flush's stages run
                            // beside the next flush's upload and decode on the batcher's context
  std::vector<StageSess> ss;
  std::vector<uint8_t> stage_closed;    // failed by a stage: its later decoded frames go nowhere
  std::vector<uint32_t> stage_resets;   // sessions whose device stage carry is zeroed before the next run
  DBuf d_resets;
  DBuf d_istate, d_iwin, d_vstate, d_astate;  // per-session stage carry (device-resident)
  DBuf* ar = nullptr;  // the stage arena at hand: its flush's dpay (decoded payloads | held frames |
                       // inflated | aggregated)
  DBuf d_sf, d_desc, d_odesc, d_res, d_ores, d_rf, d_ooff, d_tot;
  DBuf d_nheld, d_vdesc, d_vres;        // the validator's input made on the device, its results
  // two-phase inflate: a flush's message-parallel pre-decode runs on one of two contexts
  // of its own (flush t on tctx[t % kTokCtx]) as soon as its decode is done, ahead of the
  // previous flush's replay; the replay reads it through d_tmap
  bool two_phase = false;
#ifdef WSG_NO_STAGE_EARLY
  bool stage_early = false;  // (A/B build: the chains start from wsg_batcher_wait only)
#else
  bool stage_early = true;   // stage_advance from flush_async
#endif
#ifdef WSG_NO_FEED_ADVANCE
  bool feed_advance = false;  // (A/B build)
#else
  bool feed_advance = true;   // stage_advance(collect) beside wsg_batcher_feed_many's copies
#endif
  wsg_ctx* tctx[kTokCtx] = {};
  DBuf d_tdesc[kTokCtx], d_tsf[kTokCtx], d_tmap;
  PinnedBuf h_odesc, h_ores, h_rf, h_astate, h_tot, h_vres;  // stage results downloaded
  PinnedBuf h_pend;                     // aggregator bytes held for the next flush, downloaded
  DBuf d_pend;
  hipStream_t s_dl = nullptr;           // downloads of stage outputs
  StageOut* out = nullptr;              // the output the stage run at hand writes
  uint64_t tickets = 0;                 // flushes queued so far (flush t's ticket is t)
  std::shared_ptr<Notify> notify = std::make_shared<Notify>();
  uint64_t res_wire = 0, res_frames = 0;  // the sizes wsg_batcher_reserve was given
  // inflate's first output region per session: 4 KiB + infl_ratio x its compressed bytes (a
  // session that overflows runs again with a larger one); wsg_batcher_reserve_stages sets it
  // from the caller's max_out_bytes (its expected expansion), 2..8
  uint32_t infl_ratio = 8;
};

static int bset(wsg_batcher* b, int code, const char* msg) {
  if (b) b->err = msg ? msg : "";
  return code;
}

// A stage-chain step that flush_async or a feed runs on the side (advancing the chains of
// flushes already queued) failed: that call did its own job, so it returns OK and the
// error is kept for the next wsg_batcher_wait, which reports it.
static void stage_defer(wsg_batcher* b, int rc) {
  if (rc && !b->stage_rc) {
    b->stage_rc = rc;
    b->stage_msg = b->err;
  }
}

#define B_TRY(b, expr)                                                           \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    if (_e != hipSuccess) return bset((b), WSG_API_EHIP, hipGetErrorString(_e)); \
  } while (0)

// ------------------------------------------------------------------ stages after the decoder
static inline uint64_t al16(uint64_t x) { return (x + 15) & ~15ull; }

// a later stage failed session s: its result, and the session is closed
// (the host carry b->state is the loop thread's: wsg_batcher_wait closes the session)
static void stage_fail(wsg_batcher* b, uint32_t s, const wsg_session_result& r) {
  b->stage_closed[s] = 1;
  b->out->res[s].error = r.error;
  b->out->res[s].close_code = r.close_code;
  b->out->res[s].detail = r.detail;
}

// A stage list's upload: the host copy into the buffer's pinned staging, then the
// device pulls it over PCIe (k_pull: 16-B loads from the mapped staging, a few
// workgroups) in stream order.  The runtime's DMA copy costs ~11 us of engine time a
// call at these sizes (16-320 KB: 40 x 213 KB drained in 457 us against 166 us pulled,
// tools/ubench_hostapi.hip, profiles/r05_ab/r05r_hostapi.txt), and a stage flush makes
// eight of them.
__global__ __launch_bounds__(256) void k_pull(const ws_u32x4* __restrict__ src, ws_u32x4* __restrict__ dst,
                                              uint32_t n16) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256)
    dst[i] = __builtin_nontemporal_load(src + i);
}

template <typename T>
static hipError_t upload(DBuf& d, const std::vector<T>& v, hipStream_t s) {
  const size_t bytes = v.size() * sizeof(T);
  // (both sized to whole 16-B words: the pull reads and writes up to 15 B past `bytes`)
  hipError_t e = d.ensure(al16(bytes) + sizeof(T));
  if (e == hipSuccess) e = d.up.ensure(al16(bytes) + sizeof(T));
  if (e != hipSuccess || v.empty()) return e;
  {
    SP(16);
    memcpy(d.up.p, v.data(), bytes);
  }
  SP(17);
#ifdef WSG_AB_DMA_UPLOAD
  return hipMemcpyAsync(d.p, d.up.p, bytes, hipMemcpyHostToDevice, s);
#else
  void* src = nullptr;
  e = hipHostGetDevicePointer(&src, d.up.p, 0);
  if (e != hipSuccess) return e;
  const uint32_t n16 = (uint32_t)(al16(bytes) / 16);
  hipLaunchKernelGGL(k_pull, dim3(std::min<uint32_t>(256, (n16 + 255) / 256)), dim3(256), 0, s, (const ws_u32x4*)src,
                     (ws_u32x4*)d.p, n16);
  return hipGetLastError();
#endif
}

// PerMessageDeflateDecoder over a flush's frames (PerMessageDeflateDecoder.java:68-105),
// on the device, with FrameUtf8Validator behind it: each session's frames after the
// frames of a message it left open; the inflated bytes go to the arena after the
// decoded payloads and the held frames.  Launched by infl_launch (uploads, kernels,
// result downloads: no host wait), collected by infl_collect (the wait, the results,
// and a session whose output region overflowed run again with a larger one — nothing
// of it was committed).  Between the two the caller feeds the next reads: the inflate
// runs meanwhile.

// this attempt's input: the todo sessions' frames; every session takes part (the carry
// is indexed by session), the others with no frames
static int infl_launch(wsg_batcher* b, FlushSlot& f) {
  SP(13);
  const uint32_t S = b->n;
  hipStream_t st = ws::ctx_stream(b->sctx);
  InflJob& j = f.ij;
  StageList& x = j.x;
  j.oo.assign(S + 1, 0);
  std::fill(j.nheld.begin(), j.nheld.end(), 0u);  // (this attempt's sessions set theirs)
  // Two-phase, with no held frames and every session that has frames taking part (the
  // common case), the attempt's input is the pre-decode's list as it is: its copy on the
  // device (d_tdesc / d_tsf of the pre-decode context) is the replay's, with the frame
  // map the identity, so nothing is rebuilt or uploaded for it.
  bool same = j.tc >= 0;
  {
    size_t ti = 0;
    for (uint32_t s = 0; s < S && same; ++s) {
      const bool in = ti < j.todo.size() && j.todo[ti] == s;
      ti += in;
      if (in ? !b->ss[s].held_desc.empty() : j.cur.sf[s + 1] != j.cur.sf[s]) same = false;
      j.oo[s + 1] = j.oo[s] + (in ? j.cap[s] : 0);
    }
  }
  j.x_cur = same;
  if (same) {
    x.sf.clear();
    x.desc.clear();
    j.tmap.clear();
  } else {
    x.sf.assign(S + 1, 0);
    x.desc.clear();
    j.tmap.clear();
  }
  size_t ti = 0;
  if (!same) {
    SP(1);
    for (uint32_t s = 0; s < S; ++s) {
      x.sf[s] = (uint32_t)x.desc.size();
      const bool in = ti < j.todo.size() && j.todo[ti] == s;
      j.oo[s + 1] = j.oo[s] + (in ? j.cap[s] : 0);
      if (!in) continue;
      ++ti;
      const StageSess& h = b->ss[s];
      for (const wsg_frame_desc& hd : h.held_desc) {
        wsg_frame_desc d = hd;
        d.flags |= WSG_DESC_REPLAY;
        d.payload_off += j.held_at[s];
        x.desc.push_back(d);
      }
      j.nheld[s] = (uint32_t)h.held_desc.size();
      if (b->two_phase) j.tmap.insert(j.tmap.end(), h.held_desc.size(), 0xFFFFFFFFu);  // (not pre-decoded)
      for (uint32_t k = j.cur.sf[s]; k < j.cur.sf[s + 1]; ++k) {
        wsg_frame_desc d = j.cur.desc[k];
        d.flags &= (uint8_t)~WSG_DESC_REPLAY;
        x.desc.push_back(d);
        if (b->two_phase) j.tmap.push_back((uint32_t)k);
      }
    }
  }
  if (!same) x.sf[S] = (uint32_t)x.desc.size();
  const uint64_t F = same ? j.cur.desc.size() : x.desc.size();
  const uint64_t ipos = j.ipos;
  DBuf& ar = f.dpay;
  // (a move of the arena waits for the pre-decode reading it)
  if (j.tc >= 0 && ipos + j.oo[S] + 64 > ar.n) B_TRY(b, hipEventSynchronize(j.tok_done));
  B_TRY(b, ar.grow_keep(ipos + j.oo[S] + 64, ipos, st));
  if (!same) {
    B_TRY(b, upload(b->d_desc, x.desc, st));
    B_TRY(b, upload(b->d_sf, x.sf, st));
  }
  const wsg_frame_desc* dx = (const wsg_frame_desc*)(same ? b->d_tdesc[j.tc].p : b->d_desc.p);
  const uint32_t* dxsf = (const uint32_t*)(same ? b->d_tsf[j.tc].p : b->d_sf.p);
  B_TRY(b, upload(b->d_ooff, j.oo, st));
  B_TRY(b, b->d_odesc.ensure((F + 1) * sizeof(wsg_frame_desc)));
  B_TRY(b, b->d_ores.ensure((S + 1) * sizeof(wsg_session_result)));
  B_TRY(b, b->d_rf.ensure((S + 1) * sizeof(uint32_t)));
  int rc;
  {
  SP(14);
  if (j.tc >= 0) {  // the replay of the pre-decode that ran on tctx[tc]
    if (!same) B_TRY(b, upload(b->d_tmap, j.tmap, st));
    B_TRY(b, hipStreamWaitEvent(st, j.tok_done, 0));
    rc = ws::inflate_replay_phase(b->sctx, b->tctx[j.tc], same ? nullptr : (const uint32_t*)b->d_tmap.p,
                                  b->stages.inflate_no_context, dx, F, dxsf, S, ar.p, ipos,
                                  (wsg_inflate_state*)b->d_istate.p, b->d_iwin.p, ar.p + ipos,
                                  (const uint64_t*)b->d_ooff.p, (wsg_frame_desc*)b->d_odesc.p,
                                  (wsg_session_result*)b->d_ores.p, (uint32_t*)b->d_rf.p);
  } else {
    rc = wsg_inflate_batch_device(b->sctx, b->stages.inflate_no_context, dx, F, dxsf, S, ar.p, ipos,
                                  (wsg_inflate_state*)b->d_istate.p,
                                  b->d_iwin.p, ar.p + ipos, (const uint64_t*)b->d_ooff.p,
                                  (wsg_frame_desc*)b->d_odesc.p, (wsg_session_result*)b->d_ores.p,
                                  (uint32_t*)b->d_rf.p);
  }
  }
  if (rc) return bset(b, rc, wsg_last_error(b->sctx));
  // FrameUtf8Validator right behind it on the device (PerMessageDeflateExtension.java:
  // 316-326): its input made from inflate's output by k_stage_vprep, no host hop
  j.validate = b->stages.validate != 0;
  if (j.validate) {
    SP(4);
    B_TRY(b, upload(b->d_nheld, j.nheld, st));
    B_TRY(b, b->d_vdesc.ensure((F + 1) * sizeof(wsg_frame_desc)));
    B_TRY(b, b->d_vres.ensure((S + 1) * sizeof(wsg_session_result)));
    if (F) {
      hipLaunchKernelGGL(k_stage_vprep, dim3((uint32_t)((F + 255) / 256)), dim3(256), 0, st,
                         (const wsg_frame_desc*)b->d_odesc.p, dxsf, (const uint32_t*)b->d_nheld.p, (const wsg_session_result*)b->d_ores.p, ipos, S, F,
                         (wsg_frame_desc*)b->d_vdesc.p);
      B_TRY(b, hipGetLastError());
    }
    rc = wsg_validate_batch_device(b->sctx, (const wsg_frame_desc*)b->d_vdesc.p, F, dxsf, S,
                                   ar.p, ipos + j.oo[S], (wsg_session_state*)b->d_vstate.p,
                                   (wsg_session_result*)b->d_vres.p);
    if (rc) return bset(b, rc, wsg_last_error(b->sctx));
  }
  SP(15);
  B_TRY(b, b->h_odesc.ensure((F + 1) * sizeof(wsg_frame_desc)));
  B_TRY(b, b->h_ores.ensure((S + 1) * sizeof(wsg_session_result)));
  B_TRY(b, b->h_rf.ensure((S + 1) * sizeof(uint32_t)));
  if (j.validate) B_TRY(b, b->h_vres.ensure((S + 1) * sizeof(wsg_session_result)));
#ifdef WSG_AB_RUNTIME_D2H
  if (F) B_TRY(b, hipMemcpyAsync(b->h_odesc.p, b->d_odesc.p, F * sizeof(wsg_frame_desc), hipMemcpyDeviceToHost, st));
  B_TRY(b, hipMemcpyAsync(b->h_ores.p, b->d_ores.p, S * sizeof(wsg_session_result), hipMemcpyDeviceToHost, st));
  B_TRY(b, hipMemcpyAsync(b->h_rf.p, b->d_rf.p, S * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  if (j.validate)
    B_TRY(b, hipMemcpyAsync(b->h_vres.p, b->d_vres.p, S * sizeof(wsg_session_result), hipMemcpyDeviceToHost, st));
#else
  {  // the results pushed into pinned memory by one kernel (see k_push)
    PushSegs ps{};
    int n = 0;
    auto seg = [&](PinnedBuf& h, const DBuf& d, uint64_t bytes) -> hipError_t {
      void* hp = nullptr;
      const hipError_t e = hipHostGetDevicePointer(&hp, h.p, 0);
      if (e == hipSuccess && bytes) ps.s[n++] = PushSeg{d.p, (uint8_t*)hp, bytes};
      return e;
    };
    B_TRY(b, seg(b->h_odesc, b->d_odesc, F * sizeof(wsg_frame_desc)));
    B_TRY(b, seg(b->h_ores, b->d_ores, S * sizeof(wsg_session_result)));
    B_TRY(b, seg(b->h_rf, b->d_rf, S * sizeof(uint32_t)));
    if (j.validate) B_TRY(b, seg(b->h_vres, b->d_vres, S * sizeof(wsg_session_result)));
    ps.n = n;
    if (n) {
      hipLaunchKernelGGL(k_push, dim3(16, (uint32_t)n), dim3(256), 0, st, ps);
      B_TRY(b, hipGetLastError());
    }
  }
#endif
  if (!j.launched) B_TRY(b, hipEventCreateWithFlags(&j.launched, hipEventDisableTiming));
  B_TRY(b, hipEventRecord(j.launched, st));
  return WSG_API_OK;
}

// The inflate job of flush f: the frames it takes (j.cur, the decoder's delivered frames),
// per session its output region and its held frames' place in the arena, their bytes
// uploaded; then the first attempt launched.
static int infl_begin(wsg_batcher* b, FlushSlot& f) {
  const uint32_t S = b->n;
  hipStream_t st = ws::ctx_stream(b->sctx);
  InflJob& j = f.ij;
  j.todo.clear();
  j.cap.assign(S, 0);
  j.held_at.assign(S, 0);
  j.nheld.assign(S, 0);
  j.od.clear();
  j.od_at.assign(S, 0);
  j.od_n.assign(S, 0);
  j.in_order = true;
  // the held frames' bytes go after the decoded payloads; sessions a stage closed or a
  // reset gave to a new session since the input was built take no part
  uint64_t hpos = j.used;
  for (uint32_t s = 0; s < S; ++s) {
    if (b->stage_closed[s] || std::find(f.resets.begin(), f.resets.end(), s) != f.resets.end()) continue;
    const StageSess& h = b->ss[s];
    uint64_t c = 0;
    if (!h.held_desc.empty()) {
      j.held_at[s] = hpos;
      hpos = al16(hpos + h.held_bytes.size());
      for (const wsg_frame_desc& hd : h.held_desc) c += hd.payload_len + 4;
    }
    for (uint32_t k = j.cur.sf[s]; k < j.cur.sf[s + 1]; ++k) c += j.cur.desc[k].payload_len + 4;
    if (h.held_desc.empty() && j.cur.sf[s + 1] == j.cur.sf[s]) continue;
    j.todo.push_back(s);
    j.cap[s] = al16(4096 + (uint64_t)b->infl_ratio * c);
  }
  if (j.tc >= 0 && hpos + 64 > f.dpay.n) B_TRY(b, hipEventSynchronize(j.tok_done));
  B_TRY(b, f.dpay.grow_keep(hpos + 64, f.pcap, st));
  for (uint32_t s = 0; s < S; ++s) {
    if (b->stage_closed[s] || std::find(f.resets.begin(), f.resets.end(), s) != f.resets.end()) continue;
    const StageSess& h = b->ss[s];
    if (!h.held_bytes.empty())
      B_TRY(b, hipMemcpyAsync(f.dpay.p + j.held_at[s], h.held_bytes.data(), h.held_bytes.size(),
                              hipMemcpyHostToDevice, st));
  }
  j.ipos = al16(hpos);
  if (j.todo.empty()) return WSG_API_OK;
  return infl_launch(b, f);
}

// Wait for the attempt in flight, take its results (runs again what overflowed), and
// leave in j.cur the inflate stage's output frames (validated), in j.used the arena's
// extent.  Sessions reset since the flush (f.resets) take nothing from it.
static int infl_collect(wsg_batcher* b, FlushSlot& f) {
  const uint32_t S = b->n;
  hipStream_t st = ws::ctx_stream(b->sctx);
  InflJob& j = f.ij;
  while (!j.todo.empty()) {
    {
      SP(2);
      B_TRY(b, hipStreamSynchronize(st));
    }
    const StageList& x = j.x_cur ? j.cur : j.x;
    const wsg_frame_desc* odesc = (const wsg_frame_desc*)b->h_odesc.p;
    const wsg_session_result* r = (const wsg_session_result*)b->h_ores.p;
    const uint32_t* rf = (const uint32_t*)b->h_rf.p;
    const wsg_session_result* vr = j.validate ? (const wsg_session_result*)b->h_vres.p : nullptr;
    const uint64_t ipos = j.ipos;
    std::vector<uint32_t> retry;
    struct Held {
      uint32_t s;
      uint64_t src, dst, len;
    };
    std::vector<Held> hd_copies;
    {
      SP(3);
      for (uint32_t s : j.todo) {
        if (std::find(f.resets.begin(), f.resets.end(), s) != f.resets.end()) {
          j.od_at[s] = j.od.size();  // the slot has a new session: this flush is not its
          j.od_n[s] = 0;
          continue;
        }
        if (r[s].error == WSG_E_INFLATE_CAPACITY) {
          j.cap[s] *= 8;
          retry.push_back(s);
          continue;
        }
        StageSess& h = b->ss[s];
        uint32_t n = 0;
        j.od_at[s] = j.od.size();
        for (uint32_t k = x.sf[s] + j.nheld[s]; k < x.sf[s + 1] && n < r[s].n_delivered; ++k, ++n) {
          wsg_frame_desc d = odesc[k];
          if (d.flags & WSG_DESC_INFLATED) d.payload_off += ipos;  // (else the input's arena offset)
          d.flags &= 0xf0u | 0x80u;
          j.od.push_back(d);
        }
        j.od_n[s] = n;
        std::vector<wsg_frame_desc> nhd;
        uint64_t nb = 0;
        if (r[s].error) stage_fail(b, s, r[s]);
        if (vr && vr[s].error) {  // the validator failed an earlier frame: its result is the session's
          const uint32_t v = vr[s].n_delivered >= j.nheld[s] ? vr[s].n_delivered - j.nheld[s] : 0u;
          j.od_n[s] = std::min(j.od_n[s], v);
          stage_fail(b, s, vr[s]);
        }
        if (!r[s].error && rf[s] != 0xFFFFFFFFu) {  // a message left open: its frames go again with the next batch
          for (uint32_t k = x.sf[s] + rf[s]; k < x.sf[s + 1]; ++k) {
            wsg_frame_desc d = x.desc[k];
            d.flags &= (uint8_t)~WSG_DESC_REPLAY;
            hd_copies.push_back({s, d.payload_off, nb, d.payload_len});
            d.payload_off = nb;
            nb += d.payload_len;
            nhd.push_back(d);
          }
        }
        h.held_desc.swap(nhd);
        h.held_bytes.assign(nb, 0);
      }
    }
    for (const Held& c : hd_copies)
      if (c.len)
        B_TRY(b, hipMemcpyAsync(b->ss[c.s].held_bytes.data() + c.dst, f.dpay.p + c.src, c.len,
                                hipMemcpyDeviceToHost, st));
    if (!hd_copies.empty()) B_TRY(b, hipStreamSynchronize(st));
    j.ipos = al16(ipos + j.oo[S]);
    if (!retry.empty()) j.in_order = false;
    j.todo.swap(retry);
    if (!j.todo.empty()) {
      const int rc = infl_launch(b, f);
      if (rc) return rc;
    }
  }
  StageList& cur = j.cur;
  cur.sf.assign(S + 1, 0);
  cur.n_ok.assign(S, 0);
  uint64_t k = 0;
  for (uint32_t s = 0; s < S; ++s) {
    cur.sf[s] = (uint32_t)k;
    cur.n_ok[s] = j.od_n[s];
    k += j.od_n[s];
  }
  cur.sf[S] = (uint32_t)k;
  if (j.in_order && k == j.od.size()) {
    cur.desc.swap(j.od);
  } else {
    cur.desc.resize(k);
    for (uint32_t s = 0; s < S; ++s)
      std::copy(j.od.begin() + j.od_at[s], j.od.begin() + j.od_at[s] + j.od_n[s], cur.desc.begin() + cur.sf[s]);
  }
  j.used = j.ipos;
  return WSG_API_OK;
}

// A stream at the device's highest priority: the queue's dispatches go ahead of the
// other streams' (the pre-decode, the next flushes' decode).
static hipError_t high_stream(hipStream_t* s) {
  int lo = 0, hi = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
  return e != hipSuccess ? e : hipStreamCreateWithPriority(s, hipStreamNonBlocking, hi);
}

// The stage outputs' download stream, at high priority: the output gather is what a
// flush's collection waits for, and its few workgroups were dispatched behind the
// pre-decode's and replay's (stage lines +7%: burst 18.8-19.0 -> 19.7-20.9, steady
// 25.1-25.6 -> 26.5-27.7 GiB/s, profiles/r05_ab/r05u_ab_prio.txt; the gather's waves at
// s_setprio 3 instead: no gain; the stage context's stream at high priority as well: a
// tie, r05v_ab_stprio.txt).
static hipError_t dl_stream(wsg_batcher* b) {
  return b->s_dl ? hipSuccess : high_stream(&b->s_dl);
}

// append an output frame: dev_len bytes at arena offset src, after `prefix` (host bytes)
static void fin_push(wsg_batcher* b, wsg_frame_desc d, uint64_t src, uint32_t dev_len, std::vector<uint8_t>* prefix) {
  StageOut& fp = *b->out;
  const uint64_t pos = fp.len;
  const uint64_t pre = prefix ? prefix->size() : 0;
  d.payload_off = pos;
  d.payload_len = (uint32_t)(pre + dev_len);
  for (uint64_t o = 0; o < dev_len; o += COPY_MAX) {
    const uint32_t n = (uint32_t)std::min<uint64_t>(COPY_MAX, dev_len - o);
    fp.copies.push_back({src + o, pos + pre + o, n, 0});
  }
  if (pre) fp.host_parts.emplace_back(pos, std::move(*prefix));
  fp.len = al16(pos + pre + dev_len);
  fp.desc.push_back(d);
}

// FrameAggregator over `cur` (FrameAggregator.java:72-104), on the device, straight
// into the output list: pass-through frames keep their bytes, an aggregated message is
// its held bytes (earlier batches, PayloadAggregator.java:34) + this batch's.
static int stage_aggregate(wsg_batcher* b, StageList& cur, uint64_t used) {
  SP(5);
  const uint32_t S = b->n;
  hipStream_t st = ws::ctx_stream(b->sctx);
  const uint64_t F = cur.desc.size();
  std::vector<wsg_session_result> dres(S);
  uint64_t bytes = 16;
  for (uint32_t s = 0; s < S; ++s) {
    dres[s].n_delivered = cur.n_ok[s];
    for (uint32_t k = cur.sf[s]; k < cur.sf[s] + cur.n_ok[s]; ++k) bytes += cur.desc[k].payload_len;
  }
  const uint64_t A0 = al16(used), cap = al16(bytes);
  B_TRY(b, b->ar->grow_keep(A0 + cap + 64, used, st));
  B_TRY(b, upload(b->d_desc, cur.desc, st));
  B_TRY(b, upload(b->d_sf, cur.sf, st));
  B_TRY(b, upload(b->d_res, dres, st));
  B_TRY(b, b->d_odesc.ensure((F + S + 1) * sizeof(wsg_frame_desc)));
  B_TRY(b, b->d_ores.ensure((S + 1) * sizeof(wsg_session_result)));
  B_TRY(b, b->d_tot.ensure(sizeof(uint64_t)));
  int rc = wsg_aggregate_batch_device(b->sctx, b->stages.max_aggregated_len, (const wsg_frame_desc*)b->d_desc.p, F,
                                      (const uint32_t*)b->d_sf.p, S, (const wsg_session_result*)b->d_res.p,
                                      b->ar->p, used, (wsg_agg_state*)b->d_astate.p, b->ar->p + A0, cap,
                                      (wsg_frame_desc*)b->d_odesc.p, (wsg_session_result*)b->d_ores.p,
                                      (uint64_t*)b->d_tot.p);
  if (rc) return bset(b, rc, wsg_last_error(b->sctx));
  B_TRY(b, b->h_odesc.ensure((F + S + 1) * sizeof(wsg_frame_desc)));
  B_TRY(b, b->h_ores.ensure((S + 1) * sizeof(wsg_session_result)));
  B_TRY(b, b->h_astate.ensure((S + 1) * sizeof(wsg_agg_state)));
  B_TRY(b, hipMemcpyAsync(b->h_odesc.p, b->d_odesc.p, (F + S) * sizeof(wsg_frame_desc), hipMemcpyDeviceToHost, st));
  B_TRY(b, hipMemcpyAsync(b->h_ores.p, b->d_ores.p, S * sizeof(wsg_session_result), hipMemcpyDeviceToHost, st));
  B_TRY(b, hipMemcpyAsync(b->h_astate.p, b->d_astate.p, S * sizeof(wsg_agg_state), hipMemcpyDeviceToHost, st));
  B_TRY(b, hipStreamSynchronize(st));
  const wsg_frame_desc* odesc = (const wsg_frame_desc*)b->h_odesc.p;
  const wsg_session_result* r = (const wsg_session_result*)b->h_ores.p;
  const wsg_agg_state* ast = (const wsg_agg_state*)b->h_astate.p;
  std::vector<std::pair<uint32_t, StageCopy>> pending;
  for (uint32_t s = 0; s < S; ++s) {
    b->out->sf[s] = (uint32_t)b->out->desc.size();
    StageSess& h = b->ss[s];
    const uint64_t base = (uint64_t)cur.sf[s] + s;
    for (uint32_t i = 0; i < r[s].n_delivered; ++i) {
      wsg_frame_desc d = odesc[base + i];
      if (d.flags & WSG_AGG_IN_AGG) {
        std::vector<uint8_t> pre;
        if ((d.flags & WSG_AGG_PREFIXED) && h.agg_held_valid) pre.swap(h.agg_held);
        h.agg_held.clear();
        h.agg_held_valid = false;
        d.flags = (uint8_t)((d.flags & 0xf0u) | 0x80u | WSG_OUT_AGGREGATED);
        fin_push(b, d, A0 + d.payload_off, d.payload_len, &pre);
      } else {
        d.flags &= 0xf0u | 0x80u;
        fin_push(b, d, d.payload_off, d.payload_len, nullptr);
      }
    }
    b->out->res[s].n_delivered = (uint32_t)b->out->desc.size() - b->out->sf[s];
    if (r[s].error) {
      stage_fail(b, s, r[s]);
      h.agg_held.clear();
      h.agg_held_valid = false;
    } else if (ast[s].open) {  // this batch's bytes of the message still open, held after the download
      const wsg_frame_desc& d = odesc[base + r[s].n_delivered];
      if (!((d.flags & WSG_AGG_PREFIXED) && h.agg_held_valid)) h.agg_held.clear();
      h.agg_held_valid = true;
      if (d.payload_len) pending.push_back({s, StageCopy{A0 + d.payload_off, 0, d.payload_len, 0}});
    } else {
      h.agg_held.clear();
      h.agg_held_valid = false;
    }
  }
  // the held bytes are needed before the next flush's stages run: fetched now, all of
  // them by one gather into pinned memory (a copy call per session cost ~25 us each)
  if (!pending.empty()) {
    std::vector<StageCopy> pc;
    uint64_t tot = 0;
    for (auto& pe : pending) {
      for (uint64_t o = 0; o < pe.second.len; o += COPY_MAX)
        pc.push_back({pe.second.src + o, tot + o, (uint32_t)std::min<uint64_t>(COPY_MAX, pe.second.len - o), 0});
      pe.second.dst = tot;
      tot = al16(tot + pe.second.len);
    }
    B_TRY(b, b->h_pend.ensure(tot + 16));
    B_TRY(b, upload(b->d_pend, pc, st));
    uint8_t* dst = nullptr;
    B_TRY(b, hipHostGetDevicePointer((void**)&dst, b->h_pend.p, 0));
    const uint32_t n = (uint32_t)pc.size();
    hipLaunchKernelGGL(k_stage_copy, dim3(std::min<uint32_t>(n, GATHER_GROUPS)), dim3(256), 0, st, b->ar->p, dst,
                       (const StageCopy*)b->d_pend.p, n);
    B_TRY(b, hipGetLastError());
    B_TRY(b, hipStreamSynchronize(st));
    for (const auto& pe : pending) {
      std::vector<uint8_t>& held = b->ss[pe.first].agg_held;
      held.insert(held.end(), b->h_pend.p + pe.second.dst, b->h_pend.p + pe.second.dst + pe.second.len);
    }
  }
  return WSG_API_OK;
}

// A flush's stage input, built once its decode is done: the decoder's delivered frames
// (their payloads still on the device, f.dpay).  Two-phase inflate: the message-parallel
// pre-decode of those frames launched on the flush's own context (it needs no inflater
// state: it runs ahead of the previous flush's replay, while the host collects that one).
static int stage_prep(wsg_batcher* b, FlushSlot& f, const wsg_session_result* res) {
  if (ws::ctx_stage_fail(b->ctx)) return bset(b, WSG_API_EHIP, "injected stage failure (WSG_TUNE_STAGE_FAIL)");
  const uint32_t S = b->n;
  InflJob& j = f.ij;
  j.res.assign(res, res + S);
  const uint32_t* sf = (const uint32_t*)f.sf.p;
  const wsg_frame_desc* desc = (const wsg_frame_desc*)f.desc.p;
  StageList& cur = j.cur;
  cur.sf.assign(S + 1, 0);
  cur.n_ok.assign(S, 0);
  cur.desc.clear();
  {
    SP(10);
    for (uint32_t s = 0; s < S; ++s) {
      cur.sf[s] = (uint32_t)cur.desc.size();
      const uint32_t nd = b->stage_closed[s] ? 0u : res[s].n_delivered;
      for (uint32_t k = sf[s]; k < sf[s] + nd; ++k) {
        wsg_frame_desc d = desc[k];
        d.flags &= 0xf0u | 0x80u;  // FIN, RSV (the "was masked" bit is the decoder's)
        cur.desc.push_back(d);
      }
      cur.n_ok[s] = nd;
    }
  }
  cur.sf[S] = (uint32_t)cur.desc.size();
  j.prepped = true;
  j.tc = -1;
  if (!b->two_phase || cur.desc.empty()) return WSG_API_OK;
  j.tc = (int)(f.ticket % kTokCtx);
  wsg_ctx* tc = b->tctx[j.tc];
  hipStream_t ts = ws::ctx_stream(tc);
  if (!j.tok_done) B_TRY(b, hipEventCreateWithFlags(&j.tok_done, hipEventDisableTiming));
  B_TRY(b, upload(b->d_tdesc[j.tc], cur.desc, ts));
  B_TRY(b, upload(b->d_tsf[j.tc], cur.sf, ts));
  if (f.pcap) B_TRY(b, hipStreamWaitEvent(ts, f.dpay_done, 0));
  const int rc = ws::inflate_tok_phase(tc, (const wsg_frame_desc*)b->d_tdesc[j.tc].p, cur.desc.size(),
                                       (const uint32_t*)b->d_tsf[j.tc].p, S, f.dpay.p, al16(f.pcap));
  if (rc) return bset(b, rc, wsg_last_error(tc));
  B_TRY(b, hipEventRecord(j.tok_done, ts));
  return WSG_API_OK;
}

// The stage chain of a flush begun (its predecessor's chain collected): the output
// reset, the stage carry of slots handed to new sessions zeroed, and the inflate (the
// replay of its pre-decode, two-phase) + validator launched on the stage stream (no
// wait: stage_compute collects).
static int stage_begin(wsg_batcher* b, FlushSlot& f, const wsg_session_result* res) {
  int rc;
  if (!f.ij.prepped && (rc = stage_prep(b, f, res))) return rc;
  SP(18);
  const uint32_t S = b->n;
  hipStream_t st = ws::ctx_stream(b->sctx);
  StageOut& o = f.so;
  b->out = &o;
  o.res = f.ij.res;
  o.sf.assign(S + 1, 0);
  o.desc.clear();
  o.copies.clear();
  o.host_parts.clear();
  o.len = 0;
  if (!b->stage_resets.empty()) {  // sessions handed to new sessions since the last run
    B_TRY(b, upload(b->d_resets, b->stage_resets, st));
    hipLaunchKernelGGL(k_stage_reset, dim3((uint32_t)b->stage_resets.size()), dim3(256), 0, st,
                       (const uint32_t*)b->d_resets.p, (wsg_inflate_state*)b->d_istate.p, b->d_iwin.p,
                       (wsg_session_state*)b->d_vstate.p, (wsg_agg_state*)b->d_astate.p);
    B_TRY(b, hipGetLastError());
    B_TRY(b, hipStreamSynchronize(st));  // (d_resets is reused)
    b->stage_resets.clear();
  }
  // a session a stage failed in an earlier flush is closed (InternalSession.controlClose):
  // the frames decoded for it in flushes already in flight reach no stage and no handler;
  // nor do a reset slot's old session's (also when the input was built before)
  for (uint32_t s = 0; s < S; ++s)
    if (b->stage_closed[s] || std::find(f.resets.begin(), f.resets.end(), s) != f.resets.end()) {
      o.res[s] = wsg_session_result{};
      f.ij.cur.n_ok[s] = 0;
    }
  f.ij.used = al16(f.pcap);
  f.ij.todo.clear();
  f.ij.active = true;
  if (f.pcap) B_TRY(b, hipStreamWaitEvent(st, f.dpay_done, 0));
  if (b->stages.inflate) return infl_begin(b, f);  // (the validator runs inside, on the device)
  B_TRY(b, f.dpay.grow_keep(f.ij.used + 64, f.pcap, st));
  return WSG_API_OK;
}

// The rest of the chain: the inflate's results collected, the aggregator, then one
// gather, and the download of what the handler receives queued on the download
// stream (collected by stage_finish).
static int stage_compute(wsg_batcher* b, FlushSlot& f, const wsg_session_result* res) {
  int rc;
  if (!f.ij.active && (rc = stage_begin(b, f, res))) return rc;
  SP(0);
  const uint32_t S = b->n;
  hipStream_t st = ws::ctx_stream(b->sctx);
  StageOut& o = f.so;
  b->out = &o;
  b->ar = &f.dpay;
  if (b->stages.inflate && (rc = infl_collect(b, f))) return rc;
  f.ij.active = false;
  f.ij.prepped = false;
  StageList& cur = f.ij.cur;
  const uint64_t used = f.ij.used;
  if (b->stages.aggregate) {
    if ((rc = stage_aggregate(b, cur, used))) return rc;
  } else {
    SP(19);
    for (uint32_t s = 0; s < S; ++s) {
      o.sf[s] = (uint32_t)o.desc.size();
      for (uint32_t k = cur.sf[s]; k < cur.sf[s] + cur.n_ok[s]; ++k)
        fin_push(b, cur.desc[k], cur.desc[k].payload_off, cur.desc[k].payload_len, nullptr);
      o.res[s].n_delivered = cur.n_ok[s];
    }
  }
  o.sf[S] = (uint32_t)o.desc.size();
  SP(7);
  // the output: gathered from this flush's arena straight into the pinned host buffer
  // by a few workgroups on the download stream (PCIe writes), so the next flush's
  // stages have the GPU meanwhile (a runtime D2H here is a blit kernel that takes
  // every CU while it waits on PCIe: round 5 measured a device-side gather + one
  // hipMemcpyAsync D2H, profiles/r05_ab/r05q_*: the blit's 0.9-1.5 ms slowed the
  // replay and the pre-decode beside it 2-4x)
  if (!o.gathered) B_TRY(b, hipEventCreateWithFlags(&o.gathered, hipEventDisableTiming));
  if (!o.downloaded) B_TRY(b, hipEventCreateWithFlags(&o.downloaded, hipEventDisableTiming));
  B_TRY(b, dl_stream(b));
  {
    SP(11);
    B_TRY(b, o.pay.ensure(o.len + 16));
  }
  if (!o.copies.empty()) {
    {
      SP(12);
      B_TRY(b, upload(o.d_copy, o.copies, st));
    }
    B_TRY(b, hipEventRecord(o.gathered, st));
    B_TRY(b, hipStreamWaitEvent(b->s_dl, o.gathered, 0));
    const uint32_t n = (uint32_t)o.copies.size();
    uint8_t* dst = nullptr;
    B_TRY(b, hipHostGetDevicePointer((void**)&dst, o.pay.p, 0));
    hipLaunchKernelGGL(k_stage_copy, dim3(std::min<uint32_t>(n, GATHER_GROUPS)), dim3(256), 0, b->s_dl, b->ar->p,
                       dst, (const StageCopy*)o.d_copy.p, n);
    B_TRY(b, hipGetLastError());
  }
  B_TRY(b, hipEventRecord(o.downloaded, b->s_dl));
  o.staged = true;
  return WSG_API_OK;
}

// Wait for a flush's stage output and put in the bytes only the host holds.
static int stage_finish(wsg_batcher* b, FlushSlot& f) {
  SP(8);
  StageOut& o = f.so;
  B_TRY(b, hipEventSynchronize(o.downloaded));
  for (auto& hp : o.host_parts)
    if (!hp.second.empty()) memcpy(o.pay.p + hp.first, hp.second.data(), hp.second.size());
  o.host_parts.clear();
  o.staged = false;
  return WSG_API_OK;
}

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
  b->pool.reset(new Pool(b->threads - 1));
  for (FlushSlot& f : b->fs) {
    f.fo.resize(n_sessions);
    f.fb.assign(n_sessions, 0);
  }
  *out = b;
  return WSG_API_OK;
}

wsg_ctx* wsg_batcher_stage_context(wsg_batcher* b) { return b ? b->sctx : nullptr; }

int wsg_batcher_close(wsg_batcher* b) {
  if (!b) return WSG_API_EINVAL;
  (void)wsg_sync(b->ctx);
  for (wsg_ctx* t : b->tctx)
    if (t) (void)wsg_sync(t);
  if (b->sctx) (void)wsg_sync(b->sctx);
  if (b->s_dl) (void)hipStreamSynchronize(b->s_dl);
  for (FlushSlot& f : b->fs) {
    PinnedBuf* bufs[] = {&f.arena, &f.off, &f.sf, &f.payload, &f.desc, &f.result};
    for (PinnedBuf* p : bufs) p->release();
    f.dpay.release();
    f.so.pay.release();
    f.so.d_copy.release();
    if (f.so.gathered) (void)hipEventDestroy(f.so.gathered);
    if (f.so.downloaded) (void)hipEventDestroy(f.so.downloaded);
    if (f.done) (void)hipEventDestroy(f.done);
    if (f.dpay_done) (void)hipEventDestroy(f.dpay_done);
    if (f.ij.tok_done) (void)hipEventDestroy(f.ij.tok_done);
    if (f.ij.launched) (void)hipEventDestroy(f.ij.launched);
  }
  b->st.release();
  DBuf* dbufs[] = {&b->d_pend, &b->d_resets, &b->d_istate, &b->d_iwin, &b->d_vstate, &b->d_astate, &b->d_sf, &b->d_desc,
                   &b->d_odesc, &b->d_res, &b->d_ores, &b->d_rf, &b->d_ooff, &b->d_tot, &b->d_nheld, &b->d_vdesc,
                   &b->d_vres};
  for (DBuf* d : dbufs) d->release();
  PinnedBuf* hbufs[] = {&b->h_odesc, &b->h_ores, &b->h_rf, &b->h_astate, &b->h_tot, &b->h_pend, &b->h_vres};
  for (PinnedBuf* p : hbufs) p->release();
  if (b->s_dl) {
    (void)hipStreamSynchronize(b->s_dl);
    (void)hipStreamDestroy(b->s_dl);
  }
  if (b->sctx) (void)wsg_close(b->sctx);
  for (int i = 0; i < kTokCtx; ++i) {
    if (b->tctx[i]) (void)wsg_close(b->tctx[i]);
    b->d_tdesc[i].release();
    b->d_tsf[i].release();
  }
  b->d_tmap.release();
#ifdef WSG_STAGE_PROF
  for (int i = 0; i < 20; ++i)
    if (g_sp[i] > 0) fprintf(stderr, "[stage prof] %-22s %9.3f ms\n", g_sp_name[i], g_sp[i]);
#endif
  delete b;
  return WSG_API_OK;
}

const char* wsg_batcher_last_error(wsg_batcher* b) { return b ? b->err.c_str() : "null batcher"; }

// The session read loop over one session's region (StreamSession.java:798-854 over
// FrameDecoder.available, FrameDecoder.java:357-401): the region holds its carried
// partial frame and this feed's reads; every complete frame stays where it is (its
// offset is recorded), the header rules apply as soon as a header is complete
// (:197-256), and a partial tail is copied out to be carried.  Touches only session
// sid's state and region.
static void frame_region(wsg_batcher* b, FlushSlot& f, uint32_t sid, uint64_t start, uint64_t end) {
  SessIn& x = b->s[sid];
  const uint8_t* const ar = f.arena.p;
  uint64_t pos = start;
  for (;;) {
    const uint64_t rem = end - pos;
    uint8_t hdr[16] = {0};  // available() and the header rules read <= 14 bytes
    memcpy(hdr, ar + pos, rem < 14 ? rem : 14);
    int32_t e = 0;
    int64_t d1 = 0, d2 = 0;
    const int64_t r = wsg_frame_available(hdr, rem, &e, &d1, &d2);  // FrameDecoder.available
    if (r < 0) {  // the u64 length errors (:388-394)
      x.host_err = e;
      x.d1 = d1;
      x.d2 = d2;
      x.buf.clear();
      return;
    }
    if (r == 0) break;  // header incomplete
    const uint32_t hl = hdr_len(hdr);
    const int32_t he = wsg_check_header(&b->cfg, x.frag ? 1 : 0, hdr, hl, &d1);
    if (he && he != WSG_E_BATCH) {  // a header rule fails now (:197-256)
      x.host_err = he;
      x.d1 = d1;
      x.d2 = 0;
      x.buf.clear();
      return;
    }
    const uint64_t total = frame_total(hdr);
    if (rem < total) break;  // partial frame: carried (FrameDecoder.java:276-283)
    const uint32_t op = hdr[0] & 15u;
    if (op <= WSG_OP_BINARY) x.frag = !(hdr[0] & 0x80u);
    f.fo[sid].push_back(pos);
    f.fb[sid] += total;
    pos += total;
  }
  x.buf.assign(ar + pos, ar + end);
}

// Arena bytes on demand, keeping what is there (pinned: the H2D source)
static hipError_t arena_grow(FlushSlot& f, uint64_t need) {
  if (need <= f.arena.n && f.arena.p) return hipSuccess;
  PinnedBuf g;
  const hipError_t e = g.ensure(std::max<uint64_t>(need, 2 * (uint64_t)f.arena.n));
  if (e != hipSuccess) return e;
  if (f.arena_len) memcpy(g.p, f.arena.p, f.arena_len);
  f.arena.release();
  f.arena = g;
  return hipSuccess;
}

// Socket bytes into the pinned arena.  The arena is written once and then only read
// by the DMA engine, so the bulk goes out with streaming stores (no read-for-ownership
// of the destination lines, nothing of it left in the cache); the caller's
// synchronisation after the pool's run orders them (sfence here).
#if !defined(__HIP_DEVICE_COMPILE__)
__attribute__((target("avx2"))) static void copy_stream_avx2(uint8_t* d, const uint8_t* s, uint64_t n) {
  uint64_t h = (32u - ((uintptr_t)d & 31u)) & 31u;
  if (h > n) h = n;
  memcpy(d, s, h);
  d += h;
  s += h;
  n -= h;
  uint64_t i = 0;
  for (; i + 128 <= n; i += 128) {
    const __m256i x0 = _mm256_loadu_si256((const __m256i*)(s + i)), x1 = _mm256_loadu_si256((const __m256i*)(s + i + 32));
    const __m256i x2 = _mm256_loadu_si256((const __m256i*)(s + i + 64)), x3 = _mm256_loadu_si256((const __m256i*)(s + i + 96));
    _mm256_stream_si256((__m256i*)(d + i), x0);
    _mm256_stream_si256((__m256i*)(d + i + 32), x1);
    _mm256_stream_si256((__m256i*)(d + i + 64), x2);
    _mm256_stream_si256((__m256i*)(d + i + 96), x3);
  }
  memcpy(d + i, s + i, n - i);
  _mm_sfence();
}
static const bool g_avx2 = __builtin_cpu_supports("avx2");
static void copy_to_arena(uint8_t* d, const uint8_t* s, uint64_t n) {
  if (n >= 4096 && g_avx2) copy_stream_avx2(d, s, n);
  else memcpy(d, s, n);
}
#else  // (the device pass parses host code too)
static void copy_to_arena(uint8_t* d, const uint8_t* s, uint64_t n) { memcpy(d, s, n); }
#endif

// Many socket reads at once (a selector loop's reads of one iteration, in order):
// each session with reads gets one region of the open batch's pinned arena, its
// carried partial frame then its reads, copied there and framed in place by up to
// 16 threads (the sessions are independent): the bytes are copied once, into
// memory the DMA engines read.
static int stage_advance(wsg_batcher* b, bool collect);

int wsg_batcher_feed_many(wsg_batcher* b, uint32_t n, const uint32_t* sids, const uint8_t* const* data,
                          const uint64_t* lens) {
  if (!b || (n && (!sids || !data || !lens))) return WSG_API_EINVAL;
  const uint32_t S = b->n;
  for (uint32_t i = 0; i < n; ++i)
    if (sids[i] >= S || (lens[i] && !data[i])) return WSG_API_EINVAL;
  // the reads of each session, in order (a stable counting sort by session)
  std::vector<uint32_t> first(S + 1, 0), order(n);
  for (uint32_t i = 0; i < n; ++i) ++first[sids[i] + 1];
  for (uint32_t s = 0; s < S; ++s) first[s + 1] += first[s];
  {
    std::vector<uint32_t> at(first.begin(), first.end() - 1);
    for (uint32_t i = 0; i < n; ++i) order[at[sids[i]]++] = i;
  }
  FlushSlot& f = b->fs[b->open];
  // regions: the sessions that read, each its carried bytes + its reads.  A session
  // still inside one large frame after these reads only appends them to its carried
  // bytes (copying a growing partial frame into a region at every read would be
  // quadratic); the frame gets its region once complete.
  std::vector<uint32_t> ts, acc;
  std::vector<uint64_t> rs;  // region starts (then the end)
  uint64_t pos = f.arena_len;
  for (uint32_t s = 0; s < S; ++s) {
    if (first[s + 1] == first[s]) continue;
    const SessIn& x = b->s[s];
    if (b->state[s].closed || x.host_err || x.host_closed) continue;  // FrameDecoder.closed: input swallowed
    uint64_t add = 0;
    for (uint32_t j = first[s]; j < first[s + 1]; ++j) add += lens[order[j]];
    if (!add) continue;
    if (x.buf.size() >= 14 && x.buf.size() + add < frame_total(x.buf.data())) {
      acc.push_back(s);
      continue;
    }
    ts.push_back(s);
    rs.push_back(pos);
    pos += x.buf.size() + add;
  }
  for (uint32_t s : acc) {
    SessIn& x = b->s[s];
    for (uint32_t j = first[s]; j < first[s + 1]; ++j) {
      const uint32_t r = order[j];
      x.buf.insert(x.buf.end(), data[r], data[r] + lens[r]);
    }
  }
  if (ts.empty()) return WSG_API_OK;
  rs.push_back(pos);
  B_TRY(b, arena_grow(f, pos + 64));
  auto region = [&](uint32_t i) {
    const uint32_t s = ts[i];
    SessIn& x = b->s[s];
    uint8_t* d = f.arena.p + rs[i];
    if (!x.buf.empty()) copy_to_arena(d, x.buf.data(), x.buf.size());
    d += x.buf.size();
    for (uint32_t j = first[s]; j < first[s + 1]; ++j) {
      const uint32_t r = order[j];
      if (lens[r]) copy_to_arena(d, data[r], lens[r]);
      d += lens[r];
    }
    frame_region(b, f, s, rs[i], rs[i + 1]);
  };
  const uint64_t bytes = pos - f.arena_len;
  const uint32_t R = (uint32_t)ts.size();
  const uint32_t T = bytes < (4u << 20) ? 1u : std::min<uint32_t>(b->pool->size(), R);
  if (T <= 1) {
    for (uint32_t i = 0; i < R; ++i) region(i);
  } else {  // byte-balanced runs of regions, one a thread
    std::vector<uint32_t> cut(T + 1, R);
    cut[0] = 0;
    for (uint32_t t = 1; t < T; ++t) {
      const uint64_t target = f.arena_len + bytes * t / T;
      uint32_t i = cut[t - 1];
      while (i < R && rs[i + 1] <= target) ++i;
      cut[t] = i;
    }
    int side_rc = WSG_API_OK;
    const std::function<void()> side = [&] {  // (the only writer of b->err while the copies run)
      try {
        side_rc = stage_advance(b, true);
      } catch (const std::exception& ex) {  // never unwind past the pool's run: the workers use these frames
        side_rc = bset(b, WSG_API_ENOMEM, ex.what());
      } catch (...) {
        side_rc = bset(b, WSG_API_ENOMEM, "stage chain: unknown exception");
      }
    };
    const bool adv = b->has_stages && b->stage_early && b->feed_advance && !b->q.empty();
    b->pool->run(
        T, [&](uint32_t t) {
          for (uint32_t i = cut[t]; i < cut[t + 1]; ++i) region(i);
        },
        adv ? &side : nullptr);
    stage_defer(b, side_rc);
  }
  f.arena_len = pos;
  return WSG_API_OK;
}

int wsg_batcher_feed(wsg_batcher* b, uint32_t sid, const uint8_t* data, uint64_t len) {
  if (!b || sid >= b->n || (len && !data)) return WSG_API_EINVAL;
  return wsg_batcher_feed_many(b, 1, &sid, &data, &len);
}

// The carry state the next batch starts from: the previous batch's downloaded state
// (or the host copy when none is in flight) with the host's changes since applied.
static int stage_state(wsg_batcher* b) {
  const uint32_t S = b->n;
  B_TRY(b, b->st.ensure((S + 1) * sizeof(wsg_session_state)));
  wsg_session_state* st = (wsg_session_state*)b->st.p;
  if (b->q.empty()) {
    if (S) memcpy(st, b->state.data(), S * sizeof(wsg_session_state));
  } else {  // the state download of the batch in flight (it completes before its payload)
    B_TRY(b, ws::ctx_wait_prev_state(b->ctx));
  }
  for (const auto& pt : b->patch) {
    if (pt.second == 0) st[pt.first] = wsg_session_state{};  // a reset slot
    else st[pt.first].closed = 1;                            // failed on the host / by a stage
  }
  b->patch.clear();
  return WSG_API_OK;
}

// The queued flushes' stage chains started without blocking, from flush_async: the
// oldest flush whose predecessor is collected is begun once its decode is done (the
// replay + validator launched), the next one's pre-decode launched, so that the device
// inflates while the caller feeds the following reads instead of from the first
// wsg_batcher_wait on (a pipeline WSG_BATCHER_MAX_INFLIGHT flushes deep otherwise
// starts inflating only when it is full).  A decode not done yet is left to wait.
// With `collect` (from wsg_batcher_feed_many, on the calling thread while the pool's
// workers copy the reads): a begun chain whose inflate is done is collected too (its
// output gather queued), and the one behind it begun, so the chains move on during the
// feeds instead of only inside wsg_batcher_wait.  (The stage chain touches none of what
// the feed writes: the open slot, the sessions' carried input and host state.)
static void adjusted_results(wsg_batcher* b, const FlushSlot& g, std::vector<wsg_session_result>& r);
static int stage_compute(wsg_batcher* b, FlushSlot& f, const wsg_session_result* res);
static int stage_advance(wsg_batcher* b, bool collect) {
  bool pred_collected = true;  // (the flush before q[0] is)
  for (size_t qi = 0; qi < b->q.size(); ++qi) {
    FlushSlot& g = b->fs[b->q[qi]];
    if (g.so.staged) {
      pred_collected = true;
      continue;
    }
    if (!g.ij.prepped) {
      // (its pre-decode context was flush t - kTokCtx's: that one must be collected)
      if (qi >= (size_t)kTokCtx && !b->fs[b->q[qi - kTokCtx]].so.staged) break;
      const hipError_t e = hipEventQuery(g.done);
      if (e == hipErrorNotReady) break;
      B_TRY(b, e);
      std::vector<wsg_session_result> gres;
      adjusted_results(b, g, gres);
      int rc = stage_prep(b, g, gres.data());
      if (rc) return rc;
    }
    if (pred_collected && !g.ij.active) {
      int rc = stage_begin(b, g, nullptr);
      if (rc) return rc;
    }
    if (collect && pred_collected && b->stages.inflate && g.ij.active) {
      const hipError_t e = g.ij.todo.empty() ? hipSuccess : hipEventQuery(g.ij.launched);
      if (e != hipErrorNotReady) {
        B_TRY(b, e);
        int rc = stage_compute(b, g, nullptr);
        if (rc) return rc;
        continue;  // (staged: the next one may begin)
      }
    }
    pred_collected = false;
  }
  return WSG_API_OK;
}

int wsg_batcher_flush_async(wsg_batcher* b) {
  if (!b) return WSG_API_EINVAL;
  if (b->q.size() >= (size_t)kInflight)
    return bset(b, WSG_API_ERANGE, "WSG_BATCHER_MAX_INFLIGHT flushes in flight: wsg_batcher_wait first");
  const uint32_t S = b->n;
  int rc;
  const int slot = b->open;
  FlushSlot& f = b->fs[slot];
  // the batch's frames, session by session, where they landed
  uint64_t F = 0, W = 0;
  for (uint32_t i = 0; i < S; ++i) {
    F += f.fo[i].size();
    W += f.fb[i];
  }
  const uint64_t wl = f.arena_len;
  B_TRY(b, arena_grow(f, wl + 64));
  B_TRY(b, f.off.ensure((F + 1) * sizeof(uint64_t)));
  B_TRY(b, f.sf.ensure((S + 1) * sizeof(uint32_t)));
  const uint64_t pcap = wl + 16 * F + 16;
  if (!b->has_stages) B_TRY(b, f.payload.ensure(pcap));
  B_TRY(b, f.desc.ensure((F + 1) * sizeof(wsg_frame_desc)));
  B_TRY(b, f.result.ensure((S + 1) * sizeof(wsg_session_result)));
  if (!f.done) B_TRY(b, hipEventCreateWithFlags(&f.done, hipEventDisableTiming));
  uint64_t* off = (uint64_t*)f.off.p;
  uint32_t* sf = (uint32_t*)f.sf.p;
  uint64_t k = 0;
  for (uint32_t i = 0; i < S; ++i) {
    sf[i] = (uint32_t)k;
    for (uint64_t o : f.fo[i]) off[k++] = o;
  }
  sf[S] = (uint32_t)k;
  off[F] = wl;
  // a header error found on the host follows the frames fed so far: it is this batch's
  f.host_err.clear();
  for (uint32_t i = 0; i < S; ++i) {
    SessIn& x = b->s[i];
    if (x.host_err) {
      f.host_err.push_back({i, x.host_err, x.d1, x.d2});
      x.host_err = 0;
      x.host_closed = true;
      std::vector<uint8_t>().swap(x.buf);
    }
  }
  f.resets.clear();
  f.F = F;
  f.W = W;
  // the carry this batch starts from (waits for the previous batch's state download)
  rc = stage_state(b);
  if (rc) return rc;
  wsg_decoder_cfg cfg = b->cfg;
  cfg.flags |= WSG_CFG_SPARSE;
  // with stages the payloads stay on the device: copied (in stream order, before a later
  // batch can reuse the context's staging slot) to this flush's device region
  rc = wsg_decode_batch_host_async(b->ctx, &cfg, f.arena.p, wl, off, F, sf, S, (wsg_session_state*)b->st.p,
                                   b->has_stages ? nullptr : f.payload.p, pcap, (wsg_frame_desc*)f.desc.p,
                                   (wsg_session_result*)f.result.p);
  if (rc) return bset(b, rc, wsg_last_error(b->ctx));
  f.pcap = 0;
  if (b->has_stages && F) {
    if (!f.dpay_done) B_TRY(b, hipEventCreateWithFlags(&f.dpay_done, hipEventDisableTiming));
    B_TRY(b, f.dpay.ensure(pcap));
    B_TRY(b, hipMemcpyAsync(f.dpay.p, ws::ctx_async_payload(b->ctx), pcap, hipMemcpyDeviceToDevice,
                            ws::ctx_stream(b->ctx)));
    B_TRY(b, hipEventRecord(f.dpay_done, ws::ctx_stream(b->ctx)));
    f.pcap = pcap;
  }
  B_TRY(b, ws::ctx_record_out(b->ctx, f.done));
  f.ticket = b->tickets + 1;
  B_TRY(b, notify_after(ws::ctx_out_stream(b->ctx), b->notify, f.ticket));
  ++b->tickets;
  b->q.push_back(slot);
  // feeds go to the next slot (waited: at most two in flight)
  b->open = (b->open + 1) % (kInflight + 1);
  FlushSlot& g = b->fs[b->open];
  g.arena_len = 0;
  for (uint32_t i = 0; i < S; ++i) {
    g.fo[i].clear();
    g.fb[i] = 0;
  }
  if (b->has_stages && b->stage_early) stage_defer(b, stage_advance(b, false));  // (queued: OK from here on)
  return WSG_API_OK;
}

// A flush's decode results as wsg_batcher_wait hands them on: slots reset since are
// empty, host-detected header errors fill in for sessions the device did not fail.
static void adjusted_results(wsg_batcher* b, const FlushSlot& g, std::vector<wsg_session_result>& r) {
  const wsg_session_result* res = (const wsg_session_result*)g.result.p;
  r.assign(res, res + b->n);
  for (uint32_t sid : g.resets) r[sid] = wsg_session_result{};
  for (const auto& he : g.host_err) {
    if (std::find(g.resets.begin(), g.resets.end(), he.sid) != g.resets.end()) continue;
    if (!r[he.sid].error) {
      r[he.sid].error = (uint16_t)he.err;
      r[he.sid].close_code = WSG_CLOSE_PROTOCOL_ERROR;
      r[he.sid].detail = he.d1;
    }
  }
}

static int stage_advance_blocking(wsg_batcher* b) {
  int rc;
  // wsg_batcher_wait (eager mode): the chains of the flushes behind the one it collects,
  // advanced — blocking — so that the device works on them while
  // this flush's output downloads and while the caller feeds the next reads.  A chain
  // starts from the one before it (the frames of a message it left open, the sessions
  // a stage closed): it is begun only once its predecessor is collected.  So with a
  // flush behind the next one, the next one is collected and its output gather queued
  // (its inflate, begun in an earlier wait, ran meanwhile), then the one after it is
  // begun (inflate + validator launched, not waited for); the last flush in flight is
  // only begun.  A chain is begun from its flush's decode results, so those are waited
  // for (one flush's decode: short).
  // (two-phase inflate: every queued flush's pre-decode is launched first — flush t's
  // context was last used by flush t - kTokCtx, collected by now — so it runs meanwhile)
  for (size_t qi = 0; qi < b->q.size() && qi < 2; ++qi) {
    FlushSlot& g = b->fs[b->q[qi]];
    if (g.so.staged || g.ij.prepped) continue;
    B_TRY(b, hipEventSynchronize(g.done));
    std::vector<wsg_session_result> gres;
    adjusted_results(b, g, gres);
    if ((rc = stage_prep(b, g, gres.data()))) return rc;
  }
  for (size_t qi = 0; qi < b->q.size() && qi < 2; ++qi) {
    FlushSlot& g = b->fs[b->q[qi]];
    if (g.so.staged) continue;
    if (!g.ij.active && (rc = stage_begin(b, g, nullptr))) return rc;
    if (qi + 1 == b->q.size() || qi == 1) break;  // the last one: begun only
    if ((rc = stage_compute(b, g, nullptr))) return rc;
  }
  // (more pre-decode contexts than two: the pre-decodes of the flushes further back
  // whose decode is done)
  if (kTokCtx > 2 && b->stage_early) return stage_advance(b, false);
  return WSG_API_OK;
}

int wsg_batcher_wait(wsg_batcher* b, wsg_batch_view* out) {
  SP(9);
  if (!b || !out) return WSG_API_EINVAL;
  if (b->q.empty()) return bset(b, WSG_API_ERANGE, "no flush in flight");
  const int slot = b->q.front();
  b->q.pop_front();
  FlushSlot& f = b->fs[slot];
  B_TRY(b, hipEventSynchronize(f.done));
  if (b->stage_rc) {  // a stage step run on the side failed since the last wait
    const int rc = b->stage_rc;
    b->stage_rc = 0;
    b->err = b->stage_msg;
    return rc;
  }
  const uint32_t S = b->n;
  const wsg_session_state* st = (const wsg_session_state*)b->st.p;
  if (b->q.empty()) {  // the state after the last batch (else the newer batch owns the pinned copy)
    for (uint32_t i = 0; i < S; ++i) {
      const bool keep_closed = b->state[i].closed && !st[i].closed;  // latched on the host meanwhile
      b->state[i] = st[i];
      if (keep_closed) b->state[i].closed = 1;
    }
    for (const auto& pt : b->patch) {
      if (pt.second == 0) b->state[pt.first] = wsg_session_state{};
      else b->state[pt.first].closed = 1;
    }
  }
  wsg_session_result* res = (wsg_session_result*)f.result.p;
  for (uint32_t sid : f.resets) res[sid] = wsg_session_result{};  // a new session has the slot now
  f.detail2.assign(S, 0);
  // the host-detected header errors of the sessions the device did not fail first
  for (const auto& he : f.host_err) {
    const uint32_t i = he.sid;
    if (std::find(f.resets.begin(), f.resets.end(), i) != f.resets.end()) continue;
    if (!res[i].error) {
      res[i].error = (uint16_t)he.err;
      res[i].close_code = WSG_CLOSE_PROTOCOL_ERROR;  // every header / length rule closes with 1002
      res[i].detail = he.d1;
      f.detail2[i] = he.d2;
    }
    b->state[i].closed = 1;
    b->patch.push_back({i, 1});
  }
  out->n_frames = f.F;
  out->n_sessions = S;
  out->wire_bytes = f.W;
  out->session_first = (const uint32_t*)f.sf.p;
  out->desc = (const wsg_frame_desc*)f.desc.p;
  out->payload = f.payload.p;
  out->result = res;
  out->detail2 = f.detail2.data();
  out->reserved = 0;
  // a session failed by the device swallows further input
  for (uint32_t i = 0; i < S; ++i)
    if (res[i].error) {
      b->state[i].closed = 1;
      SessIn& x = b->s[i];
      std::vector<uint8_t>().swap(x.buf);
      x.host_closed = true;
    }
  if (!b->has_stages) return WSG_API_OK;
  int rc2 = f.so.staged ? WSG_API_OK : stage_compute(b, f, res);
  if (rc2) return rc2;
  if ((rc2 = stage_advance_blocking(b))) return rc2;
  if ((rc2 = stage_finish(b, f))) return rc2;
  StageOut& o = f.so;
  for (uint32_t sid : f.resets) o.res[sid] = wsg_session_result{};  // (also those reset after its stages ran)
  for (uint32_t i = 0; i < S; ++i) {
    if (o.res[i].error != res[i].error) f.detail2[i] = 0;  // (a stage's error has no second argument)
  }
  for (uint32_t i = 0; i < S; ++i)
    if (o.res[i].error && !res[i].error) {  // a stage failed it: the session swallows further input
      b->state[i].closed = 1;
      b->patch.push_back({i, 1});
      SessIn& x = b->s[i];
      std::vector<uint8_t>().swap(x.buf);
      x.host_err = 0;
      x.host_closed = true;
    }
  out->n_frames = o.desc.size();
  out->session_first = o.sf.data();
  out->desc = o.desc.data();
  out->payload = o.pay.p;
  out->result = o.res.data();
  return WSG_API_OK;
}

int wsg_batcher_flush(wsg_batcher* b, wsg_batch_view* out) {
  if (!b || !out) return WSG_API_EINVAL;
  while (!b->q.empty()) {  // (results of unwaited async flushes are dropped)
    wsg_batch_view v;
    int rc = wsg_batcher_wait(b, &v);
    if (rc) return rc;
  }
  int rc = wsg_batcher_flush_async(b);
  if (rc) return rc;
  return wsg_batcher_wait(b, out);
}

int wsg_batcher_set_stages(wsg_batcher* b, const wsg_stage_cfg* stages) {
  if (!b || !stages) return WSG_API_EINVAL;
  if (stages->aggregate && stages->max_aggregated_len < 0) return bset(b, WSG_API_EINVAL, "max_aggregated_len < 0");
  b->stages = *stages;
  b->has_stages = stages->inflate || stages->aggregate;
  // with inflate the text is validated after it (PerMessageDeflateExtension.java:316-326);
  // without, the validator is the fused check
  b->cfg.validate_utf8 = stages->inflate ? 0 : (stages->validate ? 1 : 0);
  const uint32_t S = b->n;
  b->ss.assign(S, StageSess{});
  b->stage_closed.assign(S, 0);
  b->stage_resets.clear();
  if (b->has_stages) {  // the device-resident stage carry, zeroed (fresh stage decoders)
    if (!b->sctx) {
      const int rc = wsg_open(ws::ctx_device(b->ctx), nullptr, &b->sctx);
      if (rc) return bset(b, rc, "wsg_open (stage context)");
    }
    ws::ctx_copy_tuning(b->sctx, b->ctx);  // (the batcher context's switches hold for its stages)
    b->two_phase = stages->inflate && ws::ctx_inflate_two_phase(b->ctx);
    for (int i = 0; b->two_phase && i < kTokCtx; ++i) {  // the pre-decode contexts (stream + workspace each)
      if (!b->tctx[i]) {
        const int rc = wsg_open(ws::ctx_device(b->ctx), nullptr, &b->tctx[i]);
        if (rc) return bset(b, rc, "wsg_open (pre-decode context)");
      }
      ws::ctx_copy_tuning(b->tctx[i], b->ctx);
    }
    hipStream_t st = ws::ctx_stream(b->sctx);
    B_TRY(b, b->d_istate.ensure(((uint64_t)S + 1) * sizeof(wsg_inflate_state)));
    B_TRY(b, b->d_iwin.ensure(((uint64_t)S + 1) * WSG_INFLATE_WINDOW));
    B_TRY(b, b->d_vstate.ensure(((uint64_t)S + 1) * sizeof(wsg_session_state)));
    B_TRY(b, b->d_astate.ensure(((uint64_t)S + 1) * sizeof(wsg_agg_state)));
    DBuf* z[] = {&b->d_istate, &b->d_iwin, &b->d_vstate, &b->d_astate};
    for (DBuf* d : z) B_TRY(b, hipMemsetAsync(d->p, 0, d->n, st));
    B_TRY(b, hipStreamSynchronize(st));
  }
  return WSG_API_OK;
}

uint64_t wsg_batcher_ticket(wsg_batcher* b) { return b ? b->tickets : 0; }

int64_t wsg_batcher_await(wsg_batcher* b, uint64_t seen, int64_t timeout_ms) {
  if (!b) return WSG_API_EINVAL;
  return notify_await(*b->notify, seen, timeout_ms);
}

// Every pinned and device buffer a flush of up to `max_wire` bytes and `max_frames`
// frames uses, in all three slots, sized now: such flushes allocate nothing (the
// stage chain's buffers, sized by what inflate and the aggregator produce, still
// grow on first use beyond this).
int wsg_batcher_reserve(wsg_batcher* b, uint64_t max_wire, uint64_t max_frames) {
  if (!b) return WSG_API_EINVAL;
  // growing a slot's buffers moves them: a flush in flight reads or writes them (its
  // H2D source, its D2H targets), so the batcher must be idle
  if (!b->q.empty()) return bset(b, WSG_API_ERANGE, "wsg_batcher_reserve: flushes in flight (wait for them first)");
  const uint32_t S = b->n;
  const uint64_t pcap = max_wire + 16 * max_frames + 16;
  b->res_wire = std::max(b->res_wire, max_wire);
  b->res_frames = std::max(b->res_frames, max_frames);
  B_TRY(b, b->st.ensure((S + 1) * sizeof(wsg_session_state)));
  for (FlushSlot& f : b->fs) {
    if (f.arena.n < max_wire + 64) B_TRY(b, arena_grow(f, max_wire + 64));
    B_TRY(b, f.off.ensure((max_frames + 1) * sizeof(uint64_t)));
    B_TRY(b, f.sf.ensure((S + 1) * sizeof(uint32_t)));
    if (!b->has_stages) B_TRY(b, f.payload.ensure(pcap));
    B_TRY(b, f.desc.ensure((max_frames + 1) * sizeof(wsg_frame_desc)));
    B_TRY(b, f.result.ensure((S + 1) * sizeof(wsg_session_result)));
    if (!f.done) B_TRY(b, hipEventCreateWithFlags(&f.done, hipEventDisableTiming));
    if (b->has_stages) {
      B_TRY(b, f.dpay.ensure(pcap));
      B_TRY(b, f.so.pay.ensure(pcap));
      if (!f.dpay_done) B_TRY(b, hipEventCreateWithFlags(&f.dpay_done, hipEventDisableTiming));
    }
  }
  return WSG_API_OK;
}

// The stage chain's buffers (wsg_batcher_set_stages) for flushes within the sizes of
// wsg_batcher_reserve whose stages produce up to max_out_bytes bytes in up to
// max_out_frames frames: the stage arena of every slot (decoded payloads | held frames |
// inflate's per-session output regions | aggregated bytes), the pinned output and its
// copy list, the descriptor and result lists each stage uploads and downloads, and the
// stage context's workspace.  A flush that stays within them allocates nothing; one
// beyond grows what it needs (an inflate that overflows its region is run again with a
// larger one).
int wsg_batcher_reserve_stages(wsg_batcher* b, uint64_t max_out_bytes, uint64_t max_out_frames) {
  if (!b) return WSG_API_EINVAL;
  if (!b->has_stages || !b->sctx) return bset(b, WSG_API_EINVAL, "wsg_batcher_reserve_stages: set the stages first");
  if (!b->q.empty()) return bset(b, WSG_API_ERANGE, "wsg_batcher_reserve_stages: flushes in flight (wait for them first)");
  const uint64_t S = b->n, W = b->res_wire, Fi = b->res_frames;
  const uint64_t Fo = std::max(max_out_frames, Fi);
  const uint64_t F = Fi + Fo + S + 1;               // a stage's frames: this flush's, held ones, one a session
  const uint64_t pcap = W + 16 * Fi + 16;            // the decoded payloads (flush_async's region)
  const uint64_t held = al16(W) + 16 * S;            // compressed frames of messages left open
  const uint64_t in_len = al16(pcap) + held;         // inflate's input: payloads and held frames
  // the inflate regions follow the expansion the caller sized its output for (max_out_bytes
  // over the wire bytes), not a fixed 8x: 8x of a 256 MB flush in each of the five slots
  // was tens of GB of HBM reserved for output the caller never expects
  const uint64_t ratio = std::min<uint64_t>(8, std::max<uint64_t>(2, (max_out_bytes + pcap - 1) / pcap));
  b->infl_ratio = (uint32_t)ratio;
  const uint64_t infl = b->stages.inflate ? S * (4096 + 16) + ratio * (in_len + 4 * F) : 0;
  const uint64_t maxo = std::max(max_out_bytes, pcap);
  const uint64_t agg = b->stages.aggregate ? al16(maxo + 16) : 0;  // (the aggregator's output only)
  const uint64_t arena = in_len + infl + agg + 256;
  const uint64_t out = maxo + 16 * Fo + 32;          // the handler's bytes, a 16-B slot a frame
  const uint64_t copies = maxo / COPY_MAX + Fo + S + 2;
  hipStream_t st = ws::ctx_stream(b->sctx);
  for (FlushSlot& f : b->fs) {
    B_TRY(b, f.dpay.grow_keep(arena, 0, st));
    B_TRY(b, f.so.pay.ensure(out));
    B_TRY(b, f.so.d_copy.ensure((copies + 1) * sizeof(StageCopy)));
    B_TRY(b, f.so.d_copy.up.ensure((copies + 1) * sizeof(StageCopy)));
    if (!f.dpay_done) B_TRY(b, hipEventCreateWithFlags(&f.dpay_done, hipEventDisableTiming));
    if (!f.so.gathered) B_TRY(b, hipEventCreateWithFlags(&f.so.gathered, hipEventDisableTiming));
    if (!f.so.downloaded) B_TRY(b, hipEventCreateWithFlags(&f.so.downloaded, hipEventDisableTiming));
  }
  B_TRY(b, dl_stream(b));
  struct Up {
    DBuf* d;
    uint64_t bytes;
  };
  const Up ups[] = {{&b->d_desc, (F + 1) * sizeof(wsg_frame_desc)}, {&b->d_sf, (S + 2) * sizeof(uint32_t)},
                    {&b->d_ooff, (S + 2) * sizeof(uint64_t)},      {&b->d_res, (S + 1) * sizeof(wsg_session_result)},
                    {&b->d_resets, (S + 1) * sizeof(uint32_t)},    {&b->d_pend, (copies + 1) * sizeof(StageCopy)},
                    {&b->d_nheld, (S + 1) * sizeof(uint32_t)}};
  for (const Up& u : ups) {
    B_TRY(b, u.d->ensure(u.bytes));
    B_TRY(b, u.d->up.ensure(u.bytes));
  }
  B_TRY(b, b->d_odesc.ensure((F + S + 1) * sizeof(wsg_frame_desc)));
  B_TRY(b, b->d_ores.ensure((S + 1) * sizeof(wsg_session_result)));
  B_TRY(b, b->d_rf.ensure((S + 1) * sizeof(uint32_t)));
  B_TRY(b, b->d_tot.ensure(sizeof(uint64_t)));
  B_TRY(b, b->d_vdesc.ensure((F + 1) * sizeof(wsg_frame_desc)));
  B_TRY(b, b->d_vres.ensure((S + 1) * sizeof(wsg_session_result)));
  B_TRY(b, b->h_vres.ensure((S + 1) * sizeof(wsg_session_result)));
  B_TRY(b, b->h_odesc.ensure((F + S + 1) * sizeof(wsg_frame_desc)));
  B_TRY(b, b->h_ores.ensure((S + 1) * sizeof(wsg_session_result)));
  B_TRY(b, b->h_rf.ensure((S + 1) * sizeof(uint32_t)));
  B_TRY(b, b->h_astate.ensure((S + 1) * sizeof(wsg_agg_state)));
  B_TRY(b, b->h_pend.ensure(maxo + 16 * S + 32));
  const int rc = ws::ctx_reserve_stages(b->sctx, F, (uint32_t)S, in_len + infl, agg);
  if (rc) return bset(b, rc, wsg_last_error(b->sctx));
  for (int i = 0; b->two_phase && i < kTokCtx; ++i) {  // the pre-decodes: a flush's decoded frames and payloads
    const int rc2 = wsg_reserve_inflate(b->tctx[i], Fi + 1, (uint32_t)S, al16(pcap));
    if (rc2) return bset(b, rc2, wsg_last_error(b->tctx[i]));
    B_TRY(b, b->d_tdesc[i].ensure((Fi + 2) * sizeof(wsg_frame_desc)));
    B_TRY(b, b->d_tdesc[i].up.ensure((Fi + 2) * sizeof(wsg_frame_desc)));
    B_TRY(b, b->d_tsf[i].ensure((S + 2) * sizeof(uint32_t)));
    B_TRY(b, b->d_tsf[i].up.ensure((S + 2) * sizeof(uint32_t)));
  }
  B_TRY(b, b->d_tmap.ensure((F + 1) * sizeof(uint32_t)));
  B_TRY(b, b->d_tmap.up.ensure((F + 1) * sizeof(uint32_t)));
  for (FlushSlot& f : b->fs) {
    if (!f.ij.tok_done) B_TRY(b, hipEventCreateWithFlags(&f.ij.tok_done, hipEventDisableTiming));
    if (!f.ij.launched) B_TRY(b, hipEventCreateWithFlags(&f.ij.launched, hipEventDisableTiming));
  }
  B_TRY(b, hipStreamSynchronize(st));
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
  FlushSlot& f = b->fs[b->open];  // its frames fed since the last flush are dropped (gaps now)
  f.fo[sid].clear();
  f.fb[sid] = 0;
  x.frag = false;
  x.host_err = 0;
  x.d1 = x.d2 = 0;
  x.host_closed = false;
  b->state[sid] = wsg_session_state{};
  for (int slot : b->q) b->fs[slot].resets.push_back(sid);  // the old session's results in flight are dropped
  b->patch.push_back({sid, 0});
  if (b->has_stages) {  // fresh stage decoders too (the device carry is zeroed before the next stage run)
    b->ss[sid] = StageSess{};
    b->stage_closed[sid] = 0;
    b->stage_resets.push_back(sid);
  }
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
// One encode flush's pinned staging and device buffers (three: one being filled by
// add(), up to two in flight).
struct EncSlot {
  PinnedBuf arena, frames, sf, cl, wire, off, ddesc;
  uint64_t arena_len = 0, F = 0, need = 0;
  DBuf d_pay, d_frames, d_sf, d_cl, d_off, d_ddesc, d_odesc;
  hipEvent_t ev_in = nullptr, ev_k = nullptr, ev_out = nullptr;
  std::vector<uint32_t> resets;  // sessions reset while this flush was in flight: their bytes are dropped
  // the view with those sessions' frames left out (built only when there are some)
  std::vector<uint32_t> v_sf;
  std::vector<uint64_t> v_off;
  std::vector<uint8_t> v_wire;
};

struct wsg_enc_batcher {
  wsg_ctx* ctx = nullptr;
  int client = 0;
  uint32_t n = 0;
  std::vector<uint8_t> closed;           // FrameEncoder.closed per session, as of the frames flushed so far
  std::vector<uint32_t> rec_sid;         // session of each queued frame, arrival order
  std::vector<wsg_encode_frame> rec;     // queued frames, arrival order
  std::vector<uint32_t> count;           // queued frames per session
  EncSlot es[3];
  int open = 0;                          // the slot add() fills
  std::deque<int> q;                     // flushes in flight, oldest first
  hipStream_t s_in = nullptr, s_out = nullptr;  // uploads / downloads (kernels on the context's stream)
  std::unique_ptr<Pool> pool;                   // add_many's copies
  std::string err;
  uint64_t tickets = 0;                         // flushes queued so far
  std::shared_ptr<Notify> notify = std::make_shared<Notify>();
  // permessage-deflate before the encoder (wsg_enc_batcher_set_deflate): level < 0 off;
  // the deflater state and window | head | prev of every session, on the device
  int defl_level = -1, defl_nc = 0;
  DBuf d_dstate, d_dmem;
};

// Frame k's encode record from the deflate stage's output descriptor: the payload to frame
// is the compressed one (in the out region, `out_base` bytes into the payload buffer) or the
// frame's own, with the RSV bits the PerMessageDeflateEncoder gave it; the mask stays.
__global__ __launch_bounds__(256) void k_enc_from_defl(const wsg_frame_desc* __restrict__ od,
                                                       wsg_encode_frame* __restrict__ fr, uint64_t n,
                                                       uint64_t out_base) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const wsg_frame_desc d = od[k];
  wsg_encode_frame f = fr[k];
  f.payload_off = (d.flags & WSG_DESC_DEFLATED) ? out_base + d.payload_off : d.payload_off;
  f.payload_len = d.payload_len;
  f.opcode = d.opcode;
  f.flags = d.flags & 0xF0;
  fr[k] = f;
}

static inline uint64_t java_bound_h(uint64_t len) { return len + ((len + 7) >> 3) + ((len + 63) >> 6) + 15; }

static int eset(wsg_enc_batcher* b, int code, const char* msg) {
  if (b) b->err = msg ? msg : "";
  return code;
}
#define E_TRY(b, expr)                                                           \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    if (_e != hipSuccess) return eset((b), WSG_API_EHIP, hipGetErrorString(_e)); \
  } while (0)

int wsg_enc_batcher_open(wsg_ctx* ctx, int client_mode, uint32_t n_sessions, wsg_enc_batcher** out) {
  if (!ctx || !out) return WSG_API_EINVAL;
  wsg_enc_batcher* b = new wsg_enc_batcher();
  b->ctx = ctx;
  b->client = client_mode ? 1 : 0;
  b->n = n_sessions;
  b->closed.assign(n_sessions, 0);
  b->count.assign(n_sessions, 0);
  const unsigned hw = std::thread::hardware_concurrency();
  b->pool.reset(new Pool((hw ? std::min(16u, hw) : 8u) - 1));
  *out = b;
  return WSG_API_OK;
}

int wsg_enc_batcher_close(wsg_enc_batcher* b) {
  if (!b) return WSG_API_EINVAL;
  (void)wsg_sync(b->ctx);
  if (b->s_in) (void)hipStreamSynchronize(b->s_in);
  if (b->s_out) (void)hipStreamSynchronize(b->s_out);
  for (EncSlot& e : b->es) {
    PinnedBuf* bufs[] = {&e.arena, &e.frames, &e.sf, &e.cl, &e.wire, &e.off, &e.ddesc};
    for (PinnedBuf* p : bufs) p->release();
    DBuf* dbufs[] = {&e.d_pay, &e.d_frames, &e.d_sf, &e.d_cl, &e.d_off, &e.d_ddesc, &e.d_odesc};
    for (DBuf* d : dbufs) d->release();
    hipEvent_t evs[] = {e.ev_in, e.ev_k, e.ev_out};
    for (hipEvent_t v : evs)
      if (v) (void)hipEventDestroy(v);
  }
  b->d_dstate.release();
  b->d_dmem.release();
  if (b->s_in) (void)hipStreamDestroy(b->s_in);
  if (b->s_out) (void)hipStreamDestroy(b->s_out);
  delete b;
  return WSG_API_OK;
}

// PerMessageDeflateEncoder(level, noContext) in front of the encoder for every session
// (PerMessageDeflateExtension.updateEncoders, PerMessageDeflateExtension.java:303-313): the
// state of a new deflater per session (zeros), its window and hash arrays on the device.
int wsg_enc_batcher_set_deflate(wsg_enc_batcher* b, int level, int no_context) {
  if (!b) return WSG_API_EINVAL;
  if (level < 0 || level > 9) return eset(b, WSG_API_EINVAL, "compression level is out of range");
  if (!b->q.empty() || !b->rec.empty() || b->defl_level >= 0)
    return eset(b, WSG_API_ERANGE, "wsg_enc_batcher_set_deflate: once, before the first add");
  E_TRY(b, hipSetDevice(ws::ctx_device(b->ctx)));
  const uint64_t S = b->n ? b->n : 1;
  E_TRY(b, b->d_dstate.ensure(S * sizeof(wsg_deflate_state)));
  E_TRY(b, b->d_dmem.ensure(S * (uint64_t)WSG_DEFLATE_SESSION_BYTES));
  E_TRY(b, hipMemsetAsync(b->d_dstate.p, 0, S * sizeof(wsg_deflate_state), ws::ctx_stream(b->ctx)));
  b->defl_level = level;
  b->defl_nc = no_context ? 1 : 0;
  return WSG_API_OK;
}

const char* wsg_enc_batcher_last_error(wsg_enc_batcher* b) { return b ? b->err.c_str() : "null batcher"; }

// Many frames at once (a loop iteration's writes): placed in arrival order as add()
// places them, the payload copies spread over the pool (streaming stores, as the
// decode feed's) when there are megabytes of them.
int wsg_enc_batcher_add_many(wsg_enc_batcher* b, uint32_t n, const uint32_t* sids, const uint8_t* opcodes,
                             const uint8_t* flags, const uint8_t* masks, const uint8_t* const* payloads,
                             const uint32_t* lens) {
  if (!b || (n && (!sids || !opcodes || !flags || !payloads || !lens))) return WSG_API_EINVAL;
  for (uint32_t i = 0; i < n; ++i)
    if (sids[i] >= b->n || (lens[i] && !payloads[i])) return WSG_API_EINVAL;
  EncSlot& e = b->es[b->open];
  std::vector<uint64_t> at(n, ~0ull);
  uint64_t pos = e.arena_len, bytes = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (b->closed[sids[i]]) continue;  // FrameEncoder.java:71-76
    at[i] = (pos + 15) & ~15ull;
    pos = at[i] + lens[i];
    bytes += lens[i];
  }
  if (pos + 16 > e.arena.n) {
    PinnedBuf g;
    if (g.ensure(std::max<uint64_t>(pos + 16, 2 * e.arena.n)) != hipSuccess)
      return eset(b, WSG_API_ENOMEM, "pinned arena");
    if (e.arena_len) memcpy(g.p, e.arena.p, e.arena_len);
    e.arena.release();
    e.arena = g;
  }
  const uint32_t T = bytes < (4u << 20) ? 1u : std::min<uint32_t>(b->pool->size(), n);
  auto copy = [&](uint32_t i) {
    if (at[i] != ~0ull && lens[i]) copy_to_arena(e.arena.p + at[i], payloads[i], lens[i]);
  };
  if (T <= 1) {
    for (uint32_t i = 0; i < n; ++i) copy(i);
  } else {
    b->pool->run(T, [&](uint32_t t) {
      for (uint32_t i = (uint32_t)((uint64_t)n * t / T); i < (uint32_t)((uint64_t)n * (t + 1) / T); ++i) copy(i);
    });
  }
  for (uint32_t i = 0; i < n; ++i) {
    if (at[i] == ~0ull) continue;
    wsg_encode_frame f{};
    f.payload_off = at[i];
    f.payload_len = lens[i];
    f.opcode = opcodes[i];
    f.flags = flags[i];
    if (masks) memcpy(f.mask, masks + 4 * (uint64_t)i, 4);
    b->rec.push_back(f);
    b->rec_sid.push_back(sids[i]);
    ++b->count[sids[i]];
  }
  e.arena_len = pos;
  return WSG_API_OK;
}

int wsg_enc_batcher_add(wsg_enc_batcher* b, uint32_t sid, uint8_t opcode, uint8_t flags, const uint8_t* mask,
                        const uint8_t* payload, uint32_t len) {
  if (!b || sid >= b->n || (len && !payload)) return WSG_API_EINVAL;
  if (b->closed[sid]) return WSG_API_OK;  // FrameEncoder.java:71-76: nothing after a CLOSE (latched earlier)
  EncSlot& e = b->es[b->open];
  const uint64_t at = (e.arena_len + 15) & ~15ull;
  if (at + len + 16 > e.arena.n) {  // grow, keeping what is queued (pinned: the H2D source)
    PinnedBuf g;
    if (g.ensure(std::max<uint64_t>(at + len + 16, 2 * e.arena.n)) != hipSuccess)
      return eset(b, WSG_API_ENOMEM, "pinned arena");
    if (e.arena_len) memcpy(g.p, e.arena.p, e.arena_len);
    e.arena.release();
    e.arena = g;
  }
  if (len) memcpy(e.arena.p + at, payload, len);
  e.arena_len = at + len;
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

// Queue the encode of everything added since the last flush: frames ordered by session
// (stable), H2D on the batcher's upload stream, the kernels on the context's stream,
// D2H on its download stream.  The close latch a batch starts from is known on the
// host (a CLOSE frame latches its session for every later frame, FrameEncoder.java:
// 71-76), so the next batch can be queued before this one comes back.
int wsg_enc_batcher_flush_async(wsg_enc_batcher* b) {
  if (!b) return WSG_API_EINVAL;
  if (b->q.size() >= 2) return eset(b, WSG_API_ERANGE, "two flushes in flight: wsg_enc_batcher_wait first");
  const uint32_t S = b->n;
  const uint64_t F = b->rec.size();
  const int slot = b->open;
  EncSlot& e = b->es[slot];
  E_TRY(b, hipSetDevice(ws::ctx_device(b->ctx)));
  if (!b->s_in) E_TRY(b, hipStreamCreateWithFlags(&b->s_in, hipStreamNonBlocking));
  if (!b->s_out) E_TRY(b, hipStreamCreateWithFlags(&b->s_out, hipStreamNonBlocking));
  hipEvent_t* evs[] = {&e.ev_in, &e.ev_k, &e.ev_out};
  for (hipEvent_t* v : evs)
    if (!*v) E_TRY(b, hipEventCreateWithFlags(v, hipEventDisableTiming));
  E_TRY(b, e.frames.ensure((F + 1) * sizeof(wsg_encode_frame)));
  E_TRY(b, e.sf.ensure((S + 1) * sizeof(uint32_t)));
  E_TRY(b, e.cl.ensure(S + 1));
  E_TRY(b, e.off.ensure((F + 1) * sizeof(uint64_t)));
  uint32_t* sf = (uint32_t*)e.sf.p;
  sf[0] = 0;
  for (uint32_t i = 0; i < S; ++i) sf[i + 1] = sf[i] + b->count[i];
  {  // stable counting sort of the records by session
    std::vector<uint32_t> pos(sf, sf + S);
    wsg_encode_frame* fr = (wsg_encode_frame*)e.frames.p;
    for (uint64_t k = 0; k < F; ++k) fr[pos[b->rec_sid[k]]++] = b->rec[k];
  }
  const bool defl = b->defl_level >= 0;
  ws::DeflBounds bounds;
  uint64_t need = 0;
  if (!defl) {
    for (uint64_t k = 0; k < F; ++k) need += wsg_encoded_length(b->rec[k].payload_len, b->client);
  } else {  // a compressed payload is at most ZlibEncoder.deflateBound(len) bytes
    E_TRY(b, e.ddesc.ensure((F + 1) * sizeof(wsg_frame_desc)));
    const wsg_encode_frame* fr = (const wsg_encode_frame*)e.frames.p;
    wsg_frame_desc* dd = (wsg_frame_desc*)e.ddesc.p;
    for (uint64_t k = 0; k < F; ++k) {
      dd[k] = wsg_frame_desc{fr[k].payload_off, fr[k].payload_len, fr[k].opcode, fr[k].flags, 0};
      need += wsg_encoded_length(java_bound_h(fr[k].payload_len), b->client);
      ws::deflate_bounds_add(bounds, fr[k].payload_len);
    }
    for (uint32_t i = 0; i < S; ++i)
      if (b->count[i]) ws::deflate_bounds_session(bounds);
  }
  E_TRY(b, e.wire.ensure(need + 32));
  if (S) memcpy(e.cl.p, b->closed.data(), S);
  for (uint64_t k = 0; k < F; ++k)  // the latch the next batch starts from
    if (b->rec[k].opcode == WSG_OP_CLOSE) b->closed[b->rec_sid[k]] = 1;
  // with deflate the compressed payloads follow the arena in the same device buffer
  const uint64_t out_base = (e.arena_len + 255) & ~255ull, out_cap = defl ? bounds.tot[1] : 0;
  E_TRY(b, e.d_pay.ensure(defl ? out_base + out_cap + 64 : e.arena_len + 32));
  E_TRY(b, e.d_frames.ensure((F + 1) * sizeof(wsg_encode_frame)));
  E_TRY(b, e.d_sf.ensure((S + 1) * sizeof(uint32_t)));
  E_TRY(b, e.d_cl.ensure(S + 1));
  // The kernels write the wire straight into the pinned host buffer (PCIe writes from
  // the encode kernel itself), not to the device for a runtime D2H: that D2H is a blit
  // kernel on the download stream, and where the runtime places the batcher's streams
  // on the process's hardware queues decided whether it overlapped the next flush's
  // upload — 26.6-29.5 GiB/s against 39.3-40.5 on the e2e encode line depending on the
  // streams created before it; written directly, 36.1-37.8 whatever the placement
  // (profiles/r05_ab/r05ad_ab_encdirect.txt).
  uint8_t* wire_out = nullptr;
  E_TRY(b, hipHostGetDevicePointer((void**)&wire_out, e.wire.p, 0));
  E_TRY(b, e.d_off.ensure((F + 1) * sizeof(uint64_t)));
  if (e.arena_len) E_TRY(b, hipMemcpyAsync(e.d_pay.p, e.arena.p, e.arena_len, hipMemcpyHostToDevice, b->s_in));
  if (F) E_TRY(b, hipMemcpyAsync(e.d_frames.p, e.frames.p, F * sizeof(wsg_encode_frame), hipMemcpyHostToDevice, b->s_in));
  E_TRY(b, hipMemcpyAsync(e.d_sf.p, e.sf.p, (S + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, b->s_in));
  if (S) E_TRY(b, hipMemcpyAsync(e.d_cl.p, e.cl.p, S, hipMemcpyHostToDevice, b->s_in));
  if (defl) {
    E_TRY(b, e.d_ddesc.ensure((F + 1) * sizeof(wsg_frame_desc)));
    E_TRY(b, e.d_odesc.ensure((F + 1) * sizeof(wsg_frame_desc)));
    if (F) E_TRY(b, hipMemcpyAsync(e.d_ddesc.p, e.ddesc.p, F * sizeof(wsg_frame_desc), hipMemcpyHostToDevice, b->s_in));
  }
  E_TRY(b, hipEventRecord(e.ev_in, b->s_in));
  hipStream_t ks = ws::ctx_stream(b->ctx);
  E_TRY(b, hipStreamWaitEvent(ks, e.ev_in, 0));
  int rc;
  if (defl && F) {  // the permessage-deflate-encoder stage, then the frames it hands on
    rc = ws::deflate_launch(b->ctx, b->defl_level, b->defl_nc, (const wsg_frame_desc*)e.d_ddesc.p, F,
                            (const uint32_t*)e.d_sf.p, S, e.d_pay.p, (wsg_deflate_state*)b->d_dstate.p,
                            b->d_dmem.p, e.d_pay.p + out_base, out_cap, (wsg_frame_desc*)e.d_odesc.p, &bounds,
                            nullptr);
    if (rc) return eset(b, rc, wsg_last_error(b->ctx));
    hipLaunchKernelGGL(k_enc_from_defl, dim3((uint32_t)((F + 255) / 256)), dim3(256), 0, ks,
                       (const wsg_frame_desc*)e.d_odesc.p, (wsg_encode_frame*)e.d_frames.p, F, out_base);
    E_TRY(b, hipGetLastError());
  }
  rc = wsg_encode_batch_device(b->ctx, b->client, e.d_pay.p, defl ? out_base + out_cap : e.arena_len,
                               (const wsg_encode_frame*)e.d_frames.p, F, (const uint32_t*)e.d_sf.p, S, e.d_cl.p,
                               wire_out, need + 32, (uint64_t*)e.d_off.p);
  if (rc) return eset(b, rc, wsg_last_error(b->ctx));
  if (!F) E_TRY(b, hipMemsetAsync(e.d_off.p, 0, sizeof(uint64_t), ks));
  E_TRY(b, hipEventRecord(e.ev_k, ks));
  E_TRY(b, hipStreamWaitEvent(b->s_out, e.ev_k, 0));
  E_TRY(b, hipMemcpyAsync(e.off.p, e.d_off.p, (F + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, b->s_out));
  // (the kept frames' bytes are at most `need`: frames dropped after a CLOSE take none)
  E_TRY(b, hipEventRecord(e.ev_out, b->s_out));
  E_TRY(b, notify_after(b->s_out, b->notify, b->tickets + 1));
  ++b->tickets;
  e.F = F;
  e.need = need;
  e.resets.clear();
  b->q.push_back(slot);
  b->rec.clear();
  b->rec_sid.clear();
  std::fill(b->count.begin(), b->count.end(), 0u);
  b->open = (b->open + 1) % 3;
  b->es[b->open].arena_len = 0;
  return WSG_API_OK;
}

// The oldest encode flush in flight: session s's wire bytes are
// wire[off[sf[s]], off[sf[s+1]]).  Valid until that slot is reused (two flushes later).
int wsg_enc_batcher_wait(wsg_enc_batcher* b, wsg_enc_view* out) {
  if (!b || !out) return WSG_API_EINVAL;
  if (b->q.empty()) return eset(b, WSG_API_ERANGE, "no encode flush in flight");
  const int slot = b->q.front();
  b->q.pop_front();
  EncSlot& e = b->es[slot];
  E_TRY(b, hipEventSynchronize(e.ev_out));
  const uint32_t S = b->n;
  const uint64_t F = e.F;
  const uint32_t* sf = (const uint32_t*)e.sf.p;
  const uint64_t* off = (const uint64_t*)e.off.p;
  out->n_frames = F;
  out->wire_bytes = off[F];
  out->n_sessions = S;
  out->reserved = 0;
  out->session_first = sf;
  out->wire_off = off;
  out->wire = e.wire.p;
  if (e.resets.empty()) return WSG_API_OK;
  // a slot handed to a new session while this flush was in flight: the old session's
  // frames are left out (their bytes must not reach the new session)
  std::vector<uint8_t> drop(S, 0);
  for (uint32_t s : e.resets) drop[s] = 1;
  e.v_sf.assign(S + 1, 0);
  e.v_off.assign(1, 0);
  e.v_wire.clear();
  for (uint32_t s = 0; s < S; ++s) {
    e.v_sf[s] = (uint32_t)(e.v_off.size() - 1);
    if (drop[s]) continue;
    for (uint32_t k = sf[s]; k < sf[s + 1]; ++k) {
      e.v_wire.insert(e.v_wire.end(), e.wire.p + off[k], e.wire.p + off[k + 1]);
      e.v_off.push_back(e.v_wire.size());
    }
  }
  e.v_sf[S] = (uint32_t)(e.v_off.size() - 1);
  out->n_frames = e.v_off.size() - 1;
  out->wire_bytes = e.v_wire.size();
  out->session_first = e.v_sf.data();
  out->wire_off = e.v_off.data();
  out->wire = e.v_wire.data();
  return WSG_API_OK;
}

int wsg_enc_batcher_flush(wsg_enc_batcher* b, wsg_enc_view* out) {
  if (!b || !out) return WSG_API_EINVAL;
  while (!b->q.empty()) {  // (views of unwaited async flushes are dropped)
    wsg_enc_view v;
    const int rc = wsg_enc_batcher_wait(b, &v);
    if (rc) return rc;
  }
  const int rc = wsg_enc_batcher_flush_async(b);
  if (rc) return rc;
  return wsg_enc_batcher_wait(b, out);
}

uint64_t wsg_enc_batcher_ticket(wsg_enc_batcher* b) { return b ? b->tickets : 0; }

int64_t wsg_enc_batcher_await(wsg_enc_batcher* b, uint64_t seen, int64_t timeout_ms) {
  if (!b) return WSG_API_EINVAL;
  return notify_await(*b->notify, seen, timeout_ms);
}

// The pinned and device buffers of all three slots for flushes of up to `max_frames`
// frames and `max_payload` payload bytes: such flushes allocate nothing.
int wsg_enc_batcher_reserve(wsg_enc_batcher* b, uint64_t max_frames, uint64_t max_payload) {
  if (!b) return WSG_API_EINVAL;
  if (!b->q.empty()) return eset(b, WSG_API_ERANGE, "wsg_enc_batcher_reserve: flushes in flight (wait for them first)");
  const uint32_t S = b->n;
  const uint64_t arena = max_payload + 16 * max_frames + 32;  // 16-B aligned payloads
  const uint64_t need = max_payload + 14 * max_frames + 32;   // the longest header is 14 B
  for (EncSlot& e : b->es) {
    if (e.arena.n < arena) {
      PinnedBuf g;
      if (g.ensure(arena) != hipSuccess) return eset(b, WSG_API_ENOMEM, "pinned arena");
      if (e.arena_len) memcpy(g.p, e.arena.p, e.arena_len);
      e.arena.release();
      e.arena = g;
    }
    E_TRY(b, e.frames.ensure((max_frames + 1) * sizeof(wsg_encode_frame)));
    E_TRY(b, e.sf.ensure((S + 1) * sizeof(uint32_t)));
    E_TRY(b, e.cl.ensure(S + 1));
    E_TRY(b, e.off.ensure((max_frames + 1) * sizeof(uint64_t)));
    E_TRY(b, e.wire.ensure(need + 32));
    if (b->defl_level >= 0) {  // the compressed payloads after the arena, their descriptors
      const uint64_t out = java_bound_h(max_payload) + 32 * max_frames;
      E_TRY(b, e.d_pay.ensure(((arena + 255) & ~255ull) + out + 64));
      E_TRY(b, e.wire.ensure(out + 14 * max_frames + 32));
      E_TRY(b, e.ddesc.ensure((max_frames + 1) * sizeof(wsg_frame_desc)));
      E_TRY(b, e.d_ddesc.ensure((max_frames + 1) * sizeof(wsg_frame_desc)));
      E_TRY(b, e.d_odesc.ensure((max_frames + 1) * sizeof(wsg_frame_desc)));
    }
    E_TRY(b, e.d_pay.ensure(arena + 32));
    E_TRY(b, e.d_frames.ensure((max_frames + 1) * sizeof(wsg_encode_frame)));
    E_TRY(b, e.d_sf.ensure((S + 1) * sizeof(uint32_t)));
    E_TRY(b, e.d_cl.ensure(S + 1));
    E_TRY(b, e.d_off.ensure((max_frames + 1) * sizeof(uint64_t)));
  }
  return WSG_API_OK;
}

uint64_t wsg_batcher_alloc_count(void) { return g_batcher_allocs.load() + ws::ctx_alloc_count(); }

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
  for (int slot : b->q) b->es[slot].resets.push_back(sid);
  if (b->defl_level >= 0)  // a new deflater (in stream order: after the flushes in flight)
    E_TRY(b, hipMemsetAsync((wsg_deflate_state*)b->d_dstate.p + sid, 0, sizeof(wsg_deflate_state),
                            ws::ctx_stream(b->ctx)));
  return WSG_API_OK;
}

// ------------------------------------------------------------------ device per selector loop
// One device per loop: the sessions of a loop share its batcher, and
// nothing is shared between devices.  A new loop goes to the device with the fewest
// loops, ties to the one with the fewest wire bytes accounted so far.
static std::mutex g_dev_mu;
static std::vector<uint32_t> g_dev_loops;
static std::vector<uint64_t> g_dev_bytes;
static std::map<uint64_t, int> g_dev_of;

static int dev_init_locked() {
  if (!g_dev_loops.empty()) return (int)g_dev_loops.size();
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return 0;
  g_dev_loops.assign((size_t)n, 0);
  g_dev_bytes.assign((size_t)n, 0);
  return n;
}

int wsg_device_policy_init(int n_devices) {
  if (n_devices <= 0) return WSG_API_EINVAL;
  std::lock_guard<std::mutex> g(g_dev_mu);
  g_dev_loops.assign((size_t)n_devices, 0);
  g_dev_bytes.assign((size_t)n_devices, 0);
  g_dev_of.clear();
  return WSG_API_OK;
}

int wsg_device_for_loop(uint64_t loop_id) {
  std::lock_guard<std::mutex> g(g_dev_mu);
  auto it = g_dev_of.find(loop_id);
  if (it != g_dev_of.end()) return it->second;
  const int n = dev_init_locked();
  if (n <= 0) return WSG_API_EHIP;
  int best = 0;
  for (int i = 1; i < n; ++i)
    if (g_dev_loops[i] < g_dev_loops[best] || (g_dev_loops[i] == g_dev_loops[best] && g_dev_bytes[i] < g_dev_bytes[best]))
      best = i;
  ++g_dev_loops[best];
  g_dev_of[loop_id] = best;
  return best;
}

int wsg_device_account(int device, uint64_t wire_bytes) {
  std::lock_guard<std::mutex> g(g_dev_mu);
  if (device < 0 || (size_t)device >= g_dev_bytes.size()) return WSG_API_EINVAL;
  g_dev_bytes[(size_t)device] += wire_bytes;
  return WSG_API_OK;
}

int wsg_device_release_loop(uint64_t loop_id) {
  std::lock_guard<std::mutex> g(g_dev_mu);
  auto it = g_dev_of.find(loop_id);
  if (it == g_dev_of.end()) return WSG_API_EINVAL;
  --g_dev_loops[(size_t)it->second];
  g_dev_of.erase(it);
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
