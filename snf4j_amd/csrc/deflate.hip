// deflate.hip — permessage-deflate compression on the GPU: PerMessageDeflateEncoder
// (PerMessageDeflateEncoder.java:55-99) over DeflateEncoder (DeflateEncoder.java:62-104) over
// ZlibEncoder's java.util.zip.Deflater (ZlibEncoder.java:223-287), i.e. zlib's raw deflate
// with one deflate(Z_SYNC_FLUSH) per frame, byte-identical (deflate_core.h).
//
// Levels 4-9 (deflate_slow), per batch:
//   k_defl_plan   thread per session: PerMessageDeflateEncoder's frame rules (pmd_step), the
//                 window geometry of every deflate call (where zlib's fill_window slides), and
//                 the sizes of the session's regions;  k_defl_scan: their bases.
//   k_defl_prep   workgroup per session: the stream S (32 KiB of history + the frames' bytes),
//                 hash links in position order (an LDS table of the last position of each of
//                 the 32 K hashes), the window image zlib keeps — the bytes past every frame's
//                 end before and after a slide there — and zlib's head/prev arrays for the
//                 next batch; the match-chunk list.
//   k_defl_match  one wave per 256 positions of a frame: longest_match at every position for
//                 both chain budgets (match_at).
//   k_defl_parse  lane per frame: deflate_slow's lazy evaluation over those results
//                 (parse_call), Huffman trees and the bits of every block, the sync marker.
//   k_defl_final  workgroup per session: a slide inside the last frame's tail, the state.
// Levels 1-3 (deflate_fast, whose hash chains depend on its matches) run zlib's own loop
// one lane a session (k_defl_serial); level 0 is stored blocks (k_defl_parse).
#include <hip/hip_runtime.h>

#include "deflate_core.h"
#include "deflate_pmd.h"
#include "wsgpu_internal.h"

namespace ws {

namespace {

constexpr int32_t HNONE = INT32_MIN;

__device__ inline uint32_t java_bound(uint32_t len) { return len + ((len + 7) >> 3) + ((len + 63) >> 6) + 15; }
__device__ inline uint64_t r16(uint64_t x) { return (x + 15) & ~15ull; }

// the match chunks of a frame k_defl_match takes: all of them, or with the LDS walk
// (k_defl_match_lds) on and the frame short enough for its ring, those from the first one
// holding a position of the frame's last 266 (the fast range [0, len - 266) is the ring's)
__device__ inline uint32_t chunk_first(const DeflArgs& a, uint32_t len) {
  if (!a.match_lds || len > DEFL_LDS_MAXLEN || len < 267) return 0;
  return (len - 266) / DEFL_CH;
}
__device__ inline uint32_t chunk_count(uint32_t len) { return len > 2 ? (len - 2 + DEFL_CH - 1) / DEFL_CH : 0; }

__device__ inline void wave_mem_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

struct Sums {
  uint64_t *S, *O, *Y, *C, *B;
  __device__ Sums(const DeflArgs& a) {
    const uint64_t n = (uint64_t)a.n_sessions + 1;
    S = a.sums;
    O = a.sums + n;
    Y = a.sums + 2 * n;
    C = a.sums + 3 * n;
    B = a.sums + 4 * n;
  }
};

// ------------------------------------------------------------------ k_defl_plan
__global__ __launch_bounds__(64) void k_defl_plan(DeflArgs a) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  Sums sm(a);
  if (s >= a.n_sessions) {
    if (s == a.n_sessions) sm.S[s] = sm.O[s] = sm.Y[s] = sm.C[s] = sm.B[s] = 0;
    return;
  }
  const wsg_deflate_state st = a.state[s];
  uint8_t comp = st.compressing;
  bool hasd = st.has_deflater != 0;
  uint32_t sw = hasd ? st.strstart : 0;
  const bool parallel = a.level >= 4 && !a.serial;
  const uint32_t k0 = a.session_first[s], k1 = a.session_first[s + 1];
  uint64_t orel = 0, yrel = 0, chunks = 0;
  uint32_t srel = DEFL_HIST, last = ~0u, brel = 0;
  bool any_call = false, first_fresh = false;
  for (uint32_t k = k0; k < k1; k++) {
    const wsg_frame_desc d = a.desc[k];
    const int fin = d.flags >> 7, rsv = (d.flags >> 4) & 7;
    const uint32_t len = d.payload_len;
    uint8_t rsv_out, drop;
    const int kind = pmd_step(&comp, d.opcode, fin, rsv, len, a.no_context, &rsv_out, &drop);
    uint32_t fl = (uint32_t)kind | (drop ? DF_DROP : 0u) | ((uint32_t)rsv_out << DF_RSV_SHIFT) | (fin ? DF_FIN : 0u);
    DeflFrame f{0, 0, len, s, 0, 0};
    if (kind == PMD_CALL) {
      if (!hasd) {
        fl |= DF_SEG;
        if (!any_call) first_fresh = true;
        hasd = true;
        sw = 0;
      }
      any_call = true;
      if (sw >= (uint32_t)(zd::WSIZE + zd::MAX_DIST)) {   // fill_window's slide at the call's first loop top
        if (sw == (uint32_t)(zd::WSIZE + zd::MAX_DIST)) fl |= DF_START_SLID;
        sw -= zd::WSIZE;
      }
      f.start_w = sw;
      uint32_t n = len < (uint32_t)zd::WINDOW_SIZE - sw ? len : (uint32_t)zd::WINDOW_SIZE - sw;
      uint32_t loaded = sw + n, rem = len - n;
      while (rem) {   // frames longer than the free window: slide + read again
        loaded -= zd::WSIZE;
        uint32_t m = rem < (uint32_t)zd::WINDOW_SIZE - loaded ? rem : (uint32_t)zd::WINDOW_SIZE - loaded;
        loaded += m;
        rem -= m;
      }
      if (loaded > (uint32_t)(zd::WSIZE + zd::MAX_DIST)) fl |= DF_TAIL_OK;
      sw = loaded;
      a.fout[k] = orel;
      orel += r16(java_bound(len));
      if (parallel) {
        f.s_rel = srel;
        a.fsym[k] = yrel;
        yrel += (len + 3) & ~3u;   // every block's symbols, back to back (a symbol covers >= 1 byte)
        f.blk_rel = brel;
        brel += defl_blk_cap(len);
        chunks += chunk_count(len) - chunk_first(a, len) + ((fl & DF_TAIL_OK) ? 1 : 0);
        srel += len;
      }
      last = k;
    } else if (kind == PMD_EMPTY) {
      a.fout[k] = orel;
      orel += 16;
    } else {
      a.fout[k] = 0;
    }
    if (drop) hasd = false;
    a.fflags[k] = fl;
    a.ff[k] = f;
  }
  const bool persist = hasd && last != ~0u;
  if (persist) {   // the calls of the segment that outlives the batch
    for (uint32_t k = last + 1; k-- > k0;) {
      const uint32_t fl = a.fflags[k];
      if ((fl & DF_KIND) != PMD_CALL) continue;
      a.fflags[k] = fl | DF_PERSIST;
      if (fl & DF_SEG) break;
    }
  }
  sm.S[s] = parallel && any_call ? r16((uint64_t)srel + DEFL_PAD) : 0;
  sm.O[s] = orel;
  sm.Y[s] = yrel;
  sm.C[s] = chunks;
  sm.B[s] = brel;
  DeflSess fs;
  fs.sw_final = sw;
  fs.hw_final = st.high_water;
  fs.last_call = last;
  fs.has_deflater = hasd;
  fs.compressing = comp;
  fs.first_fresh = first_fresh;
  fs.persist = persist;
  a.fs[s] = fs;
}

// exclusive scan of the five per-session size arrays (one workgroup)
__global__ __launch_bounds__(1024) void k_defl_scan(DeflArgs a) {
  __shared__ uint64_t part[1024];
  const uint32_t tid = threadIdx.x;
  const uint64_t n = a.n_sessions;
  for (int arr = 0; arr < 5; arr++) {
    uint64_t* v = a.sums + (uint64_t)arr * (n + 1);
    uint64_t carry = 0;
    for (uint64_t b = 0; b < n; b += 1024) {
      const uint64_t i = b + tid;
      const uint64_t x = i < n ? v[i] : 0;
      part[tid] = x;
      __syncthreads();
      for (uint32_t o = 1; o < 1024; o <<= 1) {
        const uint64_t y = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += y;
        __syncthreads();
      }
      if (i < n) v[i] = carry + part[tid] - x;
      carry += part[1023];
      __syncthreads();
    }
    if (tid == 0) v[n] = carry;
    __syncthreads();
  }
}

// ------------------------------------------------------------------ k_defl_prep
__device__ inline uint32_t load_u32u(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);   // unaligned global load
  return v;
}

// link pass of one segment, wave 0: strings [p_begin, p_last] in position order, 64 a
// group, 16 groups a batch.  A group's lanes atomicMax their position into the hash's LDS
// entry (hpos) and take the value returned: the last position of the hash before them,
// or, for a hash that repeats inside the group, a position of the group, which the lane
// then replaces by the nearest lane below with its hash (wave-local: hpos already holds the
// group's last position of every hash, what the groups after it must see).  So a batch's
// sixteen atomics go out back to back, nothing waiting on another's return; its stream words
// are loaded first and its links stored last (a store before a load would hold the load,
// loads and stores sharing vmcnt).
#ifndef WSG_LINK_BATCH
#define WSG_LINK_BATCH 8
#endif
constexpr int LINK_BATCH = WSG_LINK_BATCH;   // (build override for A/B)

// the lanes of a group whose hash an earlier lane of the group has (r >= g): predecessor =
// the nearest such lane below (positions are g + lane)
__device__ __noinline__ int32_t link_repeats(uint32_t h, bool part, int32_t g, int32_t r) {
  const int lane = threadIdx.x & 63;
  const uint64_t lt = (1ull << lane) - 1;
  int32_t pr = r;
  uint64_t todo = __ballot(part && r >= g);
  while (todo) {
    const uint32_t h0 = __shfl(h, __builtin_ctzll(todo));
    const uint64_t set = __ballot(part && h == h0);
    if (part && r >= g && h == h0) pr = g + (63 - __builtin_clzll(set & lt));
    todo &= ~set;
  }
  return pr;
}
// All the workgroup's waves (LINK_WAVES), batch b of a round to wave b: the waves load and
// hash their batches together, issue their atomics in turn (a barrier after each wave's
// turn, so batch order is position order), then resolve repeats and store together.
#ifndef WSG_LINK_WAVES
#define WSG_LINK_WAVES 16
#endif
constexpr int LINK_WAVES = WSG_LINK_WAVES;
__device__ void link_pass(int32_t* hpos, const uint8_t* S, uint16_t* link, uint16_t* prev, int32_t p_begin,
                          int32_t p_last, int32_t nil_pos, bool persist, int32_t base_final) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int32_t r0 = p_begin; r0 <= p_last; r0 += 64 * LINK_BATCH * LINK_WAVES) {
    const int32_t g0 = r0 + 64 * LINK_BATCH * wave;
    uint32_t wv[LINK_BATCH], hh[LINK_BATCH];
    int32_t pred[LINK_BATCH];
#pragma unroll
    for (int j = 0; j < LINK_BATCH; j++) {
      const int32_t p = g0 + 64 * j + lane;
      wv[j] = p <= p_last ? load_u32u(S + p) : 0;
    }
#pragma unroll
    for (int j = 0; j < LINK_BATCH; j++) hh[j] = zd::hash3(wv[j] & 0xff, (wv[j] >> 8) & 0xff, (wv[j] >> 16) & 0xff);
    for (int t = 0; t < LINK_WAVES; t++) {
      if (t == wave) {
#pragma unroll
        for (int j = 0; j < LINK_BATCH; j++) {   // the batch's atomics, in position order
          const int32_t p = g0 + 64 * j + lane;
          const bool part = p <= p_last && p != nil_pos;   // window index 0 of a deflater is NIL
          pred[j] = part ? atomicMax(&hpos[hh[j]], p) : HNONE;
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < LINK_BATCH; j++) {
      const int32_t g = g0 + 64 * j, p = g + lane;
      const bool part = p <= p_last && p != nil_pos;
      if (__ballot(part && pred[j] >= g)) pred[j] = link_repeats(hh[j], part, g, pred[j]);
    }
#pragma unroll
    for (int j = 0; j < LINK_BATCH; j++) {
      const int32_t p = g0 + 64 * j + lane;
      if (p <= p_last) {
        const int32_t pr = pred[j];
        link[p] = (uint16_t)((pr != HNONE && p - pr < zd::WSIZE) ? p - pr : 0);
        if (persist) {
          const int32_t v = pr != HNONE ? pr - base_final : 0;
          prev[(uint32_t)(p - base_final) & zd::WMASK] = (uint16_t)(v > 0 ? v : 0);
        }
      }
    }
  }
}

// zlib's high_water zeroing after a read into the window (fill_window's tail)
__device__ void zero_hw(uint8_t* W, uint32_t& hw, uint32_t curr) {
  const int lane = threadIdx.x & 63;
  if (hw >= (uint32_t)zd::WINDOW_SIZE) return;
  uint32_t from, init;
  if (hw < curr) {
    init = (uint32_t)zd::WINDOW_SIZE - curr < (uint32_t)zd::WIN_INIT ? (uint32_t)zd::WINDOW_SIZE - curr : (uint32_t)zd::WIN_INIT;
    from = curr;
    hw = curr + init;
  } else if (hw < curr + zd::WIN_INIT) {
    init = curr + zd::WIN_INIT - hw;
    if (init > (uint32_t)zd::WINDOW_SIZE - hw) init = (uint32_t)zd::WINDOW_SIZE - hw;
    from = hw;
    hw += init;
  } else {
    return;
  }
  for (uint32_t i = lane; i < init; i += 64) W[from + i] = 0;
  wave_mem_sync();
}

__device__ inline uint4 load16(const uint8_t* p) {
  uint4 v;
  __builtin_memcpy(&v, p, 16);   // unaligned global load
  return v;
}
__device__ inline void store16(uint8_t* p, uint4 v) { __builtin_memcpy(p, &v, 16); }

// dst[0, n) = src[0, n) by T threads from thread t (disjoint ranges): 16-B pieces, eight
// loads in flight before their stores
__device__ void copy_pieces(uint8_t* dst, const uint8_t* src, uint32_t n, uint32_t t, uint32_t T) {
  const uint32_t np = n >> 4;
  for (uint32_t i0 = 0; i0 < np; i0 += T * 8) {
    const uint32_t i_0 = i0 + t, i_1 = i_0 + T, i_2 = i_1 + T, i_3 = i_2 + T;
    const uint32_t i_4 = i_3 + T, i_5 = i_4 + T, i_6 = i_5 + T, i_7 = i_6 + T;
    uint4 v0, v1, v2, v3, v4, v5, v6, v7;
    if (i_0 < np) v0 = load16(src + 16 * (uint64_t)i_0);
    if (i_1 < np) v1 = load16(src + 16 * (uint64_t)i_1);
    if (i_2 < np) v2 = load16(src + 16 * (uint64_t)i_2);
    if (i_3 < np) v3 = load16(src + 16 * (uint64_t)i_3);
    if (i_4 < np) v4 = load16(src + 16 * (uint64_t)i_4);
    if (i_5 < np) v5 = load16(src + 16 * (uint64_t)i_5);
    if (i_6 < np) v6 = load16(src + 16 * (uint64_t)i_6);
    if (i_7 < np) v7 = load16(src + 16 * (uint64_t)i_7);
    if (i_0 < np) store16(dst + 16 * (uint64_t)i_0, v0);
    if (i_1 < np) store16(dst + 16 * (uint64_t)i_1, v1);
    if (i_2 < np) store16(dst + 16 * (uint64_t)i_2, v2);
    if (i_3 < np) store16(dst + 16 * (uint64_t)i_3, v3);
    if (i_4 < np) store16(dst + 16 * (uint64_t)i_4, v4);
    if (i_5 < np) store16(dst + 16 * (uint64_t)i_5, v5);
    if (i_6 < np) store16(dst + 16 * (uint64_t)i_6, v6);
    if (i_7 < np) store16(dst + 16 * (uint64_t)i_7, v7);
  }
  for (uint32_t i = (np << 4) + t; i < n; i += T) dst[i] = src[i];
}
__device__ void wave_copy(uint8_t* dst, const uint8_t* src, uint32_t n) {
  copy_pieces(dst, src, n, threadIdx.x & 63, 64);
  wave_mem_sync();
}
__device__ void block_copy(uint8_t* dst, const uint8_t* src, uint32_t n) {
  copy_pieces(dst, src, n, threadIdx.x, blockDim.x);
}

// batched_for over 16-B values
template <class LD, class ST>
__device__ void batched_for16(uint32_t lo, uint32_t hi, LD ld, ST st) {
  const uint32_t T = blockDim.x;
  for (uint32_t i0 = lo + threadIdx.x; i0 < hi; i0 += 8 * T) {
    uint4 v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint32_t i = i0 + j * T;
      v[j] = i < hi ? ld(i) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint32_t i = i0 + j * T;
      if (i < hi) st(i, v[j]);
    }
  }
}

// for i in [lo, hi) by the workgroup: v = ld(i) for eight of a thread's indices, then
// st(i, v) for them — the loads in flight together instead of one load, its wait and its
// store an index (the session-sized loops of k_defl_prep were a global load latency each)
template <class LD, class ST>
__device__ void batched_for(uint32_t lo, uint32_t hi, LD ld, ST st) {
  const uint32_t T = blockDim.x;
  for (uint32_t i0 = lo + threadIdx.x; i0 < hi; i0 += 8 * T) {
    uint32_t v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint32_t i = i0 + j * T;
      v[j] = i < hi ? ld(i) : 0u;
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint32_t i = i0 + j * T;
      if (i < hi) st(i, v[j]);
    }
  }
}

// window walk of one segment, wave 1: zlib's window image through the segment's calls
// (slides, reads, zeroing) and each frame's strips (window bytes after its end, before and
// after a slide there)
__device__ uint32_t window_walk(const DeflArgs& a, uint8_t* W, const uint8_t* S, uint32_t c0, uint32_t c_end,
                                uint32_t sw, uint32_t hw) {
  const int lane = threadIdx.x & 63;
  for (uint32_t k = c0; k < c_end; k++) {
    if ((a.fflags[k] & DF_KIND) != PMD_CALL) continue;
    const DeflFrame f = a.ff[k];
    if (sw >= (uint32_t)(zd::WSIZE + zd::MAX_DIST)) {
      wave_copy(W, W + zd::WSIZE, sw - zd::WSIZE);
      sw -= zd::WSIZE;
    }
    const uint32_t L = f.len;
    uint32_t n = L < (uint32_t)zd::WINDOW_SIZE - sw ? L : (uint32_t)zd::WINDOW_SIZE - sw;
    wave_copy(W + sw, S + f.s_rel, n);
    uint32_t loaded = sw + n, rem = L - n;
    zero_hw(W, hw, loaded);
    while (rem) {
      wave_copy(W, W + zd::WSIZE, loaded - zd::WSIZE);
      loaded -= zd::WSIZE;
      uint32_t m = rem < (uint32_t)zd::WINDOW_SIZE - loaded ? rem : (uint32_t)zd::WINDOW_SIZE - loaded;
      wave_copy(W + loaded, S + f.s_rel + (L - rem), m);
      loaded += m;
      rem -= m;
      zero_hw(W, hw, loaded);
    }
    // the strips: every lane's loads first, then its stores (a store between them would
    // make each next load wait for it: five round trips a frame instead of one)
    uint8_t* st0 = a.strips + (uint64_t)k * 2 * zd::STRIP;
    constexpr int SJ = (zd::STRIP + 63) / 64;
    uint8_t v0[SJ], v1[SJ];
#pragma unroll
    for (int i = 0; i < SJ; i++) {
      const uint32_t j = lane + 64 * i;
      const uint32_t q = loaded - zd::WSIZE + j;
      v0[i] = (j < (uint32_t)zd::STRIP && loaded + j < (uint32_t)zd::WINDOW_SIZE) ? W[loaded + j] : 0;
      v1[i] = (j < (uint32_t)zd::STRIP && loaded >= (uint32_t)zd::WSIZE && q < (uint32_t)zd::WINDOW_SIZE) ? W[q] : 0;
    }
#pragma unroll
    for (int i = 0; i < SJ; i++) {
      const uint32_t j = lane + 64 * i;
      if (j < (uint32_t)zd::STRIP) {
        st0[j] = v0[i];
        st0[zd::STRIP + j] = v1[i];
      }
    }
    sw = loaded;
  }
  return hw;
}

// Segments of a session: runs of calls on one deflater (a DF_SEG call starts a new one)
struct SegInfo {
  uint32_t c0, c_end, c_last;
  bool fresh, persist;
  uint32_t strstart0, ins0, H;
  int32_t seg_begin, base0, seg_end, base_final;
};
__device__ inline bool next_segment(const DeflArgs& a, const DeflSess& fs, const wsg_deflate_state& st, uint32_t& k,
                                    uint32_t k1, SegInfo& g) {
  while (k < k1 && (a.fflags[k] & DF_KIND) != PMD_CALL) k++;
  if (k >= k1) return false;
  g.c0 = k;
  g.c_last = k;
  g.c_end = k + 1;
  for (uint32_t j = k + 1; j < k1; j++) {
    const uint32_t fl = a.fflags[j];
    if ((fl & DF_KIND) != PMD_CALL) continue;
    if (fl & DF_SEG) break;
    g.c_last = j;
    g.c_end = j + 1;
  }
  const uint32_t fl0 = a.fflags[g.c0];
  g.fresh = (fl0 & DF_SEG) != 0;
  g.persist = (fl0 & DF_PERSIST) != 0;
  g.strstart0 = g.fresh ? 0 : st.strstart;
  g.ins0 = g.fresh ? 0 : st.insert;
  g.H = g.fresh ? 0 : (g.strstart0 < (uint32_t)zd::WSIZE ? g.strstart0 : (uint32_t)zd::WSIZE);
  const DeflFrame f0 = a.ff[g.c0], fl_ = a.ff[g.c_last];
  g.seg_begin = g.fresh ? (int32_t)f0.s_rel : (int32_t)(DEFL_HIST - g.H);
  g.base0 = g.fresh ? (int32_t)f0.s_rel : (int32_t)DEFL_HIST - (int32_t)g.strstart0;
  g.seg_end = (int32_t)(fl_.s_rel + fl_.len);
  g.base_final = g.seg_end - (int32_t)fs.sw_final;
  k = g.c_end;
  return true;
}

// The stream and the window (no LDS table: many sessions a CU): per segment the stream S
// (history, then the frames' bytes), the history strings' links from zlib's prev[], the
// slides applied to the prev entries no string of the batch replaces, and the window walk
// (zlib's window image, the strips); the match-chunk list.  k_defl_links then hashes the
// segment's strings.
__global__ __launch_bounds__(256) void k_defl_prep(DeflArgs a) {
  const uint32_t s = blockIdx.x, tid = threadIdx.x, wv = tid >> 6;
  const DeflSess fs = a.fs[s];
  if (fs.last_call == ~0u) return;
  Sums sm(a);
  const uint64_t soff = sm.S[s];
  uint8_t* S = a.S + soff;
  uint16_t* link = a.link + soff;
  uint8_t* W = a.smem + (uint64_t)s * WSG_DEFLATE_SESSION_BYTES;
  uint16_t* head = (uint16_t*)(W + zd::WINDOW_SIZE);
  uint16_t* prev = head + zd::WSIZE;
  const wsg_deflate_state st = a.state[s];
  const uint32_t k0 = a.session_first[s], k1 = a.session_first[s + 1];
  // the match-chunk list of the session's calls
  if (tid == 0) {
    uint64_t c = sm.C[s];
    for (uint32_t k = k0; k < k1; k++) {
      const uint32_t fl = a.fflags[k];
      if ((fl & DF_KIND) != PMD_CALL) continue;
      const uint32_t len = a.ff[k].len;
      const uint32_t nch = chunk_count(len);
      for (uint32_t i = chunk_first(a, len); i < nch; i++) a.chunks[c++] = (uint64_t)k | (uint64_t)i << 32;
      if (fl & DF_TAIL_OK) a.chunks[c++] = (uint64_t)k | 1ull << 63;
    }
  }
  uint32_t k = k0;
  SegInfo g;
  while (next_segment(a, fs, st, k, k1, g)) {
    // 1. the stream: history, then the frames' bytes
    if (!g.fresh) block_copy(S + DEFL_HIST - g.H, W + g.strstart0 - g.H, g.H);
    for (uint32_t j = g.c0; j < g.c_end; j++) {
      if ((a.fflags[j] & DF_KIND) != PMD_CALL) continue;
      const DeflFrame f = a.ff[j];
      block_copy(S + f.s_rel, a.payload + a.desc[j].payload_off, f.len);
    }
    __syncthreads();
    // 2. links of the hashed history strings (zlib's prev[])
    const int32_t base0 = g.base0, base_final = g.base_final;
    if (!g.fresh)
      batched_for(
          DEFL_HIST - g.H, DEFL_HIST - g.ins0,
          [&](uint32_t p) { return (uint32_t)prev[(uint32_t)((int32_t)p - base0) & zd::WMASK]; },
          [&](uint32_t p, uint32_t pv) {
            const uint32_t w = (uint32_t)((int32_t)p - base0);
            link[p] = (uint16_t)((pv != 0 && w - pv < (uint32_t)zd::WSIZE) ? w - pv : 0);
          });
    __syncthreads();
    // 3. the slides of this batch applied to the prev entries no string of it replaces
    if (g.persist && !g.fresh && base_final != base0) {
      uint4* prev16 = (uint4*)prev;
      const int32_t shift = base0 - base_final;
      batched_for16(0, zd::WSIZE / 8, [&](uint32_t i) { return prev16[i]; }, [&](uint32_t i, uint4 v) {
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
          uint32_t o = 0;
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const uint32_t pv = (w[e] >> (16 * h)) & 0xffff;
            const int32_t nv = pv ? (int32_t)pv + shift : 0;
            o |= (uint32_t)(nv > 0 ? nv : 0) << (16 * h);
          }
          w[e] = o;
        }
        prev16[i] = make_uint4(w[0], w[1], w[2], w[3]);
      });
    }
    // 4. the window walk (wave 0)
    if (wv == 0) {
      const uint32_t hw = window_walk(a, W, S, g.c0, g.c_end, g.strstart0, g.fresh ? 0 : st.high_water);
      if (g.persist && (tid & 63) == 0) a.fs[s].hw_final = hw;
    }
    __syncthreads();
  }
}

// The segments' strings hashed in position order (an LDS table of the last position of
// each of the 32 K hashes: one session a CU), their links, zlib's prev[] entries for them,
// and head[] for the next batch.
__global__ __launch_bounds__(64 * LINK_WAVES) void k_defl_links(DeflArgs a) {
  __shared__ int32_t hpos[zd::WSIZE];   // 128 KiB: last position of each hash (S coordinates)
  const uint32_t s = blockIdx.x, tid = threadIdx.x, wv = tid >> 6;
  const DeflSess fs = a.fs[s];
  if (fs.last_call == ~0u) return;
  Sums sm(a);
  const uint64_t soff = sm.S[s];
  const uint8_t* S = a.S + soff;
  uint16_t* link = a.link + soff;
  uint8_t* W = a.smem + (uint64_t)s * WSG_DEFLATE_SESSION_BYTES;
  uint16_t* head = (uint16_t*)(W + zd::WINDOW_SIZE);
  uint16_t* prev = head + zd::WSIZE;
  const wsg_deflate_state st = a.state[s];
  const uint32_t k0 = a.session_first[s], k1 = a.session_first[s + 1];
  uint32_t k = k0;
  SegInfo g;
  while (next_segment(a, fs, st, k, k1, g)) {
    const int32_t base0 = g.base0, base_final = g.base_final;
    if (g.fresh) {
      for (uint32_t h = tid; h < (uint32_t)zd::WSIZE; h += blockDim.x) hpos[h] = HNONE;
    } else {   // (head as 16-B pieces, eight entries each, eight pieces of a thread in flight)
      const uint4* head16 = (const uint4*)head;
      batched_for16(0, zd::WSIZE / 8, [&](uint32_t i) { return head16[i]; }, [&](uint32_t i, uint4 v) {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 8; e++) {
          const uint32_t hv = (w[e >> 1] >> (16 * (e & 1))) & 0xffff;
          hpos[8 * i + e] = hv == 0 ? HNONE : (int32_t)hv + base0;
        }
      });
    }
    __syncthreads();
    {
      const int32_t p_begin = g.fresh ? g.seg_begin : (int32_t)(DEFL_HIST - g.ins0);
      // window index 0 is NIL: a deflater's first string, also when it is still pending (strstart <= 2)
      link_pass(hpos, S, link, prev, p_begin, g.seg_end - 3, base0, g.persist, base_final);
    }
    __syncthreads();
    // zlib's head[] for the next batch
    if (g.persist)   // (eight entries a 16-B store)
      for (uint32_t i = tid; i < (uint32_t)zd::WSIZE / 8; i += blockDim.x) {
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
          uint32_t o = 0;
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const int32_t v = hpos[8 * i + 2 * e + h];
            const int32_t nv = v != HNONE ? v - base_final : 0;
            o |= (uint32_t)(nv > 0 ? nv : 0) << (16 * h);
          }
          w[e] = o;
        }
        ((uint4*)head)[i] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ k_defl_match
__device__ inline uint64_t load_u64(const uint8_t* p) {
  uint64_t v;
  __builtin_memcpy(&v, p, 8);   // unaligned global load
  return v;
}

// longest_match at a position whose scan never reaches the frame's end (p + 266 <= end):
// one candidate a call, 8 bytes a compare; the same walk as zd::match_at
struct FastWalk {
  uint32_t q, dist, k, best, best_d, qres;
  uint64_t b;
  bool done;
};

__device__ inline void fast_init(FastWalk& w, const uint8_t* S, const uint16_t* link, uint32_t p) {
  const uint32_t d = link[p];
  w.k = 1;
  w.best = 2;
  w.best_d = 0;
  w.qres = 0;
  w.dist = d;
  w.q = p - d;
  w.done = d == 0 || d > (uint32_t)zd::MAX_DIST;
  w.b = load_u64(S + p);
}

// evaluates candidate w.q; returns true when the walk is over
__device__ inline bool fast_step(FastWalk& w, const uint8_t* S, const uint16_t* link, uint32_t p, const zd::Cfg& c) {
  const uint32_t qbudget = c.chain >> 2;
  const uint8_t* mq = S + w.q;
  // (branch-light, as ring_step)
  const uint64_t x = load_u64(mq) ^ w.b;
  uint32_t len = (uint32_t)__builtin_ctzll(x | (1ull << 63)) >> 3;
  if (x == 0) {
    len = 8;
    for (;;) {
      const uint64_t y = load_u64(mq + len) ^ load_u64(S + p + len);
      if (y) {
        len += (uint32_t)__builtin_ctzll(y) >> 3;
        break;
      }
      len += 8;
      if (len >= (uint32_t)zd::MAX_MATCH) break;
    }
    if (len > (uint32_t)zd::MAX_MATCH) len = zd::MAX_MATCH;
  }
  const bool upd = len > w.best;
  w.best = upd ? len : w.best;
  w.best_d = upd ? w.dist : w.best_d;
  if (upd && len >= c.nice) return true;
  if (w.k == qbudget) w.qres = w.best > 2 ? ((w.best - 2) | w.best_d << 9) : 0;
  if (w.k >= c.chain) return true;
  const uint32_t l = link[w.q];
  if (l == 0) return true;
  w.dist += l;
  if (w.dist >= (uint32_t)zd::MAX_DIST) return true;
  w.q -= l;
  w.k++;
  return false;
}

__device__ inline void fast_result(const FastWalk& w, const zd::Cfg& c, uint32_t p0d, uint32_t* full, uint32_t* quarter) {
  if (p0d == 0 || p0d > (uint32_t)zd::MAX_DIST) {
    *full = *quarter = 0;
    return;
  }
  const uint32_t f = w.best > 2 ? ((w.best - 2) | w.best_d << 9) : 0;
  *full = f | (p0d == (uint32_t)zd::MAX_DIST ? (uint32_t)zd::MR_HEAD_AT_MAX : 0u);
  *quarter = w.k <= (uint32_t)(c.chain >> 2) ? f : w.qres;
}

// ------------------------------------------------------------------ k_defl_match_lds
// The match search of a session's frames out of LDS (round 6): k_defl_match's chain walks
// are random 8-B and 2-B gathers from L2, one request a lane a candidate, and the texture
// path's gather rate bounds them (PMC: 97% L2 hits, the waves waiting 61% of their
// cycles).  Here one 1024-thread workgroup a session holds a ring of DEFL_RING stream
// positions (bytes and links, 144 KiB) and walks every chain in LDS.  A phase loads the
// window of a run of consecutive frames (from MAX_DIST before the first one's start to the
// last one's end, DEFL_RING at most), then the lanes take the run's fast positions (a scan
// that stays inside its frame: p + 266 <= end), a wave 256 at a time from an LDS counter,
// refilled lane by lane as walks end, and write each result straight to the result array
// (no global load follows: the walk's loads are LDS).  A walk keeps ring indices, not
// stream positions (the ring's first 272 bytes are mirrored past its end, so a compare
// never wraps).  Positions nearer a frame's end, the tail variants, and frames longer than
// DEFL_LDS_MAXLEN stay with k_defl_match.
constexpr uint32_t RING_MIRROR = 272;   // bytes: the longest compare (258 + an 8-B read + 3) past a ring index
struct LdsRing {
  uint32_t bytes[(DEFL_RING + RING_MIRROR) / 4];   // position x at byte x % DEFL_RING
  uint16_t link[DEFL_RING];
  uint32_t next;                           // the run's position dispenser
};
static_assert(sizeof(LdsRing) <= 160 * 1024, "the ring fits the LDS");

__device__ inline uint64_t ring8(const LdsRing& R, uint32_t r) {   // bytes at ring index r .. r + 7
  const uint32_t w = r >> 2, sh = r & 3;
  const uint32_t w0 = R.bytes[w], w1 = R.bytes[w + 1], w2 = R.bytes[w + 2];
  const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh), hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
  return (uint64_t)hi << 32 | lo;
}
__device__ inline uint32_t ring1(const LdsRing& R, uint32_t r) { return (R.bytes[r >> 2] >> (8 * (r & 3))) & 0xff; }

// a walk over the ring: FastWalk's fields with q and the position as ring indices
struct RingWalk {
  uint32_t q, pr, dist, k, best, best_d, qres;
  uint64_t b;
  bool done;
};

__device__ inline void ring_init(RingWalk& w, const LdsRing& R, uint32_t p) {
  const uint32_t pr = p % DEFL_RING;
  const uint32_t d = R.link[pr];
  w.pr = pr;
  w.k = 1;
  w.best = 2;
  w.best_d = 0;
  w.qres = 0;
  w.dist = d;
  w.done = d == 0 || d > (uint32_t)zd::MAX_DIST;
  w.q = w.done ? pr : (pr >= d ? pr - d : pr + DEFL_RING - d);   // (a done walk still steps: in the ring)
  w.b = ring8(R, pr);
}

// one candidate; true when the walk is over.  Branch-light: the common prefix of the first
// 8 bytes comes from the compare word (a chain joins strings of one hash, so two equal
// bytes mean three), and a candidate takes the lead when that prefix is longer than the
// best: zlib's scan_end pre-checks only skip candidates that cannot.  Only a prefix of all 8
// bytes goes on comparing.
__device__ inline bool ring_step(RingWalk& w, const LdsRing& R, const zd::Cfg& c, bool live) {
  const uint64_t x = ring8(R, w.q) ^ w.b;
  const uint32_t l = R.link[w.q];
  uint32_t len = (uint32_t)__builtin_ctzll(x | (1ull << 63)) >> 3;   // (7 for x == 0 and x's top byte)
  if (x == 0 && live) {   // (a lane not walking must not compare on: its string may be itself)
    len = 8;
    for (;;) {
      const uint64_t y = ring8(R, w.q + len) ^ ring8(R, w.pr + len);
      if (y) {
        len += (uint32_t)__builtin_ctzll(y) >> 3;
        break;
      }
      len += 8;
      if (len >= (uint32_t)zd::MAX_MATCH) break;
    }
    if (len > (uint32_t)zd::MAX_MATCH) len = zd::MAX_MATCH;
  }
  const bool upd = len > w.best;
  w.best = upd ? len : w.best;
  w.best_d = upd ? w.dist : w.best_d;
  if (w.k == (uint32_t)(c.chain >> 2)) w.qres = w.best > 2 ? ((w.best - 2) | w.best_d << 9) : 0;
  const uint32_t nd = w.dist + l;
  const bool end = (upd && len >= c.nice) || w.k >= c.chain || l == 0 || nd >= (uint32_t)zd::MAX_DIST;
  if (!end) {
    w.dist = nd;
    w.q = w.q >= l ? w.q - l : w.q + DEFL_RING - l;
    w.k++;
  }
  return end;
}

__device__ inline void ring_result(const RingWalk& w, const zd::Cfg& c, uint32_t p0d, uint32_t* full, uint32_t* quarter) {
  if (p0d == 0 || p0d > (uint32_t)zd::MAX_DIST) {
    *full = *quarter = 0;
    return;
  }
  const uint32_t f = w.best > 2 ? ((w.best - 2) | w.best_d << 9) : 0;
  *full = f | (p0d == (uint32_t)zd::MAX_DIST ? (uint32_t)zd::MR_HEAD_AT_MAX : 0u);
  *quarter = w.k <= (uint32_t)(c.chain >> 2) ? f : w.qres;
}

// a frame's fast range: [start, end - 266) when the frame takes the LDS walk
__device__ inline bool lds_frame(const DeflFrame& f) { return f.len <= DEFL_LDS_MAXLEN; }

__global__ __launch_bounds__(1024) void k_defl_match_lds(DeflArgs a) {
  __shared__ LdsRing R;
  const uint32_t s = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const uint64_t lt_mask = (1ull << lane) - 1;
  const DeflSess fs = a.fs[s];
  if (fs.last_call == ~0u) return;
  Sums sm(a);
  const uint64_t soff = sm.S[s];
  const uint32_t* Sw = (const uint32_t*)(a.S + soff);   // (S regions are 16-B aligned)
  const uint16_t* link = a.link + soff;
  uint32_t* res = a.res + 2 * soff;
  const zd::Cfg cfg = zd::level_cfg(a.level);
  const uint32_t k0 = a.session_first[s], k1 = a.session_first[s + 1];
  uint32_t lo_loaded = 0, hi_loaded = 0;   // stream positions the ring holds: [lo, hi)
  uint32_t k = k0;
  for (;;) {
    // the run: consecutive LDS frames whose window fits the ring
    while (k < k1 && ((a.fflags[k] & DF_KIND) != PMD_CALL || !lds_frame(a.ff[k]))) k++;
    if (k >= k1) break;
    const DeflFrame f0 = a.ff[k];
    const uint32_t need_lo = f0.s_rel > (uint32_t)zd::MAX_DIST ? f0.s_rel - zd::MAX_DIST : 0;
    uint32_t run_end = f0.s_rel + f0.len, kn = k + 1, nfr = 0;
    uint32_t lo8[8], pre8[9];
    pre8[0] = 0;
    if (f0.len >= 267) {
      lo8[0] = f0.s_rel;
      pre8[1] = f0.len - 266;
      nfr = 1;
    }
    while (kn < k1 && nfr < 8) {
      const uint32_t fl = a.fflags[kn];
      if ((fl & DF_KIND) != PMD_CALL) {
        kn++;
        continue;
      }
      const DeflFrame f = a.ff[kn];
      if (!lds_frame(f) || f.s_rel != run_end || f.s_rel + f.len - need_lo > DEFL_RING - 16) break;
      if (f.len >= 267) {
        lo8[nfr] = f.s_rel;
        pre8[nfr + 1] = pre8[nfr] + f.len - 266;
        nfr++;
      }
      run_end = f.s_rel + f.len;
      kn++;
    }
    // load the window [need_lo, run_end): what the ring does not hold yet
    const uint32_t from = (need_lo >= lo_loaded && need_lo <= hi_loaded) ? hi_loaded : need_lo;
    __syncthreads();   // (the previous run's walks read the ring)
    // (eight global loads of a thread in flight before their LDS stores)
    batched_for((from >> 2), (run_end + 3) >> 2, [&](uint32_t wd) { return Sw[wd]; },
                [&](uint32_t wd, uint32_t v) {
                  const uint32_t r = (wd << 2) % DEFL_RING >> 2;
                  R.bytes[r] = v;
                  if (r < RING_MIRROR / 4) R.bytes[DEFL_RING / 4 + r] = v;
                });
    batched_for(from, run_end, [&](uint32_t x) { return (uint32_t)link[x]; },
                [&](uint32_t x, uint32_t v) { R.link[x % DEFL_RING] = (uint16_t)v; });
    if (tid == 0) {
      R.next = 0;
    }
    lo_loaded = need_lo;
    hi_loaded = run_end;
    k = kn;
    __syncthreads();
    const uint32_t total = pre8[nfr];
    if (total == 0) continue;
    // (the run's frames from the registers every thread computed: a select a frame, no
    // dependent LDS reads when a lane takes its next position)
    auto pos_of = [&](uint32_t v) -> uint32_t {
      uint32_t lo = lo8[0], pre = 0;
#pragma unroll
      for (uint32_t j = 1; j < 8; j++) {
        const bool c = j < nfr && pre8[j] <= v;
        lo = c ? lo8[j] : lo;
        pre = c ? pre8[j] : pre;
      }
      return lo + (v - pre);
    };
    // the wave's range of virtual indices [next, cend), 256 at a time from the dispenser
    auto grab = [&](uint32_t& nx, uint32_t& ce) {
      uint32_t b = 0;
      if (lane == 0) b = atomicAdd(&R.next, 256u);
      b = __shfl(b, 0);
      nx = b < total ? b : total;
      ce = b + 256 < total ? b + 256 : total;
    };
    uint32_t next, cend;
    grab(next, cend);
    uint32_t p = next + lane;
    bool act = p < cend;
    next = next + 64 < cend ? next + 64 : cend;
    RingWalk w;
    w.q = w.pr = 0;   // (every lane steps, active or not: its indices stay in the ring)
    uint32_t d0 = 0;
    if (act) {
      p = pos_of(p);
      ring_init(w, R, p);
      d0 = w.dist;
    }
    for (;;) {
      if (!__ballot(act)) {   // every walk ended and the range is used up: another one
        if (next >= cend) {
          grab(next, cend);
          if (next >= cend) break;
        }
        const uint32_t v = next + lane;
        act = v < cend;
        next = next + 64 < cend ? next + 64 : cend;
        if (act) {
          p = pos_of(v);
          ring_init(w, R, p);
          d0 = w.dist;
        }
        continue;
      }
      // every lane takes the step (no branch round it, no state merges): an inactive lane's
      // walk is never read, and a done lane's result is 0 whatever its walk holds
      const bool stepped = ring_step(w, R, cfg, act && !w.done);
      const bool fin = act && (w.done || stepped);
      if (fin) {
        uint32_t full, quarter;
        ring_result(w, cfg, d0, &full, &quarter);
        *(uint2*)(res + 2 * (uint64_t)p) = make_uint2(full, quarter);
      }
      const uint64_t m = __ballot(fin);
      if (m) {   // lanes whose walk ended take the next positions: the range's, then a new range's
        const uint32_t need = (uint32_t)__builtin_popcountll(m), avail = cend - next;
        uint32_t n2 = cend, c2 = cend;
        if (need > avail) grab(n2, c2);
        if (fin) {
          const uint32_t r = (uint32_t)__builtin_popcountll(m & lt_mask);
          const uint32_t v = r < avail ? next + r : n2 + (r - avail);
          act = r < avail || v < c2;
          if (act) {
            p = pos_of(v);
            ring_init(w, R, p);
            d0 = w.dist;
          }
        }
        if (need > avail) {
          const uint32_t n = n2 + (need - avail);
          next = n < c2 ? n : c2;
          cend = c2;
        } else {
          next += need;
        }
      }
    }
  }
}

// longest_match at a position of a frame's last bytes, whose compares may pass the frame's
// end into its strip (zd::match_at's walk, 8 bytes a compare where they lie before the end)
__device__ inline uint64_t tail8(const uint8_t* S, const uint8_t* strip, uint32_t end, uint32_t x) {
  if (x + 8 <= end) return load_u64(S + x);
  uint64_t v = 0;
  for (uint32_t i = 0; i < 8; i++) {
    const uint32_t y = x + i;
    const uint64_t b = y < end ? S[y] : (y - end < (uint32_t)zd::STRIP ? strip[y - end] : 0u);
    v |= b << (8 * i);
  }
  return v;
}
__device__ void tail_match_at(const uint8_t* S, const uint8_t* strip, const uint16_t* link, uint32_t s, uint32_t end,
                              const zd::Cfg& c, uint32_t* out_full, uint32_t* out_quarter) {
  const uint32_t d = link[s];
  if (d == 0 || d > (uint32_t)zd::MAX_DIST) {
    *out_full = *out_quarter = 0;
    return;
  }
  const uint32_t flags = d == (uint32_t)zd::MAX_DIST ? (uint32_t)zd::MR_HEAD_AT_MAX : 0u;
  const uint32_t nice = c.nice < end - s ? c.nice : end - s;
  const uint32_t qbudget = c.chain >> 2;
  const uint64_t b = tail8(S, strip, end, s);
  uint32_t best = 2, best_d = 0, qres = 0, q = s - d, dist = d, k = 1;
  for (;; k++) {
    // (branch-light, as ring_step)
    const uint64_t x = tail8(S, strip, end, q) ^ b;
    uint32_t len = (uint32_t)__builtin_ctzll(x | (1ull << 63)) >> 3;
    if (x == 0) {
      len = 8;
      for (;;) {
        const uint64_t y = tail8(S, strip, end, q + len) ^ tail8(S, strip, end, s + len);
        if (y) {
          len += (uint32_t)__builtin_ctzll(y) >> 3;
          break;
        }
        len += 8;
        if (len >= (uint32_t)zd::MAX_MATCH) break;
      }
      if (len > (uint32_t)zd::MAX_MATCH) len = zd::MAX_MATCH;
    }
    const bool upd = len > best;
    best = upd ? len : best;
    best_d = upd ? dist : best_d;
    if (upd && len >= nice) break;
    if (k == qbudget) qres = best > 2 ? ((best - 2) | best_d << 9) : 0;
    if (k >= c.chain) break;
    const uint32_t l = link[q];
    if (l == 0) break;
    dist += l;
    if (dist >= (uint32_t)zd::MAX_DIST) break;
    q -= l;
  }
  const uint32_t full = best > 2 ? ((best - 2) | best_d << 9) : 0;
  *out_full = full | flags;
  *out_quarter = k <= qbudget ? full : qres;
}

__global__ __launch_bounds__(64) void k_defl_match(DeflArgs a) {
  // a chunk's results are kept in LDS and written at its end: a global store would make
  // every later load of the wave wait for it (loads and stores share vmcnt)
  __shared__ uint2 rs[DEFL_CH > DEFL_TAILN ? DEFL_CH : DEFL_TAILN];
  Sums sm(a);
  const uint64_t total = sm.C[a.n_sessions];
  const zd::Cfg cfg = zd::level_cfg(a.level);
  const uint32_t lane = threadIdx.x;
  const uint64_t lt_mask = (1ull << lane) - 1;
  // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs; XCD x takes the x-th
  // eighth of the chunk list (a run of whole sessions), so the waves sharing an L2 walk the
  // same sessions' streams and links
  const uint32_t xcd = blockIdx.x & 7, g8 = gridDim.x >> 3;
  const uint64_t per_xcd = (total + 7) >> 3;
  for (uint64_t L = blockIdx.x >> 3; L < per_xcd; L += g8) {
    const uint64_t c = xcd * per_xcd + L;
    if (c >= total) break;
    const uint64_t e = a.chunks[c];
    const uint32_t k = (uint32_t)e, ci = (uint32_t)(e >> 32) & 0x7fffffffu;
    const bool var = (e >> 63) != 0;
    const DeflFrame f = a.ff[k];
    const uint64_t soff = sm.S[f.sess];
    const uint8_t* S = a.S + soff;
    const uint16_t* link = a.link + soff;
    uint32_t* res = a.res + 2 * soff;
    const uint32_t start = f.s_rel, end = start + f.len;
    const uint32_t tstart = end - start > DEFL_TAILN ? end - DEFL_TAILN : start;
    const uint32_t p0 = var ? tstart : start + ci * DEFL_CH;
    const uint32_t p1 = var ? end - 2 : (p0 + DEFL_CH < end - 2 ? p0 + DEFL_CH : end - 2);
    // positions whose scan stays inside the frame: the fast walk, lanes refilled as they finish
    const uint32_t pf = var ? p0 : (end >= 266 && end - 266 > p0 ? (end - 266 < p1 ? end - 266 : p1) : p0);
    const bool in_lds = a.match_lds && !var && lds_frame(f);   // (its fast range: k_defl_match_lds)
    if (pf > p0 && !in_lds) {
      uint32_t next = p0 + 64;
      uint32_t p = p0 + lane;
      bool act = p < pf;
      FastWalk w;
      uint32_t d0 = 0;
      if (act) {
        fast_init(w, S, link, p);
        d0 = w.dist;
      }
      while (__ballot(act)) {
        bool fin = false;
        if (act) fin = w.done || fast_step(w, S, link, p, cfg);
        if (fin) {
          uint32_t full, quarter;
          fast_result(w, cfg, d0, &full, &quarter);
          rs[p - p0] = make_uint2(full, quarter);
        }
        const uint64_t m = __ballot(fin);
        if (m) {
          if (fin) {
            p = next + (uint32_t)__builtin_popcountll(m & lt_mask);
            act = p < pf;
            if (act) {
              fast_init(w, S, link, p);
              d0 = w.dist;
            }
          }
          next += (uint32_t)__builtin_popcountll(m);
        }
      }
    }
    // the frame's last bytes (and the tail variant): the scan may pass the end
    const uint8_t* strip = a.strips + ((uint64_t)k * 2 + (var ? 1 : 0)) * zd::STRIP;
    for (uint32_t p = (pf > p0 ? pf : p0) + lane; p < p1; p += 64) {
      uint32_t full, quarter;
      tail_match_at(S, strip, link, p, end, cfg, &full, &quarter);
      rs[p - p0] = make_uint2(full, quarter);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    uint2* dst = var ? (uint2*)(a.tres + ((uint64_t)k * DEFL_TAILN + (p0 - tstart)) * 2) : (uint2*)(res + 2 * (uint64_t)p0);
    for (uint32_t i = (in_lds ? pf - p0 : 0) + lane; i < p1 - p0; i += 64) dst[i] = rs[i];
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------ k_defl_parse
// The parse lane's reads come through register windows (8 positions of results, 16 stream
// bytes) and its symbols through a 32-word LDS ring flushed in bursts: a global store in
// the loop would hold every later load of the wave until it completed (shared vmcnt).
struct ResWin {
  const uint4* res;      // session base: 2 positions a uint4
  const uint32_t* tres;  // the frame's tail results
  uint32_t tstart;
  uint32_t wbase;
  uint4 w0, w1, w2, w3;  // positions wbase .. wbase + 7
  const uint8_t* S;      // session stream
  uint64_t blo, bhi;     // its bytes wbase - 8 .. wbase + 7, loaded with the results: the
                         // literal a step may take is the byte before its position
  __device__ void operator()(uint32_t p, int variant, uint32_t* f, uint32_t* q) {
    if (variant && p >= tstart) {
      const uint32_t* t = tres + 2 * (p - tstart);
      *f = t[0];
      *q = t[1];
      return;
    }
    const uint32_t b = p & ~7u;
    if (b != wbase) {
      wbase = b;
      const uint4* r = res + (b >> 1);
      w0 = r[0];
      w1 = r[1];
      w2 = r[2];
      w3 = r[3];
      blo = b >= 8 ? *(const uint64_t*)(S + b - 8) : 0ull;
      bhi = *(const uint64_t*)(S + b);
    }
    const uint32_t i = p & 7;   // component selects only: an aggregate select would live in scratch
    const bool o = i & 1, b1 = i & 2, b2 = i & 4;
    const uint32_t ax = o ? w0.z : w0.x, ay = o ? w0.w : w0.y;
    const uint32_t bx = o ? w1.z : w1.x, by_ = o ? w1.w : w1.y;
    const uint32_t cx = o ? w2.z : w2.x, cy = o ? w2.w : w2.y;
    const uint32_t dx = o ? w3.z : w3.x, dy = o ? w3.w : w3.y;
    const uint32_t lx = b1 ? bx : ax, ly = b1 ? by_ : ay, hx = b1 ? dx : cx, hy = b1 ? dy : cy;
    *f = b2 ? hx : lx;
    *q = b2 ? hy : ly;
  }
};
// the parse's byte(p): from the results window's bytes (a byte outside them, at a frame's
// last positions where no lookup ran, from the stream)
struct ByteWin {
  const ResWin* r;
  __device__ uint32_t operator()(uint32_t p) const {
    const uint32_t o = p + 8 - r->wbase;
    if (o >= 16 || r->wbase == ~0u) return r->S[p];
    return (uint32_t)(((o < 8 ? r->blo : r->bhi) >> (8 * (o & 7))) & 0xff);
  }
};
#ifndef WSG_SYM_RING
#define WSG_SYM_RING 64
#endif
constexpr uint32_t SYM_RING = WSG_SYM_RING;
struct SymStage {
  uint32_t* ring;   // LDS: word j of this lane at ring[j * 64]
  uint32_t* dst;    // the frame's symbol region
  uint32_t n;       // symbols of the frame so far
  uint32_t staged;
  __device__ void flush() {
    uint32_t* d = dst + (n - staged);
    for (uint32_t j = 0; j < staged; j++) d[j] = ring[j * 64];
    staged = 0;
  }
  __device__ void put(uint32_t v) {
    ring[staged * 64] = v;
    staged++;
    n++;
    if (staged == SYM_RING) flush();
  }
  __device__ void block_done() { flush(); }
};
// the parse's block sink: one DeflBlock slot a block zlib flushes
struct BlockSink {
  DeflBlock* blk;
  uint64_t sym_at;   // index of the frame's first symbol in the symbol buffers
  uint32_t nb, done;
  __device__ void operator()(uint32_t nsym, uint32_t stored_s, uint32_t stored_len, bool stored_ok) {
    DeflBlock* b = blk + nb++;
    b->sym0 = sym_at + done;
    b->nsym = nsym;
    b->stored_s = stored_s;
    b->stored_len = stored_len;
    b->stored_ok = stored_ok ? 1 : 0;
    done += nsym;
  }
};
struct SBytes {
  const uint8_t* S;
  __device__ uint32_t operator()(uint32_t p) const { return S[p]; }
  __device__ const uint8_t* ptr(uint32_t p) const { return S + p; }
};

__device__ void pass_or_empty(const DeflArgs& a, uint32_t k, uint32_t fl, uint64_t obase) {
  const wsg_frame_desc d = a.desc[k];
  wsg_frame_desc o;
  o.opcode = d.opcode;
  o.flags = (uint8_t)(((fl & DF_FIN) ? 0x80 : 0) | (((fl >> DF_RSV_SHIFT) & 7) << 4));
  o.status = 0;
  if ((fl & DF_KIND) == PMD_PASS) {
    o.payload_off = d.payload_off;
    o.payload_len = d.payload_len;
  } else {
    o.payload_off = obase + a.fout[k];
    o.payload_len = 1;
    o.flags |= WSG_DESC_DEFLATED;
    a.out[o.payload_off] = 0;
  }
  a.out_desc[k] = o;
}

// lane per frame: deflate_slow's control flow over the match results; the symbols of
// every block and its stored range go to the frame's block slots (k_defl_hist/trees/emit)
__global__ __launch_bounds__(64) void k_defl_parse(DeflArgs a) {
  __shared__ uint32_t ring[SYM_RING * 64];
  Sums sm(a);
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= a.n_lanes) return;
  const zd::Cfg cfg = zd::level_cfg(a.level);
  for (uint64_t k = tid; k < a.n_frames; k += a.n_lanes) {
    const uint32_t fl = a.fflags[k];
    const DeflFrame f = a.ff[k];
    if ((fl & DF_KIND) != PMD_CALL) {
      pass_or_empty(a, (uint32_t)k, fl, sm.O[f.sess]);
      continue;
    }
    if (a.level == 0) continue;   // stored framing: k_defl_emit
    const uint64_t soff = sm.S[f.sess];
    const uint32_t end = f.s_rel + f.len;
    ResWin ra{(const uint4*)(a.res + 2 * soff), a.tres + (uint64_t)k * DEFL_TAILN * 2,
              end - f.s_rel > DEFL_TAILN ? end - DEFL_TAILN : f.s_rel, ~0u, {}, {}, {}, {}, a.S + soff, 0ull, 0ull};
    ByteWin by{&ra};
    zd::CallGeom g{f.start_w, (uint8_t)((fl & DF_START_SLID) ? 1 : 0)};
    DeflBlock* blk = a.blocks + sm.B[f.sess] + f.blk_rel;
    const uint64_t sym_at = sm.Y[f.sess] + a.fsym[k];
    SymStage sw{ring + threadIdx.x, a.sym + sym_at, 0, 0};
    BlockSink sink{blk, sym_at, 0, 0};
    const bool tail = zd::parse_call(ra, by, f.s_rel, f.len, g, cfg, sw, sink);
    for (uint32_t b = sink.nb; b < defl_blk_cap(f.len); b++) blk[b].nsym = 0;
    a.ftail[k] = tail ? 1 : 0;
    a.ff[k].nblk = sink.nb;
  }
}

// workgroup per block slot: the block's symbol frequencies (LDS atomics)
__global__ __launch_bounds__(256) void k_defl_hist(DeflArgs a) {
  __shared__ uint32_t cnt[zd::L_CODES + zd::D_CODES];
  Sums sm(a);
  const uint64_t total = sm.B[a.n_sessions];
  for (uint64_t i = blockIdx.x; i < total; i += gridDim.x) {
    DeflBlock* b = a.blocks + i;
    const uint32_t nsym = b->nsym;
    if (nsym == 0) continue;
    for (uint32_t j = threadIdx.x; j < (uint32_t)(zd::L_CODES + zd::D_CODES); j += 256) cnt[j] = 0;
    __syncthreads();
    const uint32_t* sy = a.sym + b->sym0;
    for (uint32_t j = threadIdx.x; j < nsym; j += 256) {
      const uint32_t v = sy[j], dist = v >> 8, lc = v & 255;
      if (dist == 0) {
        atomicAdd(&cnt[lc], 1u);
      } else {
        atomicAdd(&cnt[zd::len_code((int)lc) + 257], 1u);
        atomicAdd(&cnt[zd::L_CODES + zd::dist_code((int)dist - 1)], 1u);
      }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < (uint32_t)(zd::L_CODES + zd::D_CODES); j += 256) b->freq[j] = (uint16_t)cnt[j];
    __syncthreads();
  }
}

// lane per block, the block's TreeWork in LDS (TREE_LANES a workgroup, as many as the LDS
// holds: 48 of 3.2 KiB since the heap keys share their storage with the node order): the three Huffman
// trees exactly as zlib's heap builds them, the block type and its size
// The lanes are spread over TREE_WAVES waves (TREE_LANES / TREE_WAVES a wave).  Not much
// rides on it: 1, 2, 3, 4 waves ran 2.90, 2.88, 3.12, 3.06 ms (same box, 3 rounds,
// profiles/r06/r06zb_ab_tree_waves.txt) — the 48 lanes' LDS heap traffic, not one SIMD's
// issue, bounds the kernel.
#ifndef WSG_TREE_WAVES
#define WSG_TREE_WAVES 2
#endif
constexpr uint32_t TREE_LANES = 48;
constexpr uint32_t TREE_WAVES = WSG_TREE_WAVES, TREE_PER_WAVE = TREE_LANES / TREE_WAVES;
static_assert(TREE_LANES % TREE_WAVES == 0 && TREE_PER_WAVE <= 64, "whole tree lanes a wave");
static_assert(TREE_LANES * sizeof(zd::TreeWork) <= 160 * 1024, "the tree lanes' work fits the LDS");
__global__ __launch_bounds__(64 * TREE_WAVES) void k_defl_trees(DeflArgs a) {
  __shared__ zd::TreeWork tws[TREE_LANES];
  Sums sm(a);
  const uint64_t total = sm.B[a.n_sessions];
  const uint32_t lane = threadIdx.x & 63, slot = (threadIdx.x >> 6) * TREE_PER_WAVE + lane;
  if (lane >= TREE_PER_WAVE) return;
  zd::TreeWork* t = &tws[slot];
  for (uint64_t i = (uint64_t)blockIdx.x * TREE_LANES + slot; i < total; i += (uint64_t)gridDim.x * TREE_LANES) {
    DeflBlock* b = a.blocks + i;
    const uint32_t nsym = b->nsym;
    if (nsym == 0) continue;
    zd::init_block(t);
    for (int n = 0; n < zd::L_CODES; n++) t->lfc[n] = (uint16_t)(b->freq[n] + (n == zd::END_BLOCK ? 1 : 0));
    for (int n = 0; n < zd::D_CODES; n++) t->dfc[n] = b->freq[zd::L_CODES + n];
    uint32_t bits;
    int max_blindex;
    const int type = zd::plan_block(t, b->stored_ok != 0, b->stored_len, &bits, &max_blindex);
    b->type = (uint8_t)type;
    b->bits = bits;
    if (type == 2) {
      b->lcodes = (uint16_t)(t->l_max + 1);
      b->dcodes = (uint8_t)(t->d_max + 1);
      b->blcodes = (uint8_t)(max_blindex + 1);
      for (int n = 0; n <= t->l_max; n++) b->ltab[n] = t->lfc[n] | (uint32_t)t->ldl[n] << 16;
      for (int n = 0; n <= t->d_max; n++) b->dtab[n] = t->dfc[n] | (uint32_t)t->ddl[n] << 16;
      for (int n = 0; n < zd::BL_CODES; n++) b->btab[n] = t->bfc[n] | (uint32_t)t->bdl[n] << 16;
    }
  }
}

// bit output of one thread into the zeroed output words: the first and last words of the
// thread's run may be shared with a neighbour's (atomicOr), the rest are its own
struct WordSink {
  uint32_t* w;        // the frame's output as words
  uint64_t acc;
  uint32_t n;         // bits in acc
  uint32_t idx;       // word the low bits of acc go to
  bool first;
  __device__ WordSink(uint32_t* words, uint32_t bitpos) : w(words), acc(0), n(bitpos & 31), idx(bitpos >> 5),
                                                         first(true) {}
  __device__ void put(uint32_t v, uint32_t len) {
    acc |= (uint64_t)v << n;
    n += len;
    if (n >= 32) {
      if (first) {
        atomicOr(&w[idx], (uint32_t)acc);
        first = false;
      } else {
        w[idx] = (uint32_t)acc;
      }
      idx++;
      acc >>= 32;
      n -= 32;
    }
  }
  __device__ void done() {
    if (n > 0) atomicOr(&w[idx], (uint32_t)acc);
  }
};

__device__ inline void sym_code(uint32_t sy, const uint32_t* ltab, const uint32_t* dtab, bool is_static, uint32_t* c1,
                                uint32_t* l1, uint32_t* c2, uint32_t* l2) {
  // one symbol as at most two (code, length) pairs: (literal) or (length code + extra bits,
  // distance code + extra bits); at most 15 + 5 and 15 + 13 bits
  const uint32_t dist = sy >> 8;
  const int lc = (int)(sy & 255);
  if (dist == 0) {
    if (is_static) {
      *c1 = zd::static_lcode(lc);
      *l1 = (uint32_t)zd::static_llen(lc);
    } else {
      *c1 = ltab[lc] & 0xffff;
      *l1 = ltab[lc] >> 16;
    }
    *l2 = 0;
    *c2 = 0;
    return;
  }
  const int code = zd::len_code(lc);
  uint32_t c, l;
  if (is_static) {
    c = zd::static_lcode(code + 257);
    l = (uint32_t)zd::static_llen(code + 257);
  } else {
    c = ltab[code + 257] & 0xffff;
    l = ltab[code + 257] >> 16;
  }
  const int ex = zd::len_extra(code);
  *c1 = c | (ex ? (uint32_t)(lc - zd::len_base(code)) << l : 0u);
  *l1 = l + (uint32_t)ex;
  const int d = (int)dist - 1;
  const int dc = zd::dist_code(d);
  if (is_static) {
    c = zd::static_dcode(dc);
    l = 5;
  } else {
    c = dtab[dc] & 0xffff;
    l = dtab[dc] >> 16;
  }
  const int dx = zd::dist_extra(dc);
  *c2 = c | (dx ? (uint32_t)(d - zd::dist_base(dc)) << l : 0u);
  *l2 = l + (uint32_t)dx;
}

// inclusive sum over the wave's lanes
__device__ inline uint32_t wave_incl_sum(uint32_t x) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  return x;
}

// bits v (len <= 32) at bit offset off of the LDS words hb (zeroed)
__device__ inline void lds_or_bits(uint32_t* hb, uint32_t off, uint32_t v, uint32_t len) {
  if (!len) return;
  const uint32_t sh = off & 31;
  atomicOr(&hb[off >> 5], v << sh);
  if (sh + len > 32) atomicOr(&hb[(off >> 5) + 1], v >> (32 - sh));
}

// zlib's send_tree (the run-length coding of a tree's code lengths with the bit-length
// codes) by one wave, 64 code lengths a round, into the LDS words hb from bit pos on;
// returns the bit position after it.  zlib's loop cuts each run of equal lengths into
// chunks (at most 7, then 6, entries of a non-zero length; 138 of zeros) whose coding
// depends only on the chunk (its length, count, and whether it continues the run), so
// each chunk's first lane codes it: (count < min) the length count times; (non-zero) the
// length unless continued, REP_3_6 + 2 bits; (zeros) REPZ_3_10 + 3 bits or REPZ_11_138 + 7
// bits.  run_end: LDS scratch of max_code + 1 entries.
__device__ uint32_t send_tree_wave(uint32_t* hb, uint32_t pos, const uint32_t* tab, int max_code, const uint32_t* btab,
                                   uint16_t* run_end) {
  const int lane = (int)(threadIdx.x & 63);
  auto len_of = [&](int n) -> uint32_t { return n < 0 ? 0x1ffffu : (n <= max_code ? tab[n] >> 16 : 0xffffu); };
  // the last index of each index's run (a backward sweep, the carry from the window above)
  uint32_t carry = (uint32_t)max_code;
  for (int base = max_code & ~63; base >= 0; base -= 64) {
    const int n = base + lane;
    const bool valid = n <= max_code;
    const uint64_t m = __ballot(valid && len_of(n) != len_of(n + 1));
    const uint64_t hi = m & (~0ull << lane);
    if (valid) run_end[n] = (uint16_t)(hi ? (uint32_t)base + (uint32_t)__builtin_ctzll(hi) : carry);
    carry = m ? (uint32_t)base + (uint32_t)__builtin_ctzll(m) : carry;
  }
  wave_mem_sync();
  uint32_t r0c = 0;   // the first index of the run the window above ended in
  for (int base = 0; base <= max_code; base += 64) {
    const int n = base + lane;
    const bool valid = n <= max_code;
    const uint32_t v = valid ? len_of(n) : 0u;
    const uint64_t sm = __ballot(valid && v != len_of(n - 1));
    const uint64_t lo = sm & ((2ull << lane) - 1);   // (lane 63: all bits)
    const uint32_t r0 = lo ? (uint32_t)base + 63u - (uint32_t)__builtin_clzll(lo) : r0c;
    r0c = sm ? (uint32_t)base + 63u - (uint32_t)__builtin_clzll(sm) : r0c;
    const uint32_t o = (uint32_t)n - r0;
    const bool cs = valid && (v == 0 ? o % 138 == 0 : (o == 0 || (o >= 7 && (o - 7) % 6 == 0)));
    uint32_t code = 0, len = 0;
    if (cs) {
      const bool cont = o != 0;   // a chunk after the run's first: the previous length is its own
      const uint32_t rem = (uint32_t)run_end[n] - (uint32_t)n + 1;
      const uint32_t mx = v == 0 ? 138u : (cont ? 6u : 7u), mn = (v == 0 || cont) ? 3u : 4u;
      const uint32_t c = rem < mx ? rem : mx;
      auto put = [&](uint32_t cv, uint32_t cl) {
        code |= cv << len;
        len += cl;
      };
      auto bl = [&](uint32_t sym) { put(btab[sym] & 0xffff, btab[sym] >> 16); };
      if (c < mn) {
        for (uint32_t i = 0; i < c; i++) bl(v);
      } else if (v != 0) {
        uint32_t cc = c;
        if (!cont) {
          bl(v);
          cc--;
        }
        bl(zd::REP_3_6);
        put(cc - 3, 2);
      } else if (c <= 10) {
        bl(zd::REPZ_3_10);
        put(c - 3, 3);
      } else {
        bl(zd::REPZ_11_138);
        put(c - 11, 7);
      }
    }
    const uint32_t incl = wave_incl_sum(len);
    lds_or_bits(hb, pos + incl - len, code, len);
    pos += __shfl(incl, 63);
  }
  return pos;
}

// workgroup per frame: the bits of its blocks (stored copies, static or dynamic codes: the
// trees by thread 0, the symbols by every thread at offsets from a block-wide scan) and the
// sync marker, into the frame's zeroed output slot
#ifndef WSG_EMIT_T
#define WSG_EMIT_T 256
#endif
constexpr int EMIT_T = WSG_EMIT_T;
constexpr uint32_t EMIT_SYM = 4096;
constexpr uint32_t EMIT_OUT_W = 2048;   // 8 KiB
constexpr uint32_t EMIT_HDR_W = 80;   // 31 + 17 + 57 + 7 x (286 + 30) bits at most
__global__ __launch_bounds__(EMIT_T) void k_defl_emit(DeflArgs a) {
  __shared__ uint32_t s_ltab[286], s_dtab[30], s_btab[19];
  __shared__ uint32_t s_sym[EMIT_SYM];   // a block's symbols, loaded once, coalesced (blocks up to EMIT_SYM)
  __shared__ uint32_t s_wsum[EMIT_T / 64];
  __shared__ uint32_t s_hdr[EMIT_HDR_W];   // a dynamic block's header bits
  __shared__ uint16_t s_run[zd::L_CODES];  // send_tree_wave's run ends
  __shared__ uint32_t s_out[EMIT_OUT_W];   // the frame's output (frames up to EMIT_OUT_W words)
  __shared__ uint32_t s_off;   // running bit offset of the frame
  Sums sm(a);
  const uint32_t tid = threadIdx.x;
  for (uint64_t k = blockIdx.x; k < a.n_frames; k += gridDim.x) {
    const uint32_t fl = a.fflags[k];
    if ((fl & DF_KIND) != PMD_CALL) continue;
    const DeflFrame f = a.ff[k];
    const uint64_t obase = sm.O[f.sess] + a.fout[k];
    uint8_t* const ob_g = a.out + obase;
    const DeflBlock* blk = a.blocks + sm.B[f.sess] + f.blk_rel;
    const uint32_t nb = a.level == 0 ? 0 : f.nblk;
    // the frame's size: blocks in order, then the sync marker (3 bits, pad, 00 00 FF FF)
    uint64_t bitsz = 0;
    if (a.level == 0) {
      const uint32_t nst = (f.len + 65534) / 65535;
      bitsz = 8ull * (f.len + 5ull * nst);
    } else {
      for (uint32_t b = 0; b < nb; b++)
        bitsz = blk[b].type == 0 ? ((bitsz + 3 + 7) & ~7ull) + 32 + 8ull * blk[b].stored_len : bitsz + 3 + blk[b].bits;
    }
    const uint64_t bytes = (((bitsz + 3 + 7) & ~7ull) + 32) >> 3;
    // a frame's output up to EMIT_OUT_W words is put together in LDS and stored once, in
    // order (the global form's zeroing, atomics and barrier waits on stores cost more than
    // the bits); larger frames write their slot directly
    const bool lds_out = ((bytes + 3) >> 2) <= EMIT_OUT_W;
    uint8_t* const ob = lds_out ? (uint8_t*)s_out : ob_g;
    uint32_t* const ow = (uint32_t*)ob;
    for (uint64_t i = tid; i < (bytes + 3) >> 2; i += EMIT_T) ow[i] = 0;
    if (tid == 0) s_off = 0;
    __syncthreads();
    if (a.level == 0) {   // deflate_stored with Java's output buffer: 65535-byte stored blocks
      const uint8_t* src = a.payload + a.desc[k].payload_off;
      for (uint32_t o = 0, i = 0; o < f.len; o += 65535, i++) {
        const uint32_t n = f.len - o < 65535u ? f.len - o : 65535u;
        uint8_t* h = ob + (uint64_t)o + 5ull * i;
        if (tid == 0) {
          h[0] = 0;
          h[1] = (uint8_t)n;
          h[2] = (uint8_t)(n >> 8);
          h[3] = (uint8_t)~n;
          h[4] = (uint8_t)(~n >> 8);
        }
        for (uint32_t j = tid; j < n; j += EMIT_T) h[5 + j] = src[o + j];
      }
      __syncthreads();
      if (tid == 0) s_off = (uint32_t)(8ull * (f.len + 5ull * ((f.len + 65534) / 65535)));
    }
    const uint8_t* S = a.S + sm.S[f.sess];
    for (uint32_t b = 0; b < nb; b++) {
      const DeflBlock* B = blk + b;
      const uint32_t o = s_off;
      const int type = B->type;
      if (type == 0) {   // stored: 000, pad, LEN, NLEN, the bytes (as whole words, OR'ed in)
        const uint32_t pos = ((o + 3 + 7) & ~7u) >> 3;
        const uint32_t L = B->stored_len;
        const uint8_t* src = S + B->stored_s;
        const uint32_t w0 = pos >> 2, w1 = (pos + 4 + L + 3) >> 2;
        for (uint32_t w = w0 + tid; w < w1; w += EMIT_T) {
          uint32_t v = 0;
          for (uint32_t j = 0; j < 4; j++) {
            const uint32_t bp = w * 4 + j;   // byte of the frame
            uint32_t x = 0;
            if (bp >= pos && bp < pos + 4 + L) {
              const uint32_t r = bp - pos;
              x = r == 0 ? (L & 0xff) : r == 1 ? (L >> 8) & 0xff : r == 2 ? (~L) & 0xff : r == 3 ? (~L >> 8) & 0xff
                                                                                                 : src[r - 4];
            }
            v |= x << (8 * j);
          }
          if (w == w0 || w == w1 - 1) atomicOr(&ow[w], v);
          else ow[w] = v;
        }
        __syncthreads();
        if (tid == 0) s_off = (pos + 4 + L) * 8;
        __syncthreads();
        continue;
      }
      const bool is_static = type == 1;
      if (!is_static) {   // (thread 0's send_all_trees reads the three tables in turn: LDS, not global loads)
        for (uint32_t i = tid; i < B->lcodes; i += EMIT_T) s_ltab[i] = B->ltab[i];
        for (uint32_t i = tid; i < B->dcodes; i += EMIT_T) s_dtab[i] = B->dtab[i];
        if (tid < 19) s_btab[tid] = B->btab[tid];
      }
      __syncthreads();
      // the symbols: a contiguous run a thread; bit offsets from a block-wide scan
      const uint32_t nsym = B->nsym;
      const uint32_t per = (nsym + EMIT_T - 1) / EMIT_T;
      const uint32_t i0 = tid * per < nsym ? tid * per : nsym;
      const uint32_t i1 = i0 + per < nsym ? i0 + per : nsym;
      const uint32_t* sy = a.sym + B->sym0;
      const bool staged = nsym <= EMIT_SYM;   // both passes read the symbols from LDS (one coalesced load)
      if (staged) {
        batched_for(0, nsym, [&](uint32_t i) { return sy[i]; }, [&](uint32_t i, uint32_t v) { s_sym[i] = v; });
        __syncthreads();
      }
      auto sym_at = [&](uint32_t i) { return staged ? s_sym[i] : sy[i]; };
      uint32_t mybits = 0;
      for (uint32_t i = i0; i < i1; i++) {
        uint32_t c1, l1, c2, l2;
        sym_code(sym_at(i), s_ltab, s_dtab, is_static, &c1, &l1, &c2, &l2);
        mybits += l1 + l2;
      }
      // bit offsets: wave sums, then the waves' totals (one barrier)
      const uint32_t incl = wave_incl_sum(mybits);
      if ((tid & 63) == 63) s_wsum[tid >> 6] = incl;
      __syncthreads();
      uint32_t before = 0, sym_bits = 0;
#pragma unroll
      for (uint32_t w = 0; w < EMIT_T / 64; w++) {
        const uint32_t x = s_wsum[w];
        before += w < (tid >> 6) ? x : 0u;
        sym_bits += x;
      }
      const uint32_t eob_c = is_static ? zd::static_lcode(zd::END_BLOCK) : s_ltab[zd::END_BLOCK] & 0xffff;
      const uint32_t eob_l = is_static ? 7u : s_ltab[zd::END_BLOCK] >> 16;
      const uint32_t blk_end = o + 3 + B->bits;
      const uint32_t sym_start = blk_end - eob_l - sym_bits;
      {
        WordSink ws(ow, sym_start + before + incl - mybits);
        for (uint32_t i = i0; i < i1; i++) {
          uint32_t c1, l1, c2, l2;
          sym_code(sym_at(i), s_ltab, s_dtab, is_static, &c1, &l1, &c2, &l2);
          ws.put(c1, l1);
          if (l2) ws.put(c2, l2);
        }
        if (tid == EMIT_T - 1) ws.put(eob_c, eob_l);
        ws.done();
      }
      if (is_static) {   // the block header
        if (tid == 0) {
          WordSink ws(ow, o);
          ws.put(2u, 3);
          ws.done();
        }
      } else if (tid < 64) {   // the header and send_all_trees by wave 0, into LDS words, then out
        const uint32_t lane = tid, sh = o & 31;
        for (uint32_t i = lane; i < EMIT_HDR_W; i += 64) s_hdr[i] = 0;
        wave_mem_sync();
        const int lcodes = B->lcodes, dcodes = B->dcodes, blcodes = B->blcodes;
        if (lane == 0)
          lds_or_bits(s_hdr, sh, 4u | (uint32_t)(lcodes - 257) << 3 | (uint32_t)(dcodes - 1) << 8 | (uint32_t)(blcodes - 4) << 13,
                      17);
        if ((int)lane < blcodes) lds_or_bits(s_hdr, sh + 17 + 3 * lane, s_btab[zd::bl_order((int)lane)] >> 16, 3);
        uint32_t pos = sh + 17 + 3 * (uint32_t)blcodes;
        pos = send_tree_wave(s_hdr, pos, s_ltab, lcodes - 1, s_btab, s_run);
        wave_mem_sync();
        pos = send_tree_wave(s_hdr, pos, s_dtab, dcodes - 1, s_btab, s_run);
        wave_mem_sync();
        const uint32_t nw = (pos + 31) >> 5, w0 = o >> 5;   // (the first and last words shared)
        for (uint32_t i = lane; i < nw; i += 64) {
          if (i == 0 || i == nw - 1) atomicOr(&ow[w0 + i], s_hdr[i]);
          else ow[w0 + i] = s_hdr[i];
        }
      }
      __syncthreads();
      if (tid == 0) s_off = blk_end;
      __syncthreads();
    }
    // the sync marker: 000, pad, 00 00 FF FF
    if (tid == 0) {
      const uint32_t pos = ((s_off + 3 + 7) & ~7u) >> 3;
      ob[pos + 2] = 0xff;   // (bytes past the last block are zero, and only thread 0 writes here now)
      ob[pos + 3] = 0xff;
      wsg_frame_desc o;
      o.payload_off = obase;
      o.payload_len = (uint32_t)(pos + 4) - ((fl & DF_FIN) ? 4u : 0u);
      o.opcode = a.desc[k].opcode;
      o.flags = (uint8_t)(((fl & DF_FIN) ? 0x80 : 0) | (((fl >> DF_RSV_SHIFT) & 7) << 4) | WSG_DESC_DEFLATED);
      o.status = 0;
      a.out_desc[k] = o;
    }
    __syncthreads();
    if (lds_out) {
      uint32_t* const og = (uint32_t*)ob_g;
      for (uint32_t i = tid; i < (uint32_t)((bytes + 3) >> 2); i += EMIT_T) og[i] = s_out[i];
    }
  }
}

// ------------------------------------------------------------------ k_defl_final
__global__ __launch_bounds__(256) void k_defl_final(DeflArgs a) {
  const uint32_t s = blockIdx.x, tid = threadIdx.x;
  const DeflSess fs = a.fs[s];
  wsg_deflate_state st = a.state[s];
  st.compressing = fs.compressing;
  if (!fs.has_deflater) {
    st.strstart = st.high_water = 0;
    st.insert = 0;
    st.has_deflater = 0;
  } else if (fs.last_call != ~0u && a.level > 0) {
    uint32_t sw = fs.sw_final;
    if (a.ftail[fs.last_call]) {   // the window slid inside the last frame's tail
      uint8_t* W = a.smem + (uint64_t)s * WSG_DEFLATE_SESSION_BYTES;
      uint16_t* hp = (uint16_t*)(W + zd::WINDOW_SIZE);
      // (the two ranges are disjoint: sw <= 2 WSIZE; 16-B pieces, eight in flight a thread)
      const uint32_t n = sw - zd::WSIZE, n16 = n >> 4;
      uint4* W16 = (uint4*)W;
      batched_for16(0, n16, [&](uint32_t i) { return W16[i + zd::WSIZE / 16]; }, [&](uint32_t i, uint4 v) { W16[i] = v; });
      for (uint32_t i = 16 * n16 + tid; i < n; i += blockDim.x) W[i] = W[i + zd::WSIZE];
      uint4* hp16 = (uint4*)hp;
      batched_for16(0, 2u * zd::WSIZE / 8, [&](uint32_t i) { return hp16[i]; }, [&](uint32_t i, uint4 v) {
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const uint32_t lo = w[e] & 0xffff, hi = w[e] >> 16;
          w[e] = (lo >= (uint32_t)zd::WSIZE ? lo - zd::WSIZE : 0) | (hi >= (uint32_t)zd::WSIZE ? hi - zd::WSIZE : 0) << 16;
        }
        hp16[i] = make_uint4(w[0], w[1], w[2], w[3]);
      });
      sw -= zd::WSIZE;
    }
    st.strstart = sw;
    st.high_water = fs.hw_final;
    st.insert = (uint16_t)(sw < 2 ? sw : 2);
    st.has_deflater = 1;
  } else if (fs.last_call != ~0u) {   // level 0: stored blocks, the window is never read
    st.has_deflater = 1;
  }
  if (tid == 0) a.state[s] = st;
}

// ------------------------------------------------------------------ k_defl_serial
// zlib's loop, one lane a session (levels 1-3, or any level with WSG_TUNE_DEFLATE_SERIAL)
__global__ __launch_bounds__(64) void k_defl_serial(DeflArgs a) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.n_sessions) return;
  Sums sm(a);
  const DeflSess fs = a.fs[s];
  wsg_deflate_state st = a.state[s];
  uint8_t* W = a.smem + (uint64_t)s * WSG_DEFLATE_SESSION_BYTES;
  zd::SerialState ss;
  ss.window = W;
  ss.head = (uint16_t*)(W + zd::WINDOW_SIZE);
  ss.prev = ss.head + zd::WSIZE;
  ss.strstart = st.strstart;
  ss.insert = st.insert;
  ss.high_water = st.high_water;
  ss.ins_h = 0;
  ss.match_start = ss.prev_match = 0;
  ss.cfg = zd::level_cfg(a.level);
  ss.sym = a.ssym + (uint64_t)s * zd::LIT_BUFSIZE;
  ss.tw = (zd::TreeWork*)a.tw + s;
  const uint64_t obase = sm.O[s];
  for (uint32_t k = a.session_first[s]; k < a.session_first[s + 1]; k++) {
    const uint32_t fl = a.fflags[k];
    if ((fl & DF_KIND) != PMD_CALL) {
      pass_or_empty(a, k, fl, obase);
      continue;
    }
    const wsg_frame_desc d = a.desc[k];
    ss.bw = zd::BitWriter{a.out + obase + a.fout[k], 0, 0, 0};
    if (a.level == 0) {
      zd::stored_call(&ss.bw, a.payload + d.payload_off, d.payload_len);
    } else {
      if (fl & DF_SEG) {   // a new Deflater: deflateInit2's CLEAR_HASH, strstart 0
        for (uint32_t h = 0; h < (uint32_t)zd::WSIZE; h++) ss.head[h] = 0;
        ss.strstart = 0;
        ss.insert = 0;
        ss.high_water = 0;
      }
      zd::serial_call(&ss, a.payload + d.payload_off, d.payload_len, a.level);
    }
    wsg_frame_desc o;
    o.payload_off = obase + a.fout[k];
    o.payload_len = (uint32_t)ss.bw.pos - ((fl & DF_FIN) ? 4u : 0u);
    o.opcode = d.opcode;
    o.flags = (uint8_t)(((fl & DF_FIN) ? 0x80 : 0) | (((fl >> DF_RSV_SHIFT) & 7) << 4) | WSG_DESC_DEFLATED);
    o.status = 0;
    a.out_desc[k] = o;
  }
  st.compressing = fs.compressing;
  if (!fs.has_deflater) {
    st.strstart = st.high_water = 0;
    st.insert = 0;
    st.has_deflater = 0;
  } else {
    st.has_deflater = 1;
    if (a.level > 0) {
      st.strstart = ss.strstart;
      st.high_water = ss.high_water;
      st.insert = (uint16_t)ss.insert;
    }
  }
  a.state[s] = st;
}

}  // namespace

size_t defl_treework_bytes() { return sizeof(zd::TreeWork); }

void launch_defl_plan(const DeflArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_defl_plan, dim3((a.n_sessions + 1 + 63) / 64), dim3(64), 0, s, a);
  hipLaunchKernelGGL(k_defl_scan, dim3(1), dim3(1024), 0, s, a);
}
void launch_defl_prep(const DeflArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_defl_prep, dim3(a.n_sessions), dim3(256), 0, s, a);
}
void launch_defl_links(const DeflArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_defl_links, dim3(a.n_sessions), dim3(64 * LINK_WAVES), 0, s, a);
}
void launch_defl_match(const DeflArgs& a, hipStream_t s) {
  uint64_t g = a.chunk_cap < 262144 ? a.chunk_cap : 262144;
  g = (g + 7) & ~7ull;   // a multiple of the 8 XCDs (k_defl_match's chunk order)
  hipLaunchKernelGGL(k_defl_match, dim3((uint32_t)(g ? g : 8)), dim3(64), 0, s, a);
}
void launch_defl_match_lds(const DeflArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_defl_match_lds, dim3(a.n_sessions), dim3(1024), 0, s, a);
}
void launch_defl_parse(const DeflArgs& a, hipStream_t s) {
#ifndef WSG_PARSE_T
#define WSG_PARSE_T 64   // (A/B: 32 = half-full waves, twice as many)
#endif
  hipLaunchKernelGGL(k_defl_parse, dim3((a.n_lanes + WSG_PARSE_T - 1) / WSG_PARSE_T), dim3(WSG_PARSE_T), 0, s, a);
}
void launch_defl_hist(const DeflArgs& a, hipStream_t s, uint64_t n_blocks) {
  hipLaunchKernelGGL(k_defl_hist, dim3((uint32_t)(n_blocks < 262144 ? (n_blocks ? n_blocks : 1) : 262144)), dim3(256), 0,
                     s, a);
}
void launch_defl_trees(const DeflArgs& a, hipStream_t s, uint64_t n_blocks) {
  uint64_t g = (n_blocks + TREE_LANES - 1) / TREE_LANES;
  hipLaunchKernelGGL(k_defl_trees, dim3((uint32_t)(g < 65536 ? (g ? g : 1) : 65536)), dim3(64 * TREE_WAVES), 0, s, a);
}
void launch_defl_emit(const DeflArgs& a, hipStream_t s) {
  uint64_t g = a.n_frames < 262144 ? a.n_frames : 262144;
  hipLaunchKernelGGL(k_defl_emit, dim3((uint32_t)(g ? g : 1)), dim3(EMIT_T), 0, s, a);
}
void launch_defl_final(const DeflArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_defl_final, dim3(a.n_sessions), dim3(256), 0, s, a);
}
void launch_defl_serial(const DeflArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_defl_serial, dim3((a.n_sessions + 63) / 64), dim3(64), 0, s, a);
}

}  // namespace ws
