// wsgpu_scan.h — wave/block scans of the per-frame aggregates used by the decode
// and encode pipelines: the payload-length prefix sum and the "last frame of a
// kind before k" max-scans that replace the reference's sequential per-session
// state (FrameDecoder.fragmentation, FrameUtf8Validator.context, FrameEncoder.closed).
#pragma once
#include "wsgpu_internal.h"

namespace ws {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t v, int d) {
  uint32_t lo = __shfl_up((unsigned)v, d, 64), hi = __shfl_up((unsigned)(v >> 32), d, 64);
  return ((uint64_t)hi << 32) | lo;
}

// Inclusive block scan (256 threads) of {sum, max a, max b, max c}; returns the
// thread's EXCLUSIVE values and the block totals.
struct Agg {
  uint64_t sum;
  int32_t m0, m1, m2;
};

__device__ __forceinline__ Agg agg_op(const Agg& x, const Agg& y) {
  Agg r;
  r.sum = x.sum + y.sum;
  r.m0 = x.m0 > y.m0 ? x.m0 : y.m0;
  r.m1 = x.m1 > y.m1 ? x.m1 : y.m1;
  r.m2 = x.m2 > y.m2 ? x.m2 : y.m2;
  return r;
}

// DPP move of a dword across the wave: lanes without a source (row_shr past the
// start of their row of 16, rows outside RM, lane 0 of wave_shr) keep `id`.
template <int CTRL, int RM>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v, uint32_t id) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, CTRL, RM, 0xf, false);
}
template <int CTRL, int RM>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v, uint64_t id) {
  return ((uint64_t)dpp_u32<CTRL, RM>((uint32_t)(v >> 32), (uint32_t)(id >> 32)) << 32) |
         dpp_u32<CTRL, RM>((uint32_t)v, (uint32_t)id);
}
constexpr int DPP_ROW_SHR1 = 0x111, DPP_ROW_SHR2 = 0x112, DPP_ROW_SHR4 = 0x114, DPP_ROW_SHR8 = 0x118;
constexpr int DPP_ROW_BCAST15 = 0x142, DPP_ROW_BCAST31 = 0x143, DPP_WAVE_SHR1 = 0x138;

// the element of the lane the DPP control names, the identity where there is none
template <int CTRL, int RM>
__device__ __forceinline__ Agg agg_dpp(const Agg& v) {
  Agg t;
  t.sum = dpp_u64<CTRL, RM>(v.sum, 0ull);
  t.m0 = (int32_t)dpp_u32<CTRL, RM>((uint32_t)v.m0, 0xffffffffu);
  t.m1 = (int32_t)dpp_u32<CTRL, RM>((uint32_t)v.m1, 0xffffffffu);
  t.m2 = (int32_t)dpp_u32<CTRL, RM>((uint32_t)v.m2, 0xffffffffu);
  return t;
}

constexpr Agg AGG_ID = {0ull, -1, -1, -1};

// inclusive wave scan of a 32-bit sum by DPP
__device__ __forceinline__ uint32_t wave_incl_sum_u32(uint32_t v) {
  v += dpp_u32<DPP_ROW_SHR1, 0xf>(v, 0u);
  v += dpp_u32<DPP_ROW_SHR2, 0xf>(v, 0u);
  v += dpp_u32<DPP_ROW_SHR4, 0xf>(v, 0u);
  v += dpp_u32<DPP_ROW_SHR8, 0xf>(v, 0u);
  v += dpp_u32<DPP_ROW_BCAST15, 0xa>(v, 0u);
  v += dpp_u32<DPP_ROW_BCAST31, 0xc>(v, 0u);
  return v;
}

// Scans over any element type T with agg_op(T, T) (associative, applied in frame
// order: it need not commute) and agg_dpp<CTRL, RM>(T) (identity where no source).
// The wave scan is DPP moves (VALU, no LDS round trip a step): Hillis-Steele inside
// each row of 16 lanes (row_shr 1, 2, 4, 8), then row 0's total into row 1 and row
// 2's into row 3 (row_bcast:15), then rows 0-1's total into rows 2-3 (row_bcast:31).
template <class T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  v = agg_op(agg_dpp<DPP_ROW_SHR1, 0xf>(v), v);
  v = agg_op(agg_dpp<DPP_ROW_SHR2, 0xf>(v), v);
  v = agg_op(agg_dpp<DPP_ROW_SHR4, 0xf>(v), v);
  v = agg_op(agg_dpp<DPP_ROW_SHR8, 0xf>(v), v);
  v = agg_op(agg_dpp<DPP_ROW_BCAST15, 0xa>(v), v);
  v = agg_op(agg_dpp<DPP_ROW_BCAST31, 0xc>(v), v);
  return v;
}

// Block-wide exclusive scan; nthreads = blockDim.x (multiple of 64, <= 1024).
template <class T>
__device__ inline T block_excl_scan_t(T v, T* total, const T id) {
  __shared__ T wsum[16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  T inc = wave_incl_scan(v);
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  T pre = id, tot = id;
  for (int i = 0; i < nw; ++i) {
    if (i < wid) pre = agg_op(pre, wsum[i]);
    tot = agg_op(tot, wsum[i]);
  }
  __syncthreads();
  // exclusive within the wave: inclusive of lane-1 (lane 0: the identity)
  T ex = agg_dpp<DPP_WAVE_SHR1, 0xf>(inc);
  if (lane == 0) ex = id;
  *total = tot;
  return agg_op(pre, ex);
}

__device__ inline Agg block_excl_scan(Agg v, Agg* total) { return block_excl_scan_t(v, total, AGG_ID); }

// session owning frame k: largest s in [lo, hi] with session_first[s] <= k
__device__ __forceinline__ uint32_t find_session_in(const uint32_t* sf, uint32_t lo, uint32_t hi, uint64_t k) {
  while (lo < hi) {
    uint32_t mid = (lo + hi + 1) >> 1;
    if ((uint64_t)sf[mid] <= k) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}
__device__ __forceinline__ uint32_t find_session(const uint32_t* sf, uint32_t n_sessions, uint64_t k) {
  uint32_t lo = 0, hi = n_sessions ? n_sessions - 1 : 0;
  while (lo < hi) {
    uint32_t mid = (lo + hi + 1) >> 1;
    if ((uint64_t)sf[mid] <= k) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Session of frame k when a wave's 64 lanes take frames k & ~63 .. +63: two
// wave-uniform searches (scalar loads) bound the sessions of the wave's frames, and
// a lane searches only inside those bounds — not at all when they share a session.
__device__ __forceinline__ uint32_t wave_find_session(const uint32_t* sf, uint32_t n_sessions, uint64_t n_frames,
                                                      uint64_t k) {
  const uint32_t kw = __builtin_amdgcn_readfirstlane((uint32_t)(k & ~63ull));  // (frame indices < 2^30)
  const uint64_t kl = kw + 63u < n_frames ? kw + 63u : n_frames - 1;
  const uint32_t s_lo = find_session(sf, n_sessions, kw);
  if (s_lo + 1 >= n_sessions || sf[s_lo + 1] > kl) return s_lo;  // one session
  const uint32_t s_hi = find_session_in(sf, s_lo + 1, n_sessions - 1, kl);
  return find_session_in(sf, s_lo, s_hi, k);
}

// Workgroups are dealt round-robin to the 8 XCDs (blocks b and b+8 share one);
// give each XCD a contiguous run of pieces so the source lines two neighbouring
// pieces share (funnel block, UTF-8 carry word) meet in the same L2.  Bijective
// for any grid (cdna_hip_programming.md §5.5 T1).
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t n) {
  const uint32_t q = n / 8u, r = n % 8u, x = b % 8u, i = b / 8u;
  return (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + i;
}

}  // namespace ws
