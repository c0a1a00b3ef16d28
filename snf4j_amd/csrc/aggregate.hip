// aggregate.hip — FrameAggregator on gfx950 (FrameAggregator.java:72-104,
// PayloadAggregator.java:32-73), run over a decoded batch.
//
// The reference keeps one aggregated frame per session and appends each
// continuation's payload to it.  Here the per-session sequence becomes scans:
//   an aggregated frame is open before frame k  <=>  the last TEXT/BINARY non-FIN
//   frame ("start") before k comes after the last FIN continuation ("end") before
//   k (a FIN continuation closes an open frame and leaves a closed one closed;
//   a start opens or replaces) — two max-scans, session-segmented by comparing
//   with session_first, the carried-in state standing for "before the batch";
// member frames (starts, and continuations while open) have their payload bytes
// laid back to back in agg_out by a sum-scan, so every aggregated message is one
// contiguous range; the "too big" test of continuation k (:92-94) is the bytes of
// its message before k (+ the bytes carried in) + its own length > max.
//
//   k_agg_a      thread per frame: class bits, block maxima of start / end indices
//   k_agg_scan   one workgroup: exclusive scans of the block aggregates (only above
//                AGG_FOLD_MAX blocks: below, k_agg_b folds the maxima and k_agg_c the
//                sums of the blocks before its own)
//   k_agg_b      thread per frame: open-before-k, membership, emit flag; block sums
//                of member bytes and emitted frames
//   k_agg_c      thread per frame: the exclusive prefix of the block sums before its
//                block (staged in LDS, so a member's message start in an earlier block
//                is one LDS read), "too big" test, output descriptors, and the gather
//                units of each member (<= 1 KiB of agg_out, one source range)
//   k_agg_gather one wave per 2 gather units (WSG_TUNE_AGG_UNITS) (grid-stride: the
//                unit count is known only on the device): 16-B aligned stores,
//                sources funnelled from aligned loads; its first waves also do
//                k_agg_final's work, a thread per session: result, carry-out state,
//                PENDING entry (one launch less)
#include "wsgpu_internal.h"
#include "wsgpu_scan.h"

namespace ws {

constexpr uint32_t AG_VALID = 1u;    // delivered by the decoder (the aggregator sees it)
constexpr uint32_t AG_START = 2u;    // TEXT/BINARY, not FIN: opens (or replaces) the aggregated frame
constexpr uint32_t AG_END = 4u;      // CONTINUATION, FIN
constexpr uint32_t AG_CONT = 8u;     // CONTINUATION
constexpr uint32_t AG_MEMBER = 16u;  // its payload belongs to the aggregated frame
constexpr uint32_t AG_EMIT = 32u;    // emits an output frame (itself, or the aggregated frame)
constexpr uint32_t AG_CARRY = 64u;   // member of the frame carried in from an earlier batch

// grids up to this many blocks fold the block aggregates before their own in k_agg_b /
// k_agg_c (no k_agg_scan launch); k_agg_c stages the sums' prefixes in LDS (16 B a block)
#ifndef WSG_AGG_FOLD_MAX
#define WSG_AGG_FOLD_MAX 3072  // (configs[2]: 2,128 blocks fold; k_agg_c stages 16 B a block: 48 KiB of LDS at most)
#endif
constexpr uint32_t AGG_FOLD_MAX = WSG_AGG_FOLD_MAX;
uint32_t agg_fold_bound() { return AGG_FOLD_MAX; }
__device__ __forceinline__ uint64_t agg_pos(const AggArgs& a, uint64_t j) { return a.pl[j] + a.pre_sum[j / ABLOCK]; }
// cl / blk_cnt pack two counts: emitted frames (bits 0-31) and gather units (32-63)
__device__ __forceinline__ uint64_t agg_cnt(const AggArgs& a, uint64_t j) {
  return (a.cl[j] + a.pre_cnt[j / ABLOCK]) & 0xffffffffull;
}
// A member's bytes go out as gather units: 64 16-B blocks of agg_out each (the first
// and last block partial), ceil((m + 15) / 1 KiB) of them for m bytes at any
// alignment (one may come out empty).  A unit copies one source range: no lookups.
__device__ __forceinline__ uint32_t agg_units(uint64_t m) { return m ? (uint32_t)((m + 15u + PIECE - 1u) / PIECE) : 0u; }
__device__ __forceinline__ uint64_t agg_mi(const AggArgs& a, uint64_t j) { return (a.cl[j] + a.pre_cnt[j / ABLOCK]) >> 32; }

// ------------------------------------------------------------------ k_agg_a
__global__ __launch_bounds__(ABLOCK) void k_agg_a(AggArgs a) {
  const uint64_t k = (uint64_t)blockIdx.x * ABLOCK + threadIdx.x;
  Agg v = AGG_ID;
  if (k < a.n_frames) {
    const uint32_t s = wave_find_session(a.session_first, a.n_sessions, a.n_frames, k);
    const bool valid = k - a.session_first[s] < a.dec_result[s].n_delivered;
    uint32_t c = 0;
    if (valid) {
      const wsg_frame_desc d = a.desc[k];
      const bool fin = (d.flags & 0x80u) != 0;
      c = AG_VALID;
      if ((d.opcode == WSG_OP_TEXT || d.opcode == WSG_OP_BINARY) && !fin) c |= AG_START;
      if (d.opcode == WSG_OP_CONTINUATION) c |= AG_CONT | (fin ? AG_END : 0u);
    }
    a.code[k] = c;
    a.sess[k] = s;
    v.m0 = (c & AG_START) ? (int32_t)k : -1;
    v.m1 = (c & AG_END) ? (int32_t)k : -1;
  }
  Agg tot;
  block_excl_scan(v, &tot);
  if (threadIdx.x == 0) {
    a.blk_max[blockIdx.x] = tot.m0;
    a.blk_max[a.nblk + blockIdx.x] = tot.m1;
  }
}

// ------------------------------------------------------------------ k_agg_scan
// One workgroup: exclusive scans of the block aggregates in place, 4 consecutive
// entries per thread (one pass up to 4096 blocks: a pass is a dependent load ->
// block scan -> store round trip).  sums = 0: the start / end maxima; sums = 1:
// member bytes and emitted frames (+ the totals).
__global__ __launch_bounds__(1024) void k_agg_scan(AggArgs a, int sums) {
  Agg carry = AGG_ID;    // maxima (sums == 0) or member bytes (sums == 1)
  uint64_t carry_n = 0;  // emitted frames (sums == 1)
  for (uint32_t base = 0; base < a.nblk; base += 4096) {
    const uint32_t b0 = base + threadIdx.x * 4;
    Agg e[4], t = AGG_ID, tot;
    uint64_t en[4], tn = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool in = b0 + i < a.nblk;
      e[i] = AGG_ID;
      en[i] = 0;
      if (sums) {
        if (in) {
          e[i].sum = a.blk_sum[b0 + i];
          en[i] = a.blk_cnt[b0 + i];
        }
        tn += en[i];
      } else if (in) {
        e[i].m0 = a.blk_max[b0 + i];
        e[i].m1 = a.blk_max[a.nblk + b0 + i];
      }
      t = agg_op(t, e[i]);
    }
    // the emitted-frame counts ride in the m-fields' place: a second scan of sums
    Agg ex = block_excl_scan(t, &tot);
    Agg nv = AGG_ID, ntot;
    nv.sum = tn;
    Agg nex = AGG_ID;
    if (sums) nex = block_excl_scan(nv, &ntot);
    ex = agg_op(carry, ex);
    uint64_t xn = carry_n + nex.sum;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (b0 + i < a.nblk) {
        if (sums) {
          a.pre_sum[b0 + i] = ex.sum;
          a.pre_cnt[b0 + i] = xn;
        } else {
          a.blk_max[b0 + i] = ex.m0;
          a.blk_max[a.nblk + b0 + i] = ex.m1;
        }
      }
      ex = agg_op(ex, e[i]);
      xn += en[i];
    }
    carry = agg_op(carry, tot);
    if (sums) carry_n += ntot.sum;
  }
  if (sums && threadIdx.x == 0) {
    *a.agg_total = carry.sum;
    *a.n_units = carry_n >> 32;
  }
}

// ------------------------------------------------------------------ k_agg_b
__global__ __launch_bounds__(ABLOCK) void k_agg_b(AggArgs a) {
  const uint64_t k = (uint64_t)blockIdx.x * ABLOCK + threadIdx.x;
  const bool live = k < a.n_frames;
  uint32_t c = live ? a.code[k] : 0u;
  Agg v = AGG_ID;
  v.m0 = (c & AG_START) ? (int32_t)k : -1;
  v.m1 = (c & AG_END) ? (int32_t)k : -1;
  Agg tot;
  Agg ex = block_excl_scan(v, &tot);
  Agg w = AGG_ID;
  uint64_t emit = 0;  // emitted frame (bit 0) | gather units (bits 32-63)
  // the start / end maxima of every frame before this block: up to 4096 blocks the
  // block folds k_agg_a's block maxima itself (coalesced; max commutes), so the
  // first k_agg_scan launch is skipped; beyond, k_agg_scan left the exclusive maxima
  int32_t bs, be;
  if (a.nblk <= a.fold_max) {
    Agg f = AGG_ID, ft;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += ABLOCK) {
      const int32_t x0 = a.blk_max[b], x1 = a.blk_max[a.nblk + b];
      f.m0 = x0 > f.m0 ? x0 : f.m0;
      f.m1 = x1 > f.m1 ? x1 : f.m1;
    }
    block_excl_scan(f, &ft);
    bs = ft.m0;
    be = ft.m1;
  } else {
    bs = a.blk_max[blockIdx.x];
    be = a.blk_max[a.nblk + blockIdx.x];
  }
  if (live) {
    const int32_t ls = ex.m0 > bs ? ex.m0 : bs, le = ex.m1 > be ? ex.m1 : be;
    a.last[k] = ls;
    a.last[a.n_frames + k] = le;
    if (c & AG_VALID) {
      const uint32_t s = a.sess[k];
      const int32_t sf = (int32_t)a.session_first[s];
      const bool in_batch = (ls > le ? ls : le) >= sf;
      const bool open = in_batch ? ls > le : a.state[s].open != 0;  // FrameAggregator.frame != null
      const bool member = (c & AG_START) || ((c & AG_CONT) && open);
      const bool em = !member || ((c & AG_END) && open);  // out.add(data) (:103)
      if (member) {
        c |= AG_MEMBER;
        if (!(c & AG_START) && ls < sf) c |= AG_CARRY;
        w.sum = a.desc[k].payload_len;
        emit |= (uint64_t)agg_units(w.sum) << 32;
      }
      if (em) { c |= AG_EMIT; emit |= 1u; }
      a.code[k] = c;
    }
  }
  Agg tw;
  const Agg ew = block_excl_scan(w, &tw);
  Agg e = AGG_ID;
  e.sum = emit;
  Agg te;
  const Agg ee = block_excl_scan(e, &te);
  if (live) {
    a.pl[k] = ew.sum;
    a.cl[k] = ee.sum;
  }
  if (threadIdx.x == 0) {
    a.blk_sum[blockIdx.x] = tw.sum;
    a.blk_cnt[blockIdx.x] = te.sum;
  }
}

// ------------------------------------------------------------------ k_agg_c
// FOLD: the block's own fold of the block sums before it (as k_link folds k_parse's
// aggregates): loaded coalesced into LDS, each thread folds a contiguous run, a block
// scan of the runs, then the run's exclusive prefixes written back in place, so the
// prefix of ANY block up to this one (a message's first member may be in an earlier
// block) is an LDS read; the block's own prefix goes to pre_sum / pre_cnt for the
// gather and the final step, and the last block leaves the totals.
template <bool FOLD>
__global__ __launch_bounds__(ABLOCK) void k_agg_c(AggArgs a) {
  extern __shared__ uint64_t fold[];  // FOLD: [2][blockIdx.x + 1] (sum, cnt) exclusive prefixes
  const uint64_t k = (uint64_t)blockIdx.x * ABLOCK + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool live = k < a.n_frames;
  const uint32_t B = blockIdx.x;
  if (FOLD) {
    uint64_t* const fs = fold;
    uint64_t* const fc = fold + (B + 1);
    for (uint32_t b = threadIdx.x; b <= B; b += ABLOCK) {
      fs[b] = a.blk_sum[b];
      fc[b] = a.blk_cnt[b];
    }
    __syncthreads();
    const uint32_t n = B + 1, per = (n + ABLOCK - 1) / ABLOCK;
    const uint32_t b0 = threadIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
    Agg t = AGG_ID;
    uint64_t tc = 0;
    for (uint32_t b = b0; b < b1; ++b) {
      t.sum += fs[b];
      tc += fc[b];
    }
    Agg tot, totc;
    const uint64_t xs = block_excl_scan(t, &tot).sum;
    Agg tcv = AGG_ID;
    tcv.sum = tc;
    const uint64_t xc = block_excl_scan(tcv, &totc).sum;
    __syncthreads();  // (every run is read before any is overwritten)
    uint64_t rs = xs, rc = xc;
    for (uint32_t b = b0; b < b1; ++b) {
      const uint64_t vs = fs[b], vc = fc[b];
      fs[b] = rs;
      fc[b] = rc;
      rs += vs;
      rc += vc;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      a.pre_sum[B] = fs[B];
      a.pre_cnt[B] = fc[B];
      if (B + 1 == a.nblk) {  // the batch's totals (k_agg_scan's otherwise)
        *a.agg_total = tot.sum;
        *a.n_units = totc.sum >> 32;
      }
    }
  }
  // the global position / counts of frame j <= this block's last frame
  auto pos_of = [&](uint64_t j) -> uint64_t { return a.pl[j] + (FOLD ? fold[j / ABLOCK] : a.pre_sum[j / ABLOCK]); };
  auto cnt_of = [&](uint64_t j) -> uint64_t {
    return (a.cl[j] + (FOLD ? fold[(B + 1) + j / ABLOCK] : a.pre_cnt[j / ABLOCK])) & 0xffffffffull;
  };
  auto mi_of = [&](uint64_t j) -> uint64_t {
    return (a.cl[j] + (FOLD ? fold[(B + 1) + j / ABLOCK] : a.pre_cnt[j / ABLOCK])) >> 32;
  };
  const uint32_t c = live ? a.code[k] : 0u;
  uint64_t pos = live ? pos_of(k) : 0ull, src = 0;
  uint32_t mlen = 0;
  if (c & AG_VALID) {
    const uint32_t s = a.sess[k];
    const uint32_t sf = a.session_first[s];
    const wsg_frame_desc d = a.desc[k];
    if (c & AG_MEMBER) {
      mlen = d.payload_len;
      src = d.payload_off;
    }
    uint64_t first = 0;
    wsg_agg_state st = {0, 0, 0, 0, 0u};
    if ((c & AG_MEMBER) || (c & AG_END)) {
      st = a.state[s];
      first = (c & AG_START) ? k : ((c & AG_CARRY) ? (uint64_t)sf : (uint64_t)a.last[k]);
    }
    if ((c & AG_MEMBER) && !(c & AG_START)) {  // a continuation of an open aggregated frame
      const uint64_t held = ((c & AG_CARRY) ? (uint64_t)st.length : 0ull) + (pos - pos_of(first));
      if ((int64_t)(held + d.payload_len) > a.max_len)  // tooBig, FrameAggregator.java:92-94
        atomicMin((unsigned long long*)&a.sess_err[s], (unsigned long long)k);
    }
    if (c & AG_EMIT) {
      wsg_frame_desc o;
      if (c & AG_MEMBER) {  // the FIN continuation: the aggregated frame (:97-100)
        const uint64_t p0 = pos_of(first);
        uint32_t op, rsv;
        if (c & AG_CARRY) {
          op = st.opcode;
          rsv = st.rsv;
        } else {
          const wsg_frame_desc ds = a.desc[first];
          op = ds.opcode;
          rsv = (ds.flags >> 4) & 7u;
        }
        o.payload_off = p0;
        o.payload_len = (uint32_t)(pos + d.payload_len - p0);
        o.opcode = (uint8_t)op;
        o.flags = (uint8_t)(0x80u | (rsv << 4) | WSG_AGG_IN_AGG | ((c & AG_CARRY) ? WSG_AGG_PREFIXED : 0u));
      } else {  // passed through unchanged (:103)
        o = d;
        o.flags = (uint8_t)(d.flags & 0xF1u);
      }
      o.status = 0;
      a.out_desc[(uint64_t)sf + s + (cnt_of(k) - cnt_of(sf))] = o;
    }
  }
  // the member's gather units, written cooperatively (as decode.hip k_link): a wave
  // scan of the counts, then lane i writes the wave's units i, i+64, ... after a
  // shuffle search for the owner.  Unit u covers agg_out blocks [pos/16 + 64u, +64)
  // clipped to the member: info = its first output byte | its byte count << 48,
  // mask:frame = the source offset of that byte.
  const uint32_t cnt = agg_units(mlen);
  const uint64_t u0 = cnt ? mi_of(k) : 0ull;
  uint32_t cum = cnt;
  cum = wave_incl_sum_u32(cum);
  const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)cum, 63);
  cum -= cnt;
  if (!T) return;
  for (uint32_t t = lane; t < ((T + 63u) & ~63u); t += 64) {
    int o = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1)
      if ((uint32_t)__shfl((int)cum, o + step, 64) <= t) o += step;
    const uint32_t o_cum = (uint32_t)__shfl((int)cum, o, 64);
    const uint64_t o_u0 = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(u0 >> 32), o, 64) << 32) |
                          (uint32_t)__shfl((int)(uint32_t)u0, o, 64);
    const uint64_t o_pos = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(pos >> 32), o, 64) << 32) |
                           (uint32_t)__shfl((int)(uint32_t)pos, o, 64);
    const uint64_t o_src = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(src >> 32), o, 64) << 32) |
                           (uint32_t)__shfl((int)(uint32_t)src, o, 64);
    const uint32_t o_len = (uint32_t)__shfl((int)mlen, o, 64);
    if (t >= T) continue;
    const uint64_t u = o_u0 + (t - o_cum);
    if (u >= a.n_pieces) continue;  // holds bytes at or beyond agg_cap only
    const uint64_t b0 = ((o_pos >> 4) + (uint64_t)(t - o_cum) * 64u) * 16u;
    const uint64_t ubs = b0 > o_pos ? b0 : o_pos;
    const uint64_t ube = b0 + PIECE < o_pos + o_len ? b0 + PIECE : o_pos + o_len;
    const uint64_t s0 = o_src + (ubs - o_pos);
    PieceDesc pd;
    pd.info = (ubs & PD_SRC_MASK) | ((ube > ubs ? ube - ubs : 0ull) << PD_NB_SHIFT);
    pd.mask = (uint32_t)s0;
    pd.frame = (uint32_t)(s0 >> 32);
    a.pieces[u] = pd;
  }
}

// ------------------------------------------------------------------ k_agg_final
// (run by k_agg_gather's first waves, a thread a session)
__device__ void agg_final_one(const AggArgs& a, uint32_t s) {
  const uint32_t sf = a.session_first[s];
  const uint32_t nd = a.dec_result[s].n_delivered;
  wsg_agg_state st = a.state[s];
  wsg_session_result res = {0u, 0u, 0u, 0};
  const uint64_t fe = a.sess_err[s];
  if (fe != ~0ull) a.sess_err[s] = ~0ull;  // back to the idle state for the next batch
  const uint64_t base = (uint64_t)sf + s;
  if (nd == 0) {
    if (st.open) {  // the carried frame stays open: an empty PENDING entry
      wsg_frame_desc o = {0ull, 0u, st.opcode, (uint8_t)((st.rsv << 4) | WSG_AGG_IN_AGG | WSG_AGG_PREFIXED |
                                                        WSG_AGG_PENDING), 0};
      a.out_desc[base] = o;
    }
    a.out_result[s] = res;
    return;
  }
  const uint64_t cs = agg_cnt(a, sf);
  if (fe != ~0ull) {  // "Too big payload for aggregated frame" + CloseFrame(1009), :66-69
    res.n_delivered = (uint32_t)(agg_cnt(a, fe) - cs);
    res.error = WSG_E_AGG_TOO_BIG;
    res.close_code = WSG_CLOSE_TOO_BIG;
    res.detail = (int64_t)(fe - sf);
    // the aggregator keeps the open frame (without the failing fragment)
    const uint32_t c = a.code[fe];
    const uint64_t first = (c & AG_CARRY) ? (uint64_t)sf : (uint64_t)a.last[fe];
    const uint64_t inb = agg_pos(a, fe) - agg_pos(a, first);
    if (!(c & AG_CARRY)) {
      const wsg_frame_desc ds = a.desc[first];
      st.opcode = ds.opcode;
      st.rsv = (ds.flags >> 4) & 7u;
      st.length = (uint32_t)inb;
    } else {
      st.length += (uint32_t)inb;
    }
    st.open = 1;
    a.state[s] = st;
    a.out_result[s] = res;
    return;
  }
  const uint64_t L = (uint64_t)sf + nd - 1;
  const uint32_t c = a.code[L];
  res.n_delivered = (uint32_t)(agg_cnt(a, L) + ((c & AG_EMIT) ? 1u : 0u) - cs);
  bool open;
  if (c & AG_START) open = true;
  else if (c & AG_END) open = false;
  else {
    const int32_t ls = a.last[L], le = a.last[a.n_frames + L];
    open = (ls > le ? ls : le) >= (int32_t)sf ? ls > le : st.open != 0;
  }
  if (open) {
    const int32_t ls = (c & AG_START) ? (int32_t)L : a.last[L];
    const bool carry = ls < (int32_t)sf;
    const uint64_t first = carry ? (uint64_t)sf : (uint64_t)ls;
    const uint64_t p0 = agg_pos(a, first);
    const uint64_t inb = agg_pos(a, L) + ((c & AG_MEMBER) ? a.desc[L].payload_len : 0u) - p0;
    if (!carry) {
      const wsg_frame_desc ds = a.desc[first];
      st.opcode = ds.opcode;
      st.rsv = (ds.flags >> 4) & 7u;
      st.length = (uint32_t)inb;
    } else {
      st.length += (uint32_t)inb;
    }
    st.open = 1;
    wsg_frame_desc o;
    o.payload_off = p0;
    o.payload_len = (uint32_t)inb;
    o.opcode = st.opcode;
    o.flags = (uint8_t)((st.rsv << 4) | WSG_AGG_IN_AGG | WSG_AGG_PENDING | (carry ? WSG_AGG_PREFIXED : 0u));
    o.status = 0;
    a.out_desc[base + res.n_delivered] = o;
  } else {
    st.open = 0;
    st.opcode = 0;
    st.rsv = 0;
    st.length = 0;
  }
  a.state[s] = st;
  a.out_result[s] = res;
}

// ------------------------------------------------------------------ k_agg_gather
__device__ __forceinline__ uint32_t ag_dpp_from_next(uint32_t v, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x130, 0xf, 0xf, false);
}

// bytes [lo, hi) of the 16-B block at agg_out + o (a unit's partial first or last
// block: the rest of the block belongs to the neighbouring member)
__device__ __forceinline__ void ag_store_part(const AggArgs& a, uint64_t o, uint32_t lo, uint32_t hi, uint64_t lim,
                                              const uint32_t w[4]) {
  if (o + hi > lim) hi = o < lim ? (uint32_t)(lim - o) : 0u;
  for (uint32_t i = lo; i < hi; ++i) a.agg_out[o + i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
}

// One wave per N gather units, grid-stride over the unit groups: the next group's
// descriptors are loaded a group ahead, every unit's source blocks are loaded before
// any unit is stored (the kernel is latency-bound).  Lane l of a unit
// stores agg_out block ubs/16 + l: 16 bytes funnelled by the unit's (wave-uniform)
// source shift from its own aligned source block and its right neighbour's (DPP).
template <int N>
__global__ __launch_bounds__(64) void k_agg_gather(AggArgs a, uint64_t src_lim) {
  const int lane = threadIdx.x;
  {  // k_agg_final's work (it needs only the plan): a thread a session in the first waves
    const uint64_t fs = (uint64_t)blockIdx.x * 64u + (uint64_t)lane;
    if (fs < a.n_sessions) agg_final_one(a, (uint32_t)fs);
  }
  if (!a.n_frames) return;  // (no plan ran: no units)
  const uint64_t total = *a.agg_total;
  const uint64_t lim = total < a.agg_cap ? total : a.agg_cap;
  const uint64_t nu0 = *a.n_units;
  const uint64_t nu = nu0 < a.n_pieces ? nu0 : a.n_pieces;
  const uint64_t nq = (nu + N - 1) / N;
  uint64_t q = blockIdx.x;
  PieceDesc dn[N];  // the next group's descriptors, loaded a group ahead
#pragma unroll
  for (int i = 0; i < N; ++i) dn[i] = q * N + i < nu ? a.pieces[q * N + i] : PieceDesc{0ull, 0u, 0u};
  for (; q < nq; q += gridDim.x) {
    PieceDesc d[N];
    u32x4 A[N], nx[N];
#pragma unroll
    for (int i = 0; i < N; ++i) d[i] = dn[i];
    const uint64_t qn = q + gridDim.x;
#pragma unroll
    for (int i = 0; i < N; ++i) dn[i] = qn * N + i < nu ? a.pieces[qn * N + i] : PieceDesc{0ull, 0u, 0u};
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const uint64_t ubs = d[i].info & PD_SRC_MASK;
      const uint32_t nb = (uint32_t)(d[i].info >> PD_NB_SHIFT) & 2047u;
      const uint32_t head = (uint32_t)ubs & 15u;
      const uint64_t s0 = ((uint64_t)d[i].frame << 32) | d[i].mask;
      const uint32_t span = head + nb;  // bytes of the unit's blocks from the first block's start
      A[i] = (u32x4){0u, 0u, 0u, 0u};
      nx[i] = A[i];
      if (!nb) continue;
      const uint64_t sb = s0 - head;  // source of the first block's byte 0 (wraps below 0: slow path)
      const uint64_t a16 = sb & ~15ull;
      if (s0 >= head && a16 + PIECE + 16u <= src_lim) {
        // source blocks [a16, a16 + sh + span): lane l's, and the one after the wave's
        const uint32_t need = ((uint32_t)sb & 15u) + span;
        if ((uint32_t)lane * 16u < need) A[i] = *(const u32x4*)(a.payload + a16 + (uint64_t)lane * 16u);
        if (need > PIECE) nx[i] = *(const u32x4*)(a.payload + a16 + PIECE);
      } else {  // near either end of the payload buffer: byte loads
        uint32_t dd[4] = {0u, 0u, 0u, 0u}, ee[4] = {0u, 0u, 0u, 0u};
        for (uint32_t b = 0; b < 16u; ++b) {
          const uint64_t x = sb + lane * 16u + b, y = sb + PIECE + b;  // (sb + .. wraps back above 0)
          if (x < src_lim) dd[b >> 2] |= (uint32_t)a.payload[x] << (8 * (b & 3));
          if (y < src_lim) ee[b >> 2] |= (uint32_t)a.payload[y] << (8 * (b & 3));
        }
        // bytes already funnelled: shift 0 below
        A[i] = (u32x4){dd[0], dd[1], dd[2], dd[3]};
        nx[i] = (u32x4){ee[0], ee[1], ee[2], ee[3]};
        d[i].info |= 1ull << 63;  // marks the unaligned-load path
      }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const uint64_t ubs = d[i].info & PD_SRC_MASK;
      const uint32_t nb = (uint32_t)(d[i].info >> PD_NB_SHIFT) & 2047u;
      if (!nb) continue;
      const uint32_t head = (uint32_t)ubs & 15u;
      const uint64_t s0 = ((uint64_t)d[i].frame << 32) | d[i].mask;
      const uint32_t sh = (d[i].info >> 63) ? 0u : (uint32_t)(s0 - head) & 15u, b = sh & 3u;
      const uint32_t W0 = A[i].x, W1 = A[i].y, W2 = A[i].z, W3 = A[i].w;
      const uint32_t W4 = ag_dpp_from_next(A[i].x, nx[i].x), W5 = ag_dpp_from_next(A[i].y, nx[i].y);
      const uint32_t W6 = ag_dpp_from_next(A[i].z, nx[i].z), W7 = ag_dpp_from_next(A[i].w, nx[i].w);
      uint32_t w[4];
      switch (sh >> 2) {  // wave-uniform
        case 0: w[0] = alignbyte(W1, W0, b); w[1] = alignbyte(W2, W1, b); w[2] = alignbyte(W3, W2, b); w[3] = alignbyte(W4, W3, b); break;
        case 1: w[0] = alignbyte(W2, W1, b); w[1] = alignbyte(W3, W2, b); w[2] = alignbyte(W4, W3, b); w[3] = alignbyte(W5, W4, b); break;
        case 2: w[0] = alignbyte(W3, W2, b); w[1] = alignbyte(W4, W3, b); w[2] = alignbyte(W5, W4, b); w[3] = alignbyte(W6, W5, b); break;
        default: w[0] = alignbyte(W4, W3, b); w[1] = alignbyte(W5, W4, b); w[2] = alignbyte(W6, W5, b); w[3] = alignbyte(W7, W6, b); break;
      }
      const uint32_t span = head + nb, l16 = (uint32_t)lane * 16u;
      if (l16 >= span) continue;
      const uint64_t o = (ubs & ~15ull) + l16;
      const uint32_t lo = lane ? 0u : head, hi = span - l16 < 16u ? span - l16 : 16u;
      if (lo == 0 && hi == 16u && o + 16u <= lim)
        __builtin_nontemporal_store((u32x4){w[0], w[1], w[2], w[3]}, (u32x4*)(a.agg_out + o));
      else
        ag_store_part(a, o, lo, hi, lim, w);
    }
  }
}

// ------------------------------------------------------------------ launchers
void launch_agg_plan(const AggArgs& a, hipStream_t s) {
  if (!a.n_frames) return;
  hipLaunchKernelGGL(k_agg_a, dim3(a.nblk), dim3(ABLOCK), 0, s, a);
  const bool fold = a.nblk <= a.fold_max;
  if (!fold) hipLaunchKernelGGL(k_agg_scan, dim3(1), dim3(1024), 0, s, a, 0);
  hipLaunchKernelGGL(k_agg_b, dim3(a.nblk), dim3(ABLOCK), 0, s, a);
  if (fold) {
    hipLaunchKernelGGL(k_agg_c<true>, dim3(a.nblk), dim3(ABLOCK), 2 * a.nblk * sizeof(uint64_t), s, a);
  } else {
    hipLaunchKernelGGL(k_agg_scan, dim3(1), dim3(1024), 0, s, a, 1);
    hipLaunchKernelGGL(k_agg_c<false>, dim3(a.nblk), dim3(ABLOCK), 0, s, a);
  }
}
void launch_agg_gather(const AggArgs& a, hipStream_t s, uint64_t src_lim, int per_wave, uint32_t grid_cap) {
  // grid-stride over the units (their number is known only on the device; n_pieces bounds it);
  // at least a wave per 64 sessions for the final step
  const uint64_t nq = (a.n_pieces + per_wave - 1) / per_wave;
  uint64_t g = nq < grid_cap ? nq : grid_cap;
  const uint64_t gs = ((uint64_t)a.n_sessions + 63) / 64;
  if (g < gs) g = gs;
  if (!g) return;
  if (per_wave == 1) hipLaunchKernelGGL((k_agg_gather<1>), dim3((uint32_t)g), dim3(64), 0, s, a, src_lim);
  else if (per_wave == 4) hipLaunchKernelGGL((k_agg_gather<4>), dim3((uint32_t)g), dim3(64), 0, s, a, src_lim);
  else hipLaunchKernelGGL((k_agg_gather<2>), dim3((uint32_t)g), dim3(64), 0, s, a, src_lim);
}

}  // namespace ws
