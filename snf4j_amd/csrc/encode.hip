// encode.hip — the frame encode pipeline on gfx950 (FrameEncoder, FrameEncoder.java:69-135).
//
//   k_enc_len   thread per frame: session, CLOSE positions (block max).
//   k_enc_scan  one workgroup: exclusive scan of the block aggregates.
//   k_enc_kept  thread per frame: the close latch (:71-76: frames after a CLOSE of
//               the same session, or of an already closed encoder, are dropped),
//               kept wire lengths (FrameEncoder.length, :122-135), block sums.
//   k_enc_scan_sum / k_enc_fix   wire offsets; coarse piece -> frame index.
//   k_enc_kept2 / k_enc_fix2   small batches: each block reduces the aggregates of
//               the blocks before it itself (no separate scan launches).
//   k_enc_desc  thread per 1 KiB piece of wire_out: its frame and descriptor.
//   k_enc_piecesN one wave per 2 KiB of wire_out: header bytes (:80-106) and the
//               payload XOR the injected mask key (:107-117), aligned 16-B stores.
//   k_enc_final thread per session: FrameEncoder.closed carry-out.
#include "wsgpu_internal.h"
#include "wsgpu_scan.h"

namespace ws {

__device__ __forceinline__ uint32_t enc_header_len(uint32_t len, int client) {
  return 2u + (len > 0xffffu ? 8u : (len > 125u ? 2u : 0u)) + (client ? 4u : 0u);
}

__global__ __launch_bounds__(BLOCK) void k_enc_len(EncodeArgs a) {
  const uint64_t k = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  Agg v = AGG_ID;
  if (k < a.n_frames) {
    const wsg_encode_frame f = a.frames[k];
    const uint32_t s = wave_find_session(a.session_first, a.n_sessions, a.n_frames, k);
    a.sess[k] = s;
    v.sum = (uint64_t)enc_header_len(f.payload_len, a.client_mode) + f.payload_len;
    v.m0 = (f.opcode & 15u) == WSG_OP_CLOSE ? (int32_t)k : -1;
  }
  Agg tot;
  block_excl_scan(v, &tot);
  if (threadIdx.x == 0) {
    a.blk_sum[blockIdx.x] = tot.sum;
    a.blk_max[blockIdx.x] = tot.m0;
  }
}

__global__ __launch_bounds__(1024) void k_enc_scan(EncodeArgs a) {
  Agg carry = AGG_ID;
  for (uint32_t base = 0; base < a.nblk; base += 1024) {
    const uint32_t b = base + threadIdx.x;
    Agg v = AGG_ID;
    if (b < a.nblk) {
      v.sum = a.blk_sum[b];
      v.m0 = a.blk_max[b];
    }
    Agg tot;
    Agg ex = agg_op(carry, block_excl_scan(v, &tot));
    if (b < a.nblk) {
      a.blk_sum[b] = ex.sum;
      a.blk_max[b] = ex.m0;
    }
    carry = agg_op(carry, tot);
  }
}

// Kept lengths with the latch applied (a dropped frame has length 0, so the
// prefix sum is taken over kept lengths): the last CLOSE before k from the block
// scan + the scanned block prefix, then a block-local sum (reuses blk_sum).
__global__ __launch_bounds__(BLOCK) void k_enc_kept(EncodeArgs a) {
  const uint64_t k = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  const bool live = k < a.n_frames;
  wsg_encode_frame f;
  Agg v = AGG_ID;
  if (live) {
    f = a.frames[k];
    v.m0 = (f.opcode & 15u) == WSG_OP_CLOSE ? (int32_t)k : -1;
  }
  Agg tot;
  const Agg ex = block_excl_scan(v, &tot);
  Agg w = AGG_ID;
  if (live) {
    const int32_t bp = a.blk_max[blockIdx.x];
    const int32_t lc = ex.m0 > bp ? ex.m0 : bp;
    a.last_close[k] = lc;
    const uint32_t s = a.sess[k];
    const bool dropped = a.closed[s] || lc >= (int32_t)a.session_first[s];
    w.sum = dropped ? 0ull : (uint64_t)enc_header_len(f.payload_len, a.client_mode) + f.payload_len;
  }
  const Agg ew = block_excl_scan(w, &tot);
  if (live) a.wire_off[k] = ew.sum;  // block-local, fixed up by k_enc_fix
  if (threadIdx.x == 0) a.blk_sum[blockIdx.x] = tot.sum;
}

__global__ __launch_bounds__(1024) void k_enc_scan_sum(EncodeArgs a) {
  Agg carry = AGG_ID;
  for (uint32_t base = 0; base < a.nblk; base += 1024) {
    const uint32_t b = base + threadIdx.x;
    Agg v = AGG_ID;
    if (b < a.nblk) v.sum = a.blk_sum[b];
    Agg tot;
    Agg ex = agg_op(carry, block_excl_scan(v, &tot));
    if (b < a.nblk) a.blk_sum[b] = ex.sum;
    carry = agg_op(carry, tot);
  }
  if (threadIdx.x == 0) a.wire_off[a.n_frames] = carry.sum;
}

// Coarse piece index for k_enc_desc: pidx[q] = the frame holding wire byte q * IDX_SPAN
// (the frame whose extent [wire_off[k], wire_off[k+1]) contains it; dropped frames
// have an empty extent and hold nothing).
constexpr uint64_t IDX_SPAN = 64ull * PIECE;

__device__ __forceinline__ void enc_index_frame(const EncodeArgs& a, uint64_t k, uint64_t wo, uint64_t end) {
  for (uint64_t q = (wo + IDX_SPAN - 1) / IDX_SPAN; q * IDX_SPAN < end && q < a.n_idx; ++q) a.pidx[q] = (uint32_t)k;
}

// Final wire offsets (block-local prefix + block base) and the coarse index.
__global__ __launch_bounds__(BLOCK) void k_enc_fix(EncodeArgs a) {
  const uint64_t k = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (k >= a.n_frames) return;
  const uint64_t wo = a.wire_off[k] + a.blk_sum[blockIdx.x];
  a.wire_off[k] = wo;
  const uint32_t s = a.sess[k];
  if (a.closed[s] || a.last_close[k] >= (int32_t)a.session_first[s]) return;  // dropped
  const uint32_t len = a.frames[k].payload_len;
  enc_index_frame(a, k, wo, wo + enc_header_len(len, a.client_mode) + len);
}

// Small batches (<= ENC_SMALL_BLOCKS blocks of frames): the scans of the block
// aggregates are not separate launches — every block reduces the aggregates of
// the blocks before it itself (<= 256 loads, one per thread) — so the plan is
// three launches (k_enc_len, k_enc_kept2, k_enc_fix2) instead of six.
constexpr uint32_t ENC_SMALL_BLOCKS = 256;
constexpr uint32_t SESS_DROPPED = 0x80000000u;  // sess[k] bit 31: frame dropped by the latch (small path)

__device__ __forceinline__ Agg prefix_of_blocks(const EncodeArgs& a, bool want_sum) {
  Agg p = AGG_ID, tot;
  if (threadIdx.x < blockIdx.x) {
    if (want_sum) p.sum = a.blk_sum[threadIdx.x];
    else p.m0 = a.blk_max[threadIdx.x];
  }
  block_excl_scan(p, &tot);
  return tot;
}

__global__ __launch_bounds__(BLOCK) void k_enc_kept2(EncodeArgs a) {
  const int32_t bp = prefix_of_blocks(a, false).m0;  // last CLOSE before this block
  const uint64_t k = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  const bool live = k < a.n_frames;
  wsg_encode_frame f;
  Agg v = AGG_ID;
  if (live) {
    f = a.frames[k];
    v.m0 = (f.opcode & 15u) == WSG_OP_CLOSE ? (int32_t)k : -1;
  }
  Agg tot;
  const Agg ex = block_excl_scan(v, &tot);
  Agg w = AGG_ID;
  if (live) {
    const int32_t lc = ex.m0 > bp ? ex.m0 : bp;
    a.last_close[k] = lc;
    const uint32_t s = a.sess[k];
    const bool dropped = a.closed[s] || lc >= (int32_t)a.session_first[s];  // FrameEncoder.java:71-76
    if (dropped) a.sess[k] = s | SESS_DROPPED;
    w.sum = dropped ? 0ull : (uint64_t)enc_header_len(f.payload_len, a.client_mode) + f.payload_len;
  }
  const Agg ew = block_excl_scan(w, &tot);
  if (live) a.wire_off[k] = ew.sum;  // block-local
  if (threadIdx.x == 0) a.blk_sum[blockIdx.x] = tot.sum;
}

// Final offsets, coarse index, and the closed carry-out (by the last frame of
// each session: it sent or follows a CLOSE); closed[] is not read here.
__global__ __launch_bounds__(BLOCK) void k_enc_fix2(EncodeArgs a) {
  const uint64_t base = prefix_of_blocks(a, true).sum;
  const uint64_t k = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (blockIdx.x + 1 == gridDim.x && threadIdx.x == 0) a.wire_off[a.n_frames] = base + a.blk_sum[blockIdx.x];
  if (k >= a.n_frames) return;
  const uint64_t wo = a.wire_off[k] + base;
  a.wire_off[k] = wo;
  const uint32_t sk = a.sess[k], s = sk & ~SESS_DROPPED;
  const wsg_encode_frame f = a.frames[k];
  if (!(sk & SESS_DROPPED)) enc_index_frame(a, k, wo, wo + enc_header_len(f.payload_len, a.client_mode) + f.payload_len);
  const bool last = k + 1 == a.n_frames || (a.sess[k + 1] & ~SESS_DROPPED) != s;
  if (last && ((f.opcode & 15u) == WSG_OP_CLOSE || a.last_close[k] >= (int32_t)a.session_first[s])) a.closed[s] = 1;
}

// One thread per 1 KiB piece of wire_out: the frame holding the piece's first
// byte is the last k with wire_off[k] <= ps, searched between the coarse index
// entries around ps (usually one or two frames apart; the offsets stay in L2).
// A piece entirely inside that frame's payload (or ending the output there)
// takes the fast path of k_enc_piecesN.
__global__ __launch_bounds__(256) void k_enc_desc(EncodeArgs a) {
  const uint64_t pc = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (pc >= a.n_pieces) return;
  const uint64_t total = a.wire_off[a.n_frames];
  const uint64_t ps = pc * PIECE;
  if (ps >= total) return;
  const uint64_t q = ps / IDX_SPAN;
  uint64_t lo = a.pidx[q];                                                   // wire_off[lo] <= q * SPAN <= ps
  uint64_t hi = (q + 1) * IDX_SPAN < total ? (uint64_t)a.pidx[q + 1] + 1 : a.n_frames;  // ps < wire_off[hi]
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a.wire_off[mid] <= ps) lo = mid;
    else hi = mid;
  }
  const uint64_t k = lo;
  const wsg_encode_frame f = a.frames[k];
  const uint32_t hl = enc_header_len(f.payload_len, a.client_mode);
  const uint64_t wo = a.wire_off[k], pay0 = wo + hl, end = wo + hl + f.payload_len;
  const bool single = ps >= pay0 && (ps + PIECE <= end || end == total);
  PieceDesc d;
  d.frame = (uint32_t)k;
  if (single) {
    const uint32_t m = (uint32_t)f.mask[0] | ((uint32_t)f.mask[1] << 8) | ((uint32_t)f.mask[2] << 16) |
                       ((uint32_t)f.mask[3] << 24);
    const uint64_t j0 = ps - pay0;  // payload index of the piece's first byte
    const uint32_t ph = (uint32_t)(j0 & 3);
    const uint32_t mr = a.client_mode ? (ph ? (m >> (8 * ph)) | (m << (32 - 8 * ph)) : m) : 0u;
    const uint64_t nb = end - ps < PIECE ? end - ps : PIECE;
    d.info = ((f.payload_off + j0) & PD_SRC_MASK) | (nb << PD_NB_SHIFT);
    d.mask = mr;
  } else {
    d.info = PD_MULTI;
    d.mask = 0;
  }
  a.pieces[pc] = d;
}

// ------------------------------------------------------------------ k_enc_pieces
// One wave per 1 KiB of wire_out, lane i owning bytes [1024p + 16i, +16): the
// decode kernel's shape (decode.hip k_pieces) with source and sink swapped.
__device__ __forceinline__ uint32_t enc_dpp_from_next(uint32_t v, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x130, 0xf, 0xf, false);
}

// header byte r (< hl) of frame f (FrameEncoder.java:80-106)
__device__ __forceinline__ uint8_t enc_header_byte(const wsg_encode_frame& f, uint32_t r, int client) {
  const uint32_t len = f.payload_len;
  if (r == 0) return (uint8_t)((((f.flags >> 4) & 7u) << 4) | (f.flags & 0x80u) | (f.opcode & 15u));
  const uint8_t mb = client ? 0x80 : 0;
  uint32_t lb;  // bytes of extended length
  if (len > 0xffffu) {
    if (r == 1) return mb | 127;
    lb = 8;
  } else if (len > 125u) {
    if (r == 1) return mb | 126;
    lb = 2;
  } else {
    if (r == 1) return mb | (uint8_t)len;
    lb = 0;
  }
  if (r < 2 + lb) return (uint8_t)((uint64_t)len >> (8 * (lb - 1 - (r - 2))));
  const uint32_t m = (uint32_t)f.mask[0] | ((uint32_t)f.mask[1] << 8) | ((uint32_t)f.mask[2] << 16) |
                     ((uint32_t)f.mask[3] << 24);
  return (uint8_t)(m >> (8 * (r - 2 - lb)));  // client mode only
}

// One piece (fast single-frame path or the general path with headers/seams).
__device__ __forceinline__ void enc_piece(const EncodeArgs& a, const PieceDesc d, uint64_t p, uint64_t lim,
                                          int lane) {
  const uint64_t ps = p * PIECE;
  const uint32_t boff = (uint32_t)lane * 16u;
  const uint64_t o = ps + boff;
  uint32_t w[4];
  if (!(d.info & PD_MULTI)) {
    // ---- fast path: the piece is payload of one frame
    const uint64_t s = d.info & PD_SRC_MASK;
    const uint32_t nb = (uint32_t)(d.info >> PD_NB_SHIFT) & 2047u;
    const uint64_t a16 = s & ~15ull;
    const uint32_t sh = (uint32_t)(s & 15u), b = sh & 3u;
    u32x4 A;
    uint32_t e0, e1, e2, e3;
    if (a16 + PIECE + 16u <= a.payload_len) {
      const __amdgpu_buffer_rsrc_t rin =
          __builtin_amdgcn_make_buffer_rsrc((void*)(a.payload + a16), 0, (int)(PIECE + 16u), 0x00020000);
      A = __builtin_amdgcn_raw_buffer_load_b128(rin, boff, 0, 2);
      const u32x4 nx = *(const u32x4*)(a.payload + a16 + PIECE);
      e0 = nx.x; e1 = nx.y; e2 = nx.z; e3 = nx.w;
    } else {  // the payload buffer's last KiB: byte loads
      uint32_t dd[4] = {0u, 0u, 0u, 0u}, ee[4] = {0u, 0u, 0u, 0u};
      for (uint32_t i = 0; i < 16u; ++i) {
        if (a16 + boff + i < a.payload_len) dd[i >> 2] |= (uint32_t)a.payload[a16 + boff + i] << (8 * (i & 3));
        if (a16 + PIECE + i < a.payload_len) ee[i >> 2] |= (uint32_t)a.payload[a16 + PIECE + i] << (8 * (i & 3));
      }
      A = (u32x4){dd[0], dd[1], dd[2], dd[3]};
      e0 = ee[0]; e1 = ee[1]; e2 = ee[2]; e3 = ee[3];
    }
    const uint32_t W0 = A.x, W1 = A.y, W2 = A.z, W3 = A.w;
    const uint32_t W4 = enc_dpp_from_next(A.x, e0), W5 = enc_dpp_from_next(A.y, e1);
    const uint32_t W6 = enc_dpp_from_next(A.z, e2), W7 = enc_dpp_from_next(A.w, e3);
    switch (sh >> 2) {  // wave-uniform
      case 0: w[0] = alignbyte(W1, W0, b); w[1] = alignbyte(W2, W1, b); w[2] = alignbyte(W3, W2, b); w[3] = alignbyte(W4, W3, b); break;
      case 1: w[0] = alignbyte(W2, W1, b); w[1] = alignbyte(W3, W2, b); w[2] = alignbyte(W4, W3, b); w[3] = alignbyte(W5, W4, b); break;
      case 2: w[0] = alignbyte(W3, W2, b); w[1] = alignbyte(W4, W3, b); w[2] = alignbyte(W5, W4, b); w[3] = alignbyte(W6, W5, b); break;
      default: w[0] = alignbyte(W4, W3, b); w[1] = alignbyte(W5, W4, b); w[2] = alignbyte(W6, W5, b); w[3] = alignbyte(W7, W6, b); break;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] ^= d.mask;
    if (boff >= nb) return;
  } else {
    // ---- general path: headers and frame seams inside the piece
    if (o >= lim) return;
    uint32_t k = d.frame;
    uint64_t fe = a.wire_off[k + 1];
    while (o >= fe) fe = a.wire_off[++k + 1];
    wsg_encode_frame f = a.frames[k];
    uint64_t fo = a.wire_off[k];
    uint32_t hl = enc_header_len(f.payload_len, a.client_mode);
    uint32_t m = a.client_mode ? ((uint32_t)f.mask[0] | ((uint32_t)f.mask[1] << 8) | ((uint32_t)f.mask[2] << 16) |
                                  ((uint32_t)f.mask[3] << 24))
                               : 0u;
    if (o >= fo + hl && o + 16 <= fe) {  // the lane's 16 bytes are payload of one frame
      const uint64_t j0 = o - fo - hl;
      const uint64_t src = f.payload_off + j0;
      const uint64_t a4 = src & ~3ull;
      const uint32_t sh = (uint32_t)(src & 3u);
      uint32_t dd[5] = {0u, 0u, 0u, 0u, 0u};
      if (a4 + 20u <= a.payload_len) {
        const uint32_t* q = (const uint32_t*)(a.payload + a4);
        dd[0] = q[0]; dd[1] = q[1]; dd[2] = q[2]; dd[3] = q[3]; dd[4] = q[4];
      } else {
#pragma unroll
        for (uint32_t i = 0; i < 20u; ++i)  // constant indices: dd stays in registers
          if (a4 + i < a.payload_len) dd[i >> 2] |= (uint32_t)a.payload[a4 + i] << (8 * (i & 3));
      }
      const uint32_t ph = (uint32_t)(j0 & 3);
      const uint32_t mr = ph ? (m >> (8 * ph)) | (m << (32 - 8 * ph)) : m;
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = alignbyte(dd[i + 1], dd[i], sh) ^ mr;
    } else {
      uint64_t blo = 0, bhi = 0;  // the 16 bytes (no dynamically indexed array: registers only)
      for (uint32_t i = 0; i < 16u; ++i) {
        const uint64_t x = o + i;
        if (x >= lim) break;
        while (x >= fe) {  // next frame (dropped frames have an empty extent)
          ++k;
          fo = fe;
          fe = a.wire_off[k + 1];
          if (x < fe) {
            f = a.frames[k];
            hl = enc_header_len(f.payload_len, a.client_mode);
            m = a.client_mode ? ((uint32_t)f.mask[0] | ((uint32_t)f.mask[1] << 8) | ((uint32_t)f.mask[2] << 16) |
                                 ((uint32_t)f.mask[3] << 24))
                              : 0u;
          }
        }
        const uint64_t r = x - fo;
        uint32_t byte;
        if (r < hl) {
          byte = enc_header_byte(f, (uint32_t)r, a.client_mode);
        } else {
          const uint64_t j = r - hl;
          byte = a.payload[f.payload_off + j] ^ ((m >> (8 * (j & 3))) & 0xffu);
        }
        if (i < 8) blo |= (uint64_t)byte << (8 * i);
        else bhi |= (uint64_t)byte << (8 * (i - 8));
      }
      w[0] = (uint32_t)blo; w[1] = (uint32_t)(blo >> 32); w[2] = (uint32_t)bhi; w[3] = (uint32_t)(bhi >> 32);
    }
  }
  if (o + 16 <= lim) {
    __builtin_nontemporal_store((u32x4){w[0], w[1], w[2], w[3]}, (u32x4*)(a.wire_out + o));
  } else {  // the output's last bytes: wire_out is not padded
#pragma unroll
    for (uint32_t i = 0; i < 16u; ++i)
      if (o + i < lim) a.wire_out[o + i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
  }
}

// N consecutive pieces of one frame's payload per wave: all loads issued before
// any store (N KiB in flight per wave); lane 63's next block of piece i is lane
// 0's block of piece i+1.  The mask phase is the same for every piece (1024 = 0 mod 4).
template <int N>
__device__ __forceinline__ void enc_fastN(const EncodeArgs& a, const PieceDesc d, uint32_t nb_last, uint64_t ps,
                                          uint64_t lim, int lane) {
  const uint64_t s = d.info & PD_SRC_MASK;
  const uint64_t a16 = s & ~15ull;
  const uint32_t sh = (uint32_t)(s & 15u), b = sh & 3u;
  const uint32_t boff = (uint32_t)lane * 16u;
  u32x4 A[N], nx;
  if (a16 + N * PIECE + 16u <= a.payload_len) {
    const __amdgpu_buffer_rsrc_t rin =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.payload + a16), 0, (int)(N * PIECE + 16u), 0x00020000);
#pragma unroll
    for (int i = 0; i < N; ++i) A[i] = __builtin_amdgcn_raw_buffer_load_b128(rin, boff + i * PIECE, 0, 2);
    nx = *(const u32x4*)(a.payload + a16 + N * PIECE);
  } else {
#pragma unroll
    for (int i = 0; i <= N; ++i) {
      uint32_t dd[4] = {0u, 0u, 0u, 0u};
      const uint64_t base = a16 + (uint64_t)i * PIECE + (i < N ? boff : 0u);
      for (uint32_t k = 0; k < 16u; ++k)
        if (base + k < a.payload_len) dd[k >> 2] |= (uint32_t)a.payload[base + k] << (8 * (k & 3));
      if (i < N) A[i] = (u32x4){dd[0], dd[1], dd[2], dd[3]};
      else nx = (u32x4){dd[0], dd[1], dd[2], dd[3]};
    }
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    u32x4 n;
    if (i + 1 < N) {
      n.x = (uint32_t)__builtin_amdgcn_readlane((int)A[i + 1].x, 0);
      n.y = (uint32_t)__builtin_amdgcn_readlane((int)A[i + 1].y, 0);
      n.z = (uint32_t)__builtin_amdgcn_readlane((int)A[i + 1].z, 0);
      n.w = (uint32_t)__builtin_amdgcn_readlane((int)A[i + 1].w, 0);
    } else {
      n = nx;
    }
    const uint32_t W0 = A[i].x, W1 = A[i].y, W2 = A[i].z, W3 = A[i].w;
    const uint32_t W4 = enc_dpp_from_next(A[i].x, n.x), W5 = enc_dpp_from_next(A[i].y, n.y);
    const uint32_t W6 = enc_dpp_from_next(A[i].z, n.z), W7 = enc_dpp_from_next(A[i].w, n.w);
    uint32_t w[4];
    switch (sh >> 2) {
      case 0: w[0] = alignbyte(W1, W0, b); w[1] = alignbyte(W2, W1, b); w[2] = alignbyte(W3, W2, b); w[3] = alignbyte(W4, W3, b); break;
      case 1: w[0] = alignbyte(W2, W1, b); w[1] = alignbyte(W3, W2, b); w[2] = alignbyte(W4, W3, b); w[3] = alignbyte(W5, W4, b); break;
      case 2: w[0] = alignbyte(W3, W2, b); w[1] = alignbyte(W4, W3, b); w[2] = alignbyte(W5, W4, b); w[3] = alignbyte(W6, W5, b); break;
      default: w[0] = alignbyte(W4, W3, b); w[1] = alignbyte(W5, W4, b); w[2] = alignbyte(W6, W5, b); w[3] = alignbyte(W7, W6, b); break;
    }
    const uint64_t o = ps + (uint64_t)i * PIECE + boff;
    if (i + 1 == N && boff >= nb_last) continue;
    const u32x4 v = (u32x4){w[0] ^ d.mask, w[1] ^ d.mask, w[2] ^ d.mask, w[3] ^ d.mask};
    if (o + 16 <= lim) {
      __builtin_nontemporal_store(v, (u32x4*)(a.wire_out + o));
    } else {  // the output's last bytes: wire_out is not padded
      const uint64_t vlo = ((uint64_t)v.y << 32) | v.x, vhi = ((uint64_t)v.w << 32) | v.z;
#pragma unroll
      for (uint32_t k = 0; k < 16u; ++k)
        if (o + k < lim) a.wire_out[o + k] = (uint8_t)((k < 8 ? vlo : vhi) >> (8 * (k & 7)));
    }
  }
}

template <int N>
__global__ __launch_bounds__(64) void k_enc_piecesN(EncodeArgs a) {
  const int lane = threadIdx.x;
  const uint64_t p = (uint64_t)N * (uint64_t)__builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x));
  PieceDesc d[N];
#pragma unroll
  for (int i = 0; i < N; ++i) d[i] = a.pieces[p + i];
  const uint64_t total = a.wire_off[a.n_frames];
  asm volatile("" ::"s"(d[0].info), "s"(d[0].mask), "s"(d[0].frame), "s"(d[N - 1].info), "s"(d[N - 1].frame),
               "s"(total));
  const uint64_t ps = p * PIECE;
  const uint64_t lim = total < a.wire_cap ? total : a.wire_cap;
  if (ps >= lim) return;
  bool fast = ps + (uint64_t)(N - 1) * PIECE < lim && d[0].frame == d[N - 1].frame;
#pragma unroll
  for (int i = 0; i < N; ++i) fast = fast && !(d[i].info & PD_MULTI);
  if (fast) {
    enc_fastN<N>(a, d[0], (uint32_t)(d[N - 1].info >> PD_NB_SHIFT) & 2047u, ps, lim, lane);
    return;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (ps + (uint64_t)i * PIECE >= lim) return;
    enc_piece(a, d[i], p + i, lim, lane);
  }
}

void launch_enc_pieces(const EncodeArgs& a, hipStream_t s) {
  if (a.n_pieces)
    hipLaunchKernelGGL(k_enc_piecesN<ENC_PIECES_PER_WAVE>,
                       dim3((uint32_t)((a.n_pieces + ENC_PIECES_PER_WAVE - 1) / ENC_PIECES_PER_WAVE)), dim3(64), 0,
                       s, a);
}

__global__ __launch_bounds__(256) void k_enc_final(EncodeArgs a) {
  const uint32_t s = blockIdx.x * 256u + threadIdx.x;
  if (s >= a.n_sessions) return;
  const uint32_t sf = a.session_first[s], se = a.session_first[s + 1];
  if (se > sf) {
    const uint64_t last = se - 1;
    const bool close_here = (a.frames[last].opcode & 15u) == WSG_OP_CLOSE || a.last_close[last] >= (int32_t)sf;
    if (close_here) a.closed[s] = 1;
  }
}

bool enc_plan_small(const EncodeArgs& a) { return a.nblk <= ENC_SMALL_BLOCKS; }

void launch_enc_len(const EncodeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_enc_len, dim3(a.nblk), dim3(BLOCK), 0, s, a);
}
void launch_enc_scan(const EncodeArgs& a, hipStream_t s) {
  if (enc_plan_small(a)) {
    hipLaunchKernelGGL(k_enc_kept2, dim3(a.nblk), dim3(BLOCK), 0, s, a);
    hipLaunchKernelGGL(k_enc_fix2, dim3(a.nblk), dim3(BLOCK), 0, s, a);
    return;
  }
  hipLaunchKernelGGL(k_enc_scan, dim3(1), dim3(1024), 0, s, a);
  hipLaunchKernelGGL(k_enc_kept, dim3(a.nblk), dim3(BLOCK), 0, s, a);
  hipLaunchKernelGGL(k_enc_scan_sum, dim3(1), dim3(1024), 0, s, a);
  hipLaunchKernelGGL(k_enc_fix, dim3(a.nblk), dim3(BLOCK), 0, s, a);
}
void launch_enc_desc(const EncodeArgs& a, hipStream_t s) {
  if (a.n_pieces) hipLaunchKernelGGL(k_enc_desc, dim3((uint32_t)((a.n_pieces + 255) / 256)), dim3(256), 0, s, a);
}
void launch_enc_final(const EncodeArgs& a, hipStream_t s) {
  if (enc_plan_small(a)) return;  // k_enc_fix2 wrote the carry-out
  hipLaunchKernelGGL(k_enc_final, dim3((a.n_sessions + 255) / 256), dim3(256), 0, s, a);
}

}  // namespace ws
