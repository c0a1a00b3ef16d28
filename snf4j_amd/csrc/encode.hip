// encode.hip — the frame encode pipeline on gfx950 (FrameEncoder, FrameEncoder.java:69-135).
//
//   k_enc_len   thread per frame: wire length (FrameEncoder.length, :122-135),
//               the close latch (:71-76: frames after a CLOSE of the same session,
//               or of an already closed encoder, are dropped); block aggregates.
//   k_enc_scan  one workgroup: exclusive scan of the block aggregates.
//   k_enc_link  thread per frame: wire offset of each frame (prefix sum).
//   k_enc_emit  one wave per frame: header bytes (:80-106) and the payload XOR
//               the injected mask key (:107-117), written with aligned 16-B
//               stores over the frame's interior and byte stores at its seams.
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
    const uint32_t s = find_session(a.session_first, a.n_sessions, k);
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

// Frame lengths are recomputed here with the latch applied: a dropped frame has
// length 0, so the prefix sum is taken over "kept" lengths.  The first scan
// (k_enc_len) only located CLOSE frames; kept lengths need the latch first.
__global__ __launch_bounds__(BLOCK) void k_enc_link(EncodeArgs a) {
  const uint64_t k = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  const bool live = k < a.n_frames;
  Agg v = AGG_ID;
  int32_t lc = -1;
  if (live) {
    v.m0 = (a.frames[k].opcode & 15u) == WSG_OP_CLOSE ? (int32_t)k : -1;
  }
  Agg tot;
  Agg ex = block_excl_scan(v, &tot);
  if (live) {
    const int32_t bp = a.blk_max[blockIdx.x];
    lc = ex.m0 > bp ? ex.m0 : bp;
    a.last_close[k] = lc;
  }
}

// Second length pass: kept lengths with the latch, block sums (reuses blk_sum).
__global__ __launch_bounds__(BLOCK) void k_enc_kept(EncodeArgs a) {
  const uint64_t k = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  Agg v = AGG_ID;
  if (k < a.n_frames) {
    const uint32_t s = a.sess[k];
    const bool dropped = a.closed[s] || a.last_close[k] >= (int32_t)a.session_first[s];
    const uint32_t len = a.frames[k].payload_len;
    v.sum = dropped ? 0ull : (uint64_t)enc_header_len(len, a.client_mode) + len;
  }
  Agg tot;
  Agg ex = block_excl_scan(v, &tot);
  if (k < a.n_frames) a.wire_off[k] = ex.sum;  // block-local, fixed up below
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

__global__ __launch_bounds__(BLOCK) void k_enc_fix(EncodeArgs a) {
  const uint64_t k = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (k < a.n_frames) a.wire_off[k] += a.blk_sum[blockIdx.x];
}

__global__ __launch_bounds__(256) void k_enc_emit(EncodeArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave0 = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 4u;
  for (uint64_t k = wave0; k < a.n_frames; k += nw) {
    const uint64_t wo = a.wire_off[k], we = a.wire_off[k + 1];
    if (we == wo) continue;  // dropped by the close latch
    const wsg_encode_frame f = a.frames[k];
    const uint32_t len = f.payload_len;
    const uint32_t hl = enc_header_len(len, a.client_mode);
    // header bytes (FrameEncoder.java:80-106)
    uint8_t hb[14];
    hb[0] = (uint8_t)(((f.flags >> 4) & 7u) << 4 | (f.flags & 0x80u) | (f.opcode & 15u));
    const uint8_t mb = a.client_mode ? 0x80 : 0;
    uint32_t p = 1;
    if (len > 0xffffu) {
      hb[p++] = mb | 127;
      for (int i = 7; i >= 0; --i) hb[p++] = (uint8_t)((uint64_t)len >> (8 * i));
    } else if (len > 125u) {
      hb[p++] = mb | 126;
      hb[p++] = (uint8_t)(len >> 8);
      hb[p++] = (uint8_t)len;
    } else {
      hb[p++] = mb | (uint8_t)len;
    }
    uint32_t m = 0;
    if (a.client_mode) {
      for (int i = 0; i < 4; ++i) hb[p++] = f.mask[i];
      m = (uint32_t)f.mask[0] | ((uint32_t)f.mask[1] << 8) | ((uint32_t)f.mask[2] << 16) | ((uint32_t)f.mask[3] << 24);
    }
    // output chunks: aligned 16-B blocks covering [wo, we)
    const uint64_t A0 = wo & ~15ull;
    const uint64_t nchunk = ((we + 15) & ~15ull) - A0 >> 4;
    const uint64_t ps = f.payload_off;  // payload byte j lives at payload[ps + j]
    const uint64_t pa4 = ps & ~3ull;
    const uint64_t pavail = a.payload_len - pa4;
    const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.payload + pa4), 0, (int)(pavail > 0x7fffffffull ? 0x7fffffffull : pavail), 0x00020000);
    const uint64_t pay0 = wo + hl;  // wire offset of payload byte 0
    for (uint64_t c = lane; c < nchunk; c += 64) {
      const uint64_t A = A0 + c * 16;
      if (A >= pay0 && A + 16 <= we) {
        // interior: payload bytes j0..j0+15, unaligned source, rotated mask
        const uint64_t j0 = A - pay0;
        const uint64_t rel = (ps & 3) + j0;
        const uint32_t sh = (uint32_t)(rel & 3);
        const uint32_t off = (uint32_t)(rel & ~3ull);
        u32x4 q;
        uint32_t t;
        if ((uint64_t)off + 20u <= pavail) {
          q = __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, 0);
          t = __builtin_amdgcn_raw_buffer_load_b32(rin, off + 16, 0, 0);
        } else {  // the last bytes of the payload buffer: byte loads
          uint32_t d[5] = {0u, 0u, 0u, 0u, 0u};
          for (uint32_t i = 0; i < 20u && (uint64_t)off + i < pavail; ++i)
            d[i >> 2] |= (uint32_t)a.payload[pa4 + off + i] << (8 * (i & 3));
          q = (u32x4){d[0], d[1], d[2], d[3]};
          t = d[4];
        }
        const uint32_t ph = (uint32_t)(j0 & 3);
        const uint32_t mr = ph ? ((m >> (8 * ph)) | (m << (32 - 8 * ph))) : m;
        u32x4 o;
        o.x = alignbyte(q.y, q.x, sh) ^ mr;
        o.y = alignbyte(q.z, q.y, sh) ^ mr;
        o.z = alignbyte(q.w, q.z, sh) ^ mr;
        o.w = alignbyte(t, q.w, sh) ^ mr;
        *(u32x4*)(a.wire_out + A) = o;
      } else {
        // seam chunk: header bytes and/or shared with a neighbouring frame
        for (uint32_t i = 0; i < 16; ++i) {
          const uint64_t x = A + i;
          if (x < wo || x >= we) continue;
          const uint64_t r = x - wo;
          uint8_t b;
          if (r < hl) {
            b = hb[r];
          } else {
            const uint64_t j = r - hl;
            b = a.payload[ps + j] ^ (uint8_t)(m >> (8 * (j & 3)));
          }
          a.wire_out[x] = b;
        }
      }
    }
  }
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

void launch_enc_len(const EncodeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_enc_len, dim3(a.nblk), dim3(BLOCK), 0, s, a);
}
void launch_enc_scan(const EncodeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_enc_scan, dim3(1), dim3(1024), 0, s, a);
  hipLaunchKernelGGL(k_enc_link, dim3(a.nblk), dim3(BLOCK), 0, s, a);
  hipLaunchKernelGGL(k_enc_kept, dim3(a.nblk), dim3(BLOCK), 0, s, a);
  hipLaunchKernelGGL(k_enc_scan_sum, dim3(1), dim3(1024), 0, s, a);
  hipLaunchKernelGGL(k_enc_fix, dim3(a.nblk), dim3(BLOCK), 0, s, a);
}
void launch_enc_emit(const EncodeArgs& a, hipStream_t s, uint32_t grid) {
  hipLaunchKernelGGL(k_enc_emit, dim3(grid), dim3(256), 0, s, a);
}
void launch_enc_final(const EncodeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_enc_final, dim3((a.n_sessions + 255) / 256), dim3(256), 0, s, a);
}

}  // namespace ws
