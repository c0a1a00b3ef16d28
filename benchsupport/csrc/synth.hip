// synth.hip — libwsbench.so: synthetic frame batches generated in HBM and the
// streaming-copy ceiling (bench.py / GPU tests only; include/wsbench.h).  Not part
// of the codec library.  Byte-identical to the oracle's or_synth_uniform
// (oracle/ws_oracle.c), so a sample copied back can be checked on the host.
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "../../include/wsbench.h"

namespace wsb {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// 16 bytes of valid UTF-8 whose code points never straddle the chunk.
__device__ void synth_text16(uint64_t h, uint8_t out[16]) {
  int i = 0, draws = 0;
  uint64_t r = h;
  while (i < 16) {
    if (draws == 8) { r = splitmix64(r); draws = 0; }
    const unsigned v = (unsigned)(r & 0xff);
    r >>= 8;
    ++draws;
    const int room = 16 - i;
    const unsigned kind = v % 10;
    if (kind <= 6 || room < 2) {
      out[i++] = (uint8_t)(0x20 + (v % 95));
    } else if (kind == 7 || room < 3) {
      const unsigned cp = 0x80 + (v * 7u) % (0x800 - 0x80);
      out[i++] = (uint8_t)(0xC0 | (cp >> 6));
      out[i++] = (uint8_t)(0x80 | (cp & 0x3f));
    } else if (kind == 8 || room < 4) {
      unsigned cp = 0x800 + (v * 211u) % (0x10000 - 0x800);
      if (cp >= 0xD800 && cp <= 0xDFFF) cp += 0x800;
      out[i++] = (uint8_t)(0xE0 | (cp >> 12));
      out[i++] = (uint8_t)(0x80 | ((cp >> 6) & 0x3f));
      out[i++] = (uint8_t)(0x80 | (cp & 0x3f));
    } else {
      const unsigned cp = 0x10000 + (v * 4099u) % (0x110000 - 0x10000);
      out[i++] = (uint8_t)(0xF0 | (cp >> 18));
      out[i++] = (uint8_t)(0x80 | ((cp >> 12) & 0x3f));
      out[i++] = (uint8_t)(0x80 | ((cp >> 6) & 0x3f));
      out[i++] = (uint8_t)(0x80 | (cp & 0x3f));
    }
  }
}

__device__ __forceinline__ uint32_t hdr_len(uint32_t len, int masked) {
  return 2u + (len > 0xffffu ? 8u : (len > 125u ? 2u : 0u)) + (masked ? 4u : 0u);
}

__global__ __launch_bounds__(256) void k_synth_payload(uint64_t seed, uint64_t n_frames, uint32_t payload_len,
                                                       uint32_t fps, int masked, int text, uint8_t* wire) {
  const uint32_t hl = hdr_len(payload_len, masked);
  const uint64_t flen = hl + (uint64_t)payload_len;
  const uint64_t nch = (payload_len + 15u) / 16u;
  const uint64_t total = n_frames * nch;
  for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (uint64_t)gridDim.x * 256) {
    const uint64_t k = t / nch, c = t - k * nch;
    const uint64_t sseed = seed ^ (k / fps);
    const uint64_t fh = splitmix64(sseed ^ (k * 0x9E3779B97F4A7C15ull));
    const uint64_t h = splitmix64(fh + c);
    uint8_t tmp[16];
    if (text) {
      synth_text16(h, tmp);
    } else {
      const uint64_t h2 = splitmix64(h);
      for (int i = 0; i < 8; ++i) { tmp[i] = (uint8_t)(h >> (8 * i)); tmp[8 + i] = (uint8_t)(h2 >> (8 * i)); }
    }
    const uint32_t n = payload_len - c * 16 < 16 ? (uint32_t)(payload_len - c * 16) : 16u;
    if (text && n < 16) {
      uint32_t cut = n;
      while (cut > 0 && (tmp[cut] & 0xC0) == 0x80) --cut;
      for (uint32_t i = cut; i < n; ++i) tmp[i] = 'a';
    }
    uint8_t* pl = wire + k * flen + hl + c * 16;
    for (uint32_t i = 0; i < n; ++i) pl[i] = masked ? (uint8_t)(tmp[i] ^ (uint8_t)(fh >> (8 * (i & 3)))) : tmp[i];
  }
}

__global__ __launch_bounds__(256) void k_synth_header(uint64_t seed, uint64_t n_frames, uint32_t payload_len,
                                                      uint32_t fps, int opcode, int masked, uint8_t* wire,
                                                      uint64_t* frame_off, uint32_t* session_first) {
  const uint32_t hl = hdr_len(payload_len, masked);
  const uint64_t flen = hl + (uint64_t)payload_len;
  const uint64_t n_sessions = (n_frames + fps - 1) / fps;
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k <= n_frames; k += (uint64_t)gridDim.x * 256) {
    frame_off[k] = k * flen;
    if (k <= n_sessions) {
      const uint64_t f = k * fps;
      session_first[k] = (uint32_t)(f < n_frames ? f : n_frames);
    }
    if (k == n_frames) continue;
    const uint64_t fh = splitmix64((seed ^ (k / fps)) ^ (k * 0x9E3779B97F4A7C15ull));
    uint8_t* w = wire + k * flen;
    uint32_t p = 0;
    w[p++] = (uint8_t)(0x80 | (opcode & 0x0f));
    const uint8_t b1 = masked ? 0x80 : 0;
    if (payload_len > 0xffffu) {
      w[p++] = b1 | 127;
      for (int i = 7; i >= 0; --i) w[p++] = (uint8_t)((uint64_t)payload_len >> (8 * i));
    } else if (payload_len > 125u) {
      w[p++] = b1 | 126;
      w[p++] = (uint8_t)(payload_len >> 8);
      w[p++] = (uint8_t)payload_len;
    } else {
      w[p++] = b1 | (uint8_t)payload_len;
    }
    if (masked)
      for (int i = 0; i < 4; ++i) w[p++] = (uint8_t)(fh >> (8 * i));
  }
}

// Table-driven batches (wsb_synth_frames): one workgroup per frame; thread 0
// writes the header, the threads generate the message's 16-B chunks that
// overlap this fragment and store the fragment's bytes (masked).
__device__ __forceinline__ void msg_chunk(const wsb_synth_frame& f, uint64_t c, uint8_t tmp[16]) {
  const uint64_t h = splitmix64(f.msg_seed + c);
  if (f.text) {
    synth_text16(h, tmp);
    const uint32_t n = f.msg_len - c * 16 < 16 ? (uint32_t)(f.msg_len - c * 16) : 16u;
    if (n < 16) {  // message end: never cut a code point
      uint32_t cut = n;
      while (cut > 0 && (tmp[cut] & 0xC0) == 0x80) --cut;
      for (uint32_t i = cut; i < n; ++i) tmp[i] = 'a';
    }
    if (f.inject_pos >= 0) {
      const uint8_t seqs[5][4] = {{0xC0, 0x80}, {0xED, 0xA0, 0x80}, {0xF4, 0x90, 0x80, 0x80}, {0xE2, 0x82, 'a'},
                                  {0xFF}};
      const uint32_t lens[5] = {2, 3, 4, 3, 1};
      const uint32_t kind = f.inject_kind < 5 ? f.inject_kind : 0;
      for (uint32_t i = 0; i < lens[kind]; ++i) {
        const int64_t m = (int64_t)f.inject_pos + i - (int64_t)(c * 16);
        if (m >= 0 && m < 16 && (uint64_t)f.inject_pos + i < f.msg_len) tmp[m] = seqs[kind][i];
      }
    }
  } else {
    const uint64_t h2 = splitmix64(h);
    for (int i = 0; i < 8; ++i) { tmp[i] = (uint8_t)(h >> (8 * i)); tmp[8 + i] = (uint8_t)(h2 >> (8 * i)); }
  }
}

__global__ __launch_bounds__(256) void k_synth_frames(const wsb_synth_frame* __restrict__ t, uint64_t n,
                                                      uint8_t* wire) {
  for (uint64_t k = blockIdx.x; k < n; k += gridDim.x) {
    const wsb_synth_frame f = t[k];
    const int masked = f.flags & 1;
    uint8_t* w = wire + f.wire_off;
    const uint32_t hl = hdr_len(f.payload_len, masked);
    if (threadIdx.x == 0) {
      uint32_t p = 0;
      w[p++] = (uint8_t)((f.flags & 0x80) | (f.opcode & 0x0f));
      const uint8_t b1 = masked ? 0x80 : 0;
      if (f.payload_len > 0xffffu) {
        w[p++] = b1 | 127;
        for (int i = 7; i >= 0; --i) w[p++] = (uint8_t)((uint64_t)f.payload_len >> (8 * i));
      } else if (f.payload_len > 125u) {
        w[p++] = b1 | 126;
        w[p++] = (uint8_t)(f.payload_len >> 8);
        w[p++] = (uint8_t)f.payload_len;
      } else {
        w[p++] = b1 | (uint8_t)f.payload_len;
      }
      if (masked)
        for (int i = 0; i < 4; ++i) w[p++] = (uint8_t)(f.mask >> (8 * i));
    }
    if (!f.payload_len) continue;
    uint8_t* pl = w + hl;
    const uint64_t m0 = f.msg_pos, m1 = (uint64_t)f.msg_pos + f.payload_len;
    for (uint64_t c = m0 / 16 + threadIdx.x; c < (m1 + 15) / 16; c += 256) {
      uint8_t tmp[16];
      msg_chunk(f, c, tmp);
      for (uint32_t i = 0; i < 16; ++i) {
        const uint64_t m = c * 16 + i;
        if (m < m0 || m >= m1) continue;
        const uint64_t j = m - m0;
        pl[j] = masked ? (uint8_t)(tmp[i] ^ (uint8_t)(f.mask >> (8 * (j & 3)))) : tmp[i];
      }
    }
  }
}

void launch_synth_frames(const wsb_synth_frame* t, uint64_t n, uint8_t* wire, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_synth_frames, dim3((uint32_t)(n < 65536 ? n : 65536)), dim3(256), 0, s, t, n, wire);
}

// Streaming copy of `n16` 16-B blocks with the chip's best copy pattern (one
// 64-lane workgroup per KiB, nontemporal): the measured read+write ceiling the
// decode kernel is compared with (bench.py roofline.copy_ceiling_GBs).
typedef unsigned int cu32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(64) void k_copy_ceiling(const cu32x4* __restrict__ s, cu32x4* __restrict__ d,
                                                     uint64_t n16) {
  const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (i < n16) __builtin_nontemporal_store(__builtin_nontemporal_load(&s[i]), &d[i]);
}

void launch_copy_ceiling(const void* src, void* dst, uint64_t bytes, hipStream_t s) {
  const uint64_t n16 = bytes / 16;
  hipLaunchKernelGGL(k_copy_ceiling, dim3((uint32_t)((n16 + 63) / 64)), dim3(64), 0, s, (const cu32x4*)src,
                     (cu32x4*)dst, n16);
}

void launch_synth(uint64_t seed, uint64_t n_frames, uint32_t payload_len, uint32_t fps, int opcode, int masked,
                  int text, uint8_t* wire, uint64_t* frame_off, uint32_t* session_first, hipStream_t s) {
  hipLaunchKernelGGL(k_synth_header, dim3(2048), dim3(256), 0, s, seed, n_frames, payload_len, fps, opcode, masked,
                     wire, frame_off, session_first);
  if (payload_len)
    hipLaunchKernelGGL(k_synth_payload, dim3(8192), dim3(256), 0, s, seed, n_frames, payload_len, fps, masked, text,
                       wire);
}

}  // namespace wsb

// ------------------------------------------------------------------ C ABI (wsbench.h)
extern "C" {

static int ready(int device) { return hipSetDevice(device) == hipSuccess ? 0 : -1; }

int wsb_synth_uniform(int device, void* stream, uint64_t seed, uint64_t n_frames, uint32_t payload_len, uint32_t fps,
                      int opcode, int masked, int text, uint8_t* wire, uint64_t* frame_off, uint32_t* session_first) {
  if (fps == 0 || !wire || !frame_off || !session_first) return -1;
  if (ready(device)) return -2;
  wsb::launch_synth(seed, n_frames, payload_len, fps, opcode, masked, text, wire, frame_off, session_first,
                    (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int wsb_synth_frames(int device, void* stream, const wsb_synth_frame* table, uint64_t n_frames, uint8_t* wire) {
  if (n_frames && (!table || !wire)) return -1;
  if (ready(device)) return -2;
  wsb::launch_synth_frames(table, n_frames, wire, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int wsb_copy_ceiling(int device, void* stream, const void* src, void* dst, uint64_t bytes, int reps, double* gbs) {
  if (!gbs || reps <= 0 || !src || !dst) return -1;
  if (ready(device)) return -2;
  hipStream_t s = (hipStream_t)stream;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -2;
  float best = 1e30f;
  int rc = 0;
  for (int r = 0; r <= reps && !rc; ++r) {
    float ms = 0.f;
    if (hipEventRecord(e0, s) != hipSuccess) rc = -2;
    wsb::launch_copy_ceiling(src, dst, bytes, s);
    if (!rc && (hipEventRecord(e1, s) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                hipEventElapsedTime(&ms, e0, e1) != hipSuccess))
      rc = -2;
    if (!rc && r > 0 && ms < best) best = ms;  // the first run warms up
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (rc) return rc;
  *gbs = 2.0 * (double)(bytes / 16 * 16) / (best * 1e-3) / 1e9;
  return 0;
}

}  // extern "C"
