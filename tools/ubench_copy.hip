// ubench_copy.hip — streaming read+write ceiling of the box for a 4.3 GB
// buffer (the decode working set): copy-kernel variants (unroll depth, cache
// policy, block size, persistent vs one-shot grid), interleaved in one process.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// grid-stride, one 16-B element per iteration
__global__ __launch_bounds__(256) void k_gs(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) d[i] = s[i];
}

// one-shot: block b copies elements [b*T*U, (b+1)*T*U), U loads in flight per thread
template <int T, int U, int NT>
__global__ __launch_bounds__(T) void k_oneshot(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t base = (uint64_t)blockIdx.x * T * U + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t i = base + (uint64_t)u * T;
    if (i < n) v[u] = (NT & 1) ? __builtin_nontemporal_load(&s[i]) : s[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t i = base + (uint64_t)u * T;
    if (i < n) {
      if (NT & 2) __builtin_nontemporal_store(v[u], &d[i]);
      else d[i] = v[u];
    }
  }
}

// wave-per-chunk, mirroring k_unmask's shape: a wave copies a CHUNK-byte chunk,
// U loads per lane in flight, optional nt (aux=2) buffer loads/stores, source
// offset by SRCOFF bytes (dword loads + alignbyte, as for a frame payload at +8/+6)
template <int U, int CHUNK, int NT, int SRCOFF>
__global__ __launch_bounds__(256) void k_wave(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, uint64_t nchunks) {
  const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= nchunks) return;
  const __amdgpu_buffer_rsrc_t rin =
      __builtin_amdgcn_make_buffer_rsrc((void*)(s + w * CHUNK + (SRCOFF & ~3)), 0, CHUNK + 64, 0x00020000);
  const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc((void*)(d + w * CHUNK), 0, CHUNK, 0x00020000);
  for (int c0 = 0; c0 < CHUNK / 16; c0 += 64 * U) {
    u32x4 v[U];
    uint32_t t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, (c0 + u * 64 + lane) * 16, 0, NT ? 2 : 0);
      if (SRCOFF & 3) t[u] = __builtin_amdgcn_raw_buffer_load_b32(rin, (c0 + u * 64 + lane) * 16 + 16, 0, NT ? 2 : 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      u32x4 o = v[u];
      if (SRCOFF & 3) {
        o.x = __builtin_amdgcn_alignbyte(v[u].y, v[u].x, SRCOFF & 3);
        o.y = __builtin_amdgcn_alignbyte(v[u].z, v[u].y, SRCOFF & 3);
        o.z = __builtin_amdgcn_alignbyte(v[u].w, v[u].z, SRCOFF & 3);
        o.w = __builtin_amdgcn_alignbyte(t[u], v[u].w, SRCOFF & 3);
      }
      __builtin_amdgcn_raw_buffer_store_b128(o, rout, (c0 + u * 64 + lane) * 16, 0, NT ? 2 : 0);
    }
  }
}

// a workgroup per CHUNK, each of its 4 waves one quarter (wave i: bytes i*CHUNK/4..)
template <int CHUNK, int NT>
__global__ __launch_bounds__(256) void k_wg(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, uint64_t nchunks) {
  const uint64_t w = blockIdx.x;
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void*)(s + w * CHUNK), 0, CHUNK, 0x00020000);
  const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc((void*)(d + w * CHUNK), 0, CHUNK, 0x00020000);
  for (int c = threadIdx.x; c < CHUNK / 16; c += 256) {
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rin, c * 16, 0, NT ? 2 : 0);
    __builtin_amdgcn_raw_buffer_store_b128(v, rout, c * 16, 0, NT ? 2 : 0);
  }
}

// read-only / write-only ceilings (bytes counted once): U 16-B loads (stores) per
// thread in flight; the read result is kept alive by a never-taken store
template <int T, int U, int NT>
__global__ __launch_bounds__(T) void k_read(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t base = (uint64_t)blockIdx.x * T * U + threadIdx.x;
  u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t i = base + (uint64_t)u * T;
    if (i < n) acc ^= NT ? __builtin_nontemporal_load(&s[i]) : s[i];
  }
  if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u) d[base] = acc;
}
template <int T, int U, int NT>
__global__ __launch_bounds__(T) void k_write(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t base = (uint64_t)blockIdx.x * T * U + threadIdx.x;
  const u32x4 v = {(uint32_t)base, 1u, 2u, 3u};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t i = base + (uint64_t)u * T;
    if (i < n) {
      if (NT) __builtin_nontemporal_store(v, &d[i]);
      else d[i] = v;
    }
  }
}

int main(int argc, char** argv) {
  const uint64_t bytes = argc > 1 ? strtoull(argv[1], 0, 0) : 4303355904ull;
  const uint64_t n = bytes / 16;
  u32x4 *a, *b;
  CK(hipMalloc(&a, n * 16 + 4096));
  CK(hipMalloc(&b, n * 16 + 4096));
  CK(hipMemset(a, 1, n * 16));
  CK(hipMemset(b, 0, n * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V { const char* name; int id; };
  std::vector<V> vs = {{"oneshot T256 U1", 2},        {"oneshot T256 U1 ntLS", 20}, {"oneshot T64 U1 ntLS", 21},
                       {"oneshot T64 U4 ntLS", 22},    {"oneshot T256 U2 ntLS", 23}, {"oneshot T256 U4 ntLS", 7},
                       {"wave U4 4K", 10},             {"wave U4 4K nt", 11},        {"wave U1 4K nt", 12},
                       {"wave U4 4K nt src+8", 13},    {"wave U4 4K nt src+6", 14},  {"wave U1 4K nt src+6", 15},
                       {"wg 4K nt", 16},               {"wg 16K nt", 17},            {"wg 64K nt", 18},
                       {"wave U1 1K nt src+6", 19},
                       {"READ T64 U4 nt", 30},         {"READ T256 U4", 31},         {"READ T64 U1 nt", 32},
                       {"READ T256 U8 nt", 33},        {"WRITE T64 U4 nt", 40},      {"WRITE T256 U4", 41},
                       {"WRITE T64 U1 nt", 42},        {"WRITE T256 U8 nt", 43}};
  std::vector<double> best(vs.size(), 1e30);
  for (int r = 0; r < 6; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipEventRecord(e0, 0));
      switch (vs[i].id) {
        case 2: k_oneshot<256, 1, 0><<<(n + 255) / 256, 256>>>(a, b, n); break;
        case 20: k_oneshot<256, 1, 3><<<(n + 255) / 256, 256>>>(a, b, n); break;
        case 21: k_oneshot<64, 1, 3><<<(n + 63) / 64, 64>>>(a, b, n); break;
        case 22: k_oneshot<64, 4, 3><<<(n + 255) / 256, 64>>>(a, b, n); break;
        case 23: k_oneshot<256, 2, 3><<<(n + 511) / 512, 256>>>(a, b, n); break;
        case 7: k_oneshot<256, 4, 3><<<(n + 1023) / 1024, 256>>>(a, b, n); break;
        case 10: k_wave<4, 4096, 0, 0><<<(n / 256 + 3) / 4, 256>>>((const uint8_t*)a, (uint8_t*)b, n / 256 - 1); break;
        case 11: k_wave<4, 4096, 1, 0><<<(n / 256 + 3) / 4, 256>>>((const uint8_t*)a, (uint8_t*)b, n / 256 - 1); break;
        case 12: k_wave<1, 4096, 1, 0><<<(n / 256 + 3) / 4, 256>>>((const uint8_t*)a, (uint8_t*)b, n / 256 - 1); break;
        case 13: k_wave<4, 4096, 1, 8><<<(n / 256 + 3) / 4, 256>>>((const uint8_t*)a, (uint8_t*)b, n / 256 - 1); break;
        case 14: k_wave<4, 4096, 1, 6><<<(n / 256 + 3) / 4, 256>>>((const uint8_t*)a, (uint8_t*)b, n / 256 - 1); break;
        case 15: k_wave<1, 4096, 1, 6><<<(n / 256 + 3) / 4, 256>>>((const uint8_t*)a, (uint8_t*)b, n / 256 - 1); break;
        case 16: k_wg<4096, 1><<<n / 256, 256>>>((const uint8_t*)a, (uint8_t*)b, n / 256); break;
        case 17: k_wg<16384, 1><<<n / 1024, 256>>>((const uint8_t*)a, (uint8_t*)b, n / 1024); break;
        case 18: k_wg<65536, 1><<<n / 4096, 256>>>((const uint8_t*)a, (uint8_t*)b, n / 4096); break;
        case 19: k_wave<1, 1024, 1, 6><<<(n / 64 + 3) / 4, 256>>>((const uint8_t*)a, (uint8_t*)b, n / 64 - 1); break;
        case 30: k_read<64, 4, 1><<<(n + 255) / 256, 64>>>(a, b, n); break;
        case 31: k_read<256, 4, 0><<<(n + 1023) / 1024, 256>>>(a, b, n); break;
        case 32: k_read<64, 1, 1><<<(n + 63) / 64, 64>>>(a, b, n); break;
        case 33: k_read<256, 8, 1><<<(n + 2047) / 2048, 256>>>(a, b, n); break;
        case 40: k_write<64, 4, 1><<<(n + 255) / 256, 64>>>(a, b, n); break;
        case 41: k_write<256, 4, 0><<<(n + 1023) / 1024, 256>>>(a, b, n); break;
        case 42: k_write<64, 1, 1><<<(n + 63) / 64, 64>>>(a, b, n); break;
        case 43: k_write<256, 8, 1><<<(n + 2047) / 2048, 256>>>(a, b, n); break;
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < best[i]) best[i] = ms;
    }
  }
  for (size_t i = 0; i < vs.size(); ++i) {
    const double dirs = vs[i].id >= 30 ? 1.0 : 2.0;  // read-only / write-only move the bytes once
    printf("%-24s %.4f ms  %.1f GB/s  %.1f%% of 8 TB/s\n", vs[i].name, best[i], dirs * n * 16 / best[i] / 1e6,
           dirs * n * 16 / best[i] / 1e6 / 80.0);
  }
  return 0;
}
