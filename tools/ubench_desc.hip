// ubench_desc.hip — what a per-wave work descriptor costs the streaming kernel.
// Each wave unmasks 2 KiB (2 x 16 B per lane, nontemporal buffer loads/stores,
// XCD-aware block order), 4.3 GB in + 4.3 GB out, variants interleaved:
//   copy     addresses from blockIdx, mask constant (the ceiling of this shape)
//   dep      descriptor (16 B scalar load) first, data address taken from it
//   par      data address from blockIdx, descriptor loaded in parallel (mask from it)
//   par2     as par, with a 2-step dependent chain (piece index -> 32-B record)
//   *_valu   + ~230 dependent VALU ops per lane-chunk pair (the UTF-8 rule's cost)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_desc.hip -o /tmp/ubench_desc
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Desc {
  uint64_t src;
  uint32_t mask, frame;
};
struct Rec {
  uint64_t src;
  uint64_t pad;
  uint32_t len, mask, code, sess;
};

__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t n) {
  const uint32_t q = n / 8u, r = n % 8u, x = b % 8u, i = b / 8u;
  return (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + i;
}

__device__ __forceinline__ uint32_t valu_work(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  uint32_t x = a, y = b;
#pragma unroll
  for (int i = 0; i < 28; ++i) {
    x = __builtin_amdgcn_alignbyte(y, x, 1) ^ (c + i);
    y = __builtin_amdgcn_perm(x, d, 0x05010400u + i) & (y | 0x80808080u);
  }
  return x ^ y;
}

// MODE 0 copy, 1 dep, 2 par, 3 par2; VALU: add the per-chunk work; W bytes per wave
template <int MODE, int VALU, int W = 2048>
__global__ __launch_bounds__(64) void k_uw(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                           const Desc* __restrict__ desc, const uint32_t* __restrict__ pidx,
                                           const Rec* __restrict__ rec, uint32_t* __restrict__ flag) {
  const int lane = threadIdx.x;
  const uint32_t w = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x));
  uint64_t src = (uint64_t)w * W;
  uint32_t mask = 0x5A5A5A5Au;
  u32x4 a, b;
  const uint32_t boff = (uint32_t)lane * 16u;
  if (MODE == 1) {
    const Desc d = desc[w];
    asm volatile("" ::"s"(d.src), "s"(d.mask));
    src = d.src;
    mask = d.mask;
  }
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void*)(in + src), 0, W, 0x00020000);
  a = __builtin_amdgcn_raw_buffer_load_b128(rin, boff, 0, 2);
  if (W > 1024) b = __builtin_amdgcn_raw_buffer_load_b128(rin, boff + 1024, 0, 2);
  else b = a;
  if (MODE == 2) {
    const Desc d = desc[w];
    mask = d.mask;
  } else if (MODE == 3) {
    const uint32_t k = pidx[w];
    const Rec r = rec[k];
    mask = r.mask ^ r.code;
  }
  a ^= mask;
  b ^= mask;
  if (VALU) {
    const uint32_t e = W > 1024 ? (valu_work(a.x, a.y, a.z, a.w) | valu_work(b.x, b.y, b.z, b.w))
                                : valu_work(a.x, a.y, a.z, a.w);
    if (__builtin_amdgcn_read_exec() && e == 0x12345678u) atomicOr(flag, 1u);
  }
  const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc((void*)(out + (uint64_t)w * W), 0, W,
                                                                        0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(a, rout, boff, 0, 2);
  if (W > 1024) __builtin_amdgcn_raw_buffer_store_b128(b, rout, boff + 1024, 0, 2);
}

// shape variants without descriptors: W bytes per wave (1 or 2 KiB), G = 1: global
// nontemporal builtins instead of buffer intrinsics, WPB waves per workgroup
template <int W, int G, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_shape(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                    const Desc* __restrict__, const uint32_t* __restrict__,
                                                    const Rec* __restrict__, uint32_t* __restrict__) {
  const int lane = threadIdx.x & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * WPB + (threadIdx.x >> 6));
  const uint64_t base = (uint64_t)w * W;
  if (G) {
    const u32x4* s = (const u32x4*)(in + base) + lane;
    u32x4* d = (u32x4*)(out + base) + lane;
    u32x4 v[W / 1024];
#pragma unroll
    for (int i = 0; i < W / 1024; ++i) v[i] = __builtin_nontemporal_load(s + 64 * i);
#pragma unroll
    for (int i = 0; i < W / 1024; ++i) __builtin_nontemporal_store(v[i] ^ 0x5A5A5A5Au, d + 64 * i);
  } else {
    const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void*)(in + base), 0, W, 0x00020000);
    const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc((void*)(out + base), 0, W, 0x00020000);
    u32x4 v[W / 1024];
#pragma unroll
    for (int i = 0; i < W / 1024; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rin, lane * 16 + 1024 * i, 0, 2);
#pragma unroll
    for (int i = 0; i < W / 1024; ++i)
      __builtin_amdgcn_raw_buffer_store_b128(v[i] ^ 0x5A5A5A5Au, rout, lane * 16 + 1024 * i, 0, 2);
  }
}

// 2 KiB per wave, other layouts: IL = 1: lane i takes bytes [32i, 32i+32) (two adjacent
// 16-B loads); IL = 2: the wave's two KiB are far apart (piece w and w + n/2)
template <int IL>
__global__ __launch_bounds__(64) void k_lay(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                            const Desc* __restrict__, const uint32_t* __restrict__,
                                            const Rec* __restrict__, uint32_t* __restrict__) {
  const int lane = threadIdx.x;
  const uint32_t w = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x));
  uint64_t b0, b1;
  uint32_t o0, o1;
  if (IL == 1) {
    b0 = b1 = (uint64_t)w * 2048u;
    o0 = lane * 32u;
    o1 = lane * 32u + 16u;
  } else {
    b0 = (uint64_t)w * 1024u;
    b1 = ((uint64_t)w + gridDim.x) * 1024u;
    o0 = o1 = lane * 16u;
  }
  const __amdgpu_buffer_rsrc_t r0 = __builtin_amdgcn_make_buffer_rsrc((void*)(in + b0), 0, 2048, 0x00020000);
  const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc((void*)(in + b1), 0, 2048, 0x00020000);
  u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r0, o0, 0, 2);
  u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r1, o1, 0, 2);
  const __amdgpu_buffer_rsrc_t q0 = __builtin_amdgcn_make_buffer_rsrc((void*)(out + b0), 0, 2048, 0x00020000);
  const __amdgpu_buffer_rsrc_t q1 = __builtin_amdgcn_make_buffer_rsrc((void*)(out + b1), 0, 2048, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(a ^ 0x5A5A5A5Au, q0, o0, 0, 2);
  __builtin_amdgcn_raw_buffer_store_b128(b ^ 0x5A5A5A5Au, q1, o1, 0, 2);
}

int main(int argc, char** argv) {
  const uint64_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 4200ull) << 20;  // MiB
  const uint32_t waves = (uint32_t)(bytes / 2048);
  uint8_t *in, *out;
  Desc* desc;
  uint32_t *pidx, *flag;
  Rec* rec;
  CK(hipMalloc(&in, bytes));
  CK(hipMalloc(&out, bytes));
  CK(hipMalloc(&desc, (uint64_t)waves * sizeof(Desc)));
  CK(hipMalloc(&pidx, (uint64_t)waves * 4));
  Desc* desc1;
  uint32_t* pidx1;
  CK(hipMalloc(&desc1, (uint64_t)waves * 2 * sizeof(Desc)));
  CK(hipMalloc(&pidx1, (uint64_t)waves * 2 * 4));
  CK(hipMalloc(&rec, (uint64_t)waves / 2 * sizeof(Rec) + 64));
  CK(hipMalloc(&flag, 4));
  CK(hipMemset(in, 0x3c, bytes));
  {
    std::vector<Desc> hd(waves);
    std::vector<uint32_t> hp(waves);
    std::vector<Rec> hr(waves / 2 + 1);
    for (uint32_t i = 0; i < waves; ++i) {
      hd[i] = {(uint64_t)i * 2048u, 0x01020304u ^ i, i / 2};
      hp[i] = i / 2;  // two 2-KiB waves per 4 KiB "frame"
    }
    for (uint32_t i = 0; i <= waves / 2; ++i) hr[i] = {(uint64_t)i * 4096u, 0, 4096, 0x11223344u ^ i, 0, 0};
    CK(hipMemcpy(desc, hd.data(), hd.size() * sizeof(Desc), hipMemcpyHostToDevice));
    CK(hipMemcpy(pidx, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(rec, hr.data(), hr.size() * sizeof(Rec), hipMemcpyHostToDevice));
    std::vector<Desc> hd1(2 * (uint64_t)waves);
    std::vector<uint32_t> hp1(2 * (uint64_t)waves);
    for (uint32_t i = 0; i < 2 * waves; ++i) {
      hd1[i] = {(uint64_t)i * 1024u, 0x01020304u ^ i, i / 4};
      hp1[i] = i / 4;
    }
    CK(hipMemcpy(desc1, hd1.data(), hd1.size() * sizeof(Desc), hipMemcpyHostToDevice));
    CK(hipMemcpy(pidx1, hp1.data(), hp1.size() * 4, hipMemcpyHostToDevice));
  }
  struct V {
    const char* name;
    void (*k)(const uint8_t*, uint8_t*, const Desc*, const uint32_t*, const Rec*, uint32_t*);
  } vs[] = {
      {"copy", k_uw<0, 0>},      {"dep", k_uw<1, 0>},       {"par", k_uw<2, 0>},       {"par2", k_uw<3, 0>},
      {"copy_valu", k_uw<0, 1>}, {"dep_valu", k_uw<1, 1>}, {"par_valu", k_uw<2, 1>}, {"par2_valu", k_uw<3, 1>},
      {"b1k", k_shape<1024, 0, 1>}, {"g1k", k_shape<1024, 1, 1>}, {"b2k", k_shape<2048, 0, 1>},
      {"g2k", k_shape<2048, 1, 1>}, {"b1k_x4", k_shape<1024, 0, 4>}, {"g1k_x4", k_shape<1024, 1, 4>},
      {"b4k", k_shape<4096, 0, 1>}, {"g4k", k_shape<4096, 1, 1>},
      {"1copy_valu", k_uw<0, 1, 1024>}, {"1dep", k_uw<1, 0, 1024>}, {"1dep_valu", k_uw<1, 1, 1024>},
      {"1par_valu", k_uw<2, 1, 1024>}, {"1par2_valu", k_uw<3, 1, 1024>},
      {"lay_il", k_lay<1>}, {"lay_far", k_lay<2>}, {"b1k_x2", k_shape<1024, 0, 2>}, {"b1k_b", k_shape<1024, 0, 1>},
  };
  // grid in workgroups per variant: 2 KiB per wave by default
  const int nv = sizeof vs / sizeof vs[0];
  std::vector<float> best(nv, 1e30f);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 6; ++rep) {
    for (int v = 0; v < nv; ++v) {
      CK(hipEventRecord(e0, 0));
      uint32_t grid = waves, block = 64;
      const char* n = vs[v].name;
      if (n[0] == '1') {
        grid = (uint32_t)(bytes / 1024u);
      } else if (n[0] == 'b' || n[0] == 'g') {
        const int kb = n[1] - '0';
        const int wpb = n[3] == '_' ? (n[5] == '2' ? 2 : (n[5] == '4' ? 4 : 1)) : 1;
        grid = (uint32_t)(bytes / (1024u * kb) / wpb);
        block = 64 * wpb;
      }
      const bool one = n[0] == '1';
      hipLaunchKernelGGL(vs[v].k, dim3(grid), dim3(block), 0, 0, in, out, one ? desc1 : desc, one ? pidx1 : pidx, rec,
                         flag);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 0 && ms < best[v]) best[v] = ms;
    }
  }
  for (int v = 0; v < nv; ++v)
    printf("%-10s %8.4f ms  %7.1f GB/s (read+write)\n", vs[v].name, best[v], 2.0 * bytes / (best[v] * 1e-3) / 1e9);
  return 0;
}
