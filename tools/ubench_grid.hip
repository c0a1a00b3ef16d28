// The validator stage's bound: its piece kernel reads 4.3 GB as 1.05 M
// one-wave workgroups of 4 KiB.  Is the dispatch of that many workgroups the floor, or
// the read stream?  Times (HIP events, best of 8):
//   empty    N one-wave workgroups that return at once (the dispatch-rate floor)
//   readK    the same bytes read by one-wave workgroups of K KiB each (K = 4, 8, 16, 32):
//            16-B nontemporal buffer loads, K/1 KiB in flight a lane group, a dword
//            written only if a never-true test on the data holds (so nothing is dead code)
//   hipMemcpy D2D of the same bytes (read + write, for scale)
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_grid.hip -o tools/bin/ubench_grid
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void k_empty(unsigned* out) {
  if (threadIdx.x == 1000) out[0] = 1;  // never: keeps the kernel from being elided
}

template <int K>
__global__ __launch_bounds__(64) void k_read(const unsigned char* __restrict__ src, unsigned* out, unsigned magic) {
  const size_t base = (size_t)blockIdx.x * (K * 1024);
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(src + base), 0, K * 1024, 0x00020000);
  u32x4 v[K];
#pragma unroll
  for (int i = 0; i < K; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(r, threadIdx.x * 16u + i * 1024u, 0, 2);
  unsigned x = 0;
#pragma unroll
  for (int i = 0; i < K; ++i) x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  if (x == magic) out[threadIdx.x] = x;  // (magic is chosen so this never holds)
}

template <int K>
static float run_read(const unsigned char* d, unsigned* o, size_t bytes, hipEvent_t a, hipEvent_t b) {
  float best = 1e9f;
  const unsigned grid = (unsigned)(bytes / (K * 1024));
  for (int rep = 0; rep < 8; ++rep) {
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(k_read<K>, dim3(grid), dim3(64), 0, 0, d, o, 0xDEADBEEFu);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  printf("{\"mode\": \"read%d\", \"workgroups\": %u, \"bytes\": %zu, \"best_ms\": %.4f, \"GB_per_s\": %.1f}\n", K,
         grid, bytes, best, bytes / (best * 1e-3) / 1e9);
  return best;
}

int main() {
  const size_t bytes = (size_t)1048576 * 4096;  // the validator line's payload region (4.3 GB)
  unsigned char *d, *d2;
  unsigned* o;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&d2, bytes));
  CK(hipMalloc(&o, 4096));
  CK(hipMemset(d, 0x5A, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (unsigned grid : {1048576u, 1060000u, 524288u}) {
    float best = 1e9f;
    for (int rep = 0; rep < 8; ++rep) {
      CK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(k_empty, dim3(grid), dim3(64), 0, 0, o);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    printf("{\"mode\": \"empty\", \"workgroups\": %u, \"best_ms\": %.4f, \"Mwg_per_s\": %.1f}\n", grid, best,
           grid / (best * 1e-3) / 1e6);
  }
  run_read<4>(d, o, bytes, a, b);
  run_read<8>(d, o, bytes, a, b);
  run_read<16>(d, o, bytes, a, b);
  run_read<32>(d, o, bytes, a, b);
  float best = 1e9f;
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipEventRecord(a, 0));
    CK(hipMemcpyAsync(d2, d, bytes, hipMemcpyDeviceToDevice, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  printf("{\"mode\": \"d2d_copy\", \"bytes\": %zu, \"best_ms\": %.4f, \"GB_per_s_read_plus_write\": %.1f}\n", bytes, best,
         2 * bytes / (best * 1e-3) / 1e9);
  return 0;
}
