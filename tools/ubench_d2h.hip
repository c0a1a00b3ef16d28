// Device -> pinned host bandwidth on this box, the ceiling k_stage_copy (the stage chain's
// gather of inflated bytes into pinned memory, batcher.hip) works against: GB/s of
//   copy    hipMemcpyAsync device -> pinned host
//   kwrite  a kernel storing 16-B vectors into the pinned buffer (mapped), as k_stage_copy does
//   kwrite+h2d  the same with a host -> device copy of the same size in flight on another stream
//   copy+h2d    hipMemcpyAsync both ways at once
// for 8, 54 and 256 MB (54 MB: a bench stage flush's inflated output).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_d2h.hip -o tools/bin/ubench_d2h
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

__global__ __launch_bounds__(256) void k_write(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

int main() {
  hipStream_t s, t;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
  const size_t MAXB = 256u << 20;
  void *d, *d2, *h, *h2, *hmap;
  CK(hipMalloc(&d, MAXB));
  CK(hipMalloc(&d2, MAXB));
  CK(hipHostMalloc(&h, MAXB, 0));
  CK(hipHostMalloc(&h2, MAXB, 0));
  CK(hipMemset(d, 1, MAXB));
  CK(hipHostGetDevicePointer(&hmap, h, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const size_t sizes[] = {8u << 20, 54u << 20, 256u << 20};
  for (size_t sz : sizes) {
    for (int mode = 0; mode < 4; mode++) {
      const bool kern = mode == 1 || mode == 2, h2d = mode >= 2;
      float best = 1e9f;
      for (int rep = 0; rep < 8; rep++) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, s));
        if (h2d) CK(hipMemcpyAsync(d2, h2, sz, hipMemcpyHostToDevice, t));
        if (kern)
          hipLaunchKernelGGL(k_write, dim3(1024), dim3(256), 0, s, (const uint4*)d, (uint4*)hmap, sz / 16);
        else
          CK(hipMemcpyAsync(h, d, sz, hipMemcpyDeviceToHost, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
      }
      CK(hipDeviceSynchronize());
      static const char* names[] = {"copy", "kwrite", "kwrite+h2d", "copy+h2d"};
      printf("{\"mode\": \"%s\", \"bytes\": %zu, \"best_ms\": %.4f, \"GB_per_s\": %.1f}\n", names[mode], sz, best,
             sz / (best * 1e-3) / 1e9);
    }
  }
  return 0;
}
