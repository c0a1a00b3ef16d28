// Latency of the serial-decoder building blocks on one wave: a dependent chain of
// uniform LDS lookups (ds_read + readfirstlane), with and without a uniform byte
// store per step.  Diagnostic for k_inflate; not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int V, int RING = 32768>
__global__ __launch_bounds__(64) void k_chain(const uint32_t* init, uint64_t* out, int iters) {
  __shared__ uint32_t tab[512];
  __shared__ uint8_t ring[RING];
  for (int i = threadIdx.x; i < 512; i += 64) tab[i] = init[i];
  __syncthreads();
  uint32_t h = 1, pos = 0;
  const uint64_t t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    const uint32_t e = (uint32_t)__builtin_amdgcn_readfirstlane((int)tab[h & 511]);
    if (V == 1) ring[pos & (RING - 1)] = (uint8_t)e;
    if (V == 2) { if (threadIdx.x == 0) ring[pos & (RING - 1)] = (uint8_t)e; }
    if (V == 3) { const uint8_t v = ring[(pos - 100) & (RING - 1)]; ring[(pos + threadIdx.x) & (RING - 1)] = v; }
    h = (h >> 3) ^ e;
    pos += 1;
  }
  const uint64_t t1 = clock64();
  if (threadIdx.x == 0) out[blockIdx.x] = (t1 - t0) + (h == 12345 ? ring[pos & (RING - 1)] : 0);
}

int main() {
  uint32_t hinit[512];
  for (int i = 0; i < 512; ++i) hinit[i] = (uint32_t)(i * 2654435761u) >> 7;
  uint32_t* d_init;
  uint64_t* d_out;
  hipMalloc(&d_init, sizeof(hinit));
  hipMalloc(&d_out, 1024 * 8);
  hipMemcpy(d_init, hinit, sizeof(hinit), hipMemcpyHostToDevice);
  const int iters = 100000;
  for (int blocks : {1, 256, 1024}) {
    for (int v = 0; v < 4; ++v) {
      if (v == 0) hipLaunchKernelGGL(k_chain<0>, dim3(blocks), dim3(64), 0, 0, d_init, d_out, iters);
      if (v == 1) hipLaunchKernelGGL(k_chain<1>, dim3(blocks), dim3(64), 0, 0, d_init, d_out, iters);
      if (v == 2) hipLaunchKernelGGL(k_chain<2>, dim3(blocks), dim3(64), 0, 0, d_init, d_out, iters);
      if (v == 3) hipLaunchKernelGGL(k_chain<3>, dim3(blocks), dim3(64), 0, 0, d_init, d_out, iters);
      hipDeviceSynchronize();
      uint64_t c;
      hipMemcpy(&c, d_out, 8, hipMemcpyDeviceToHost);
      printf("blocks %4d variant %d: %.1f cycles/step\n", blocks, v, (double)c / iters);
    }
  }
  // occupancy: 4 KiB rings, 1..8 waves per SIMD
  for (int blocks : {1024, 2048, 4096, 8192}) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_chain<1, 4096>), dim3(blocks), dim3(64), 0, 0, d_init, d_out, iters);
    hipEventRecord(e1);
    hipDeviceSynchronize();
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    uint64_t c;
    hipMemcpy(&c, d_out, 8, hipMemcpyDeviceToHost);
    printf("small ring, blocks %5d: %.1f cycles/step per wave, %.3f ms, %.2f Gsteps/s\n", blocks, (double)c / iters, ms,
           (double)blocks * iters / ms / 1e6);
  }
  return 0;
}
