// What an agent-scope release costs a workgroup on MI355X (8 XCDs, an L2 each): the
// price of a single-pass (decoupled look-back) aggregator plan.  Each of nblk blocks
// writes 256 x 24 B of per-frame results (as the plan's k_agg_b does), then publishes
// a per-block flag: (0) plain store, (1) a device-scope release fence before it
// (__threadfence: buffer_wbl2 sc1 + waits), (2) (1) plus a look-back: thread 0 waits
// with acquire loads for the previous block's flag.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int MODE>
__global__ __launch_bounds__(256) void k(unsigned* flags, unsigned long long* data, unsigned* ticket, unsigned epoch) {
  __shared__ unsigned s_b;
  if (threadIdx.x == 0) s_b = atomicAdd(ticket, 1u);
  __syncthreads();
  const unsigned b = s_b;
  const unsigned long long i = (unsigned long long)b * 256 + threadIdx.x;
  data[3 * i] = i;
  data[3 * i + 1] = i * 7;
  data[3 * i + 2] = i ^ 5;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (MODE == 2 && b > 0) {
      unsigned f;
      do { f = __hip_atomic_load(&flags[b - 1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT); } while (f != epoch);
    }
    if (MODE >= 1) __hip_atomic_store(&flags[b], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_store(&flags[b], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

int main(int argc, char** argv) {
  const unsigned nblk = argc > 1 ? (unsigned)atoi(argv[1]) : 2128u;
  unsigned *flags, *ticket;
  unsigned long long* data;
  CK(hipMalloc(&flags, nblk * 4));
  CK(hipMalloc(&ticket, 4));
  CK(hipMalloc(&data, (size_t)nblk * 256 * 24));
  CK(hipMemset(flags, 0, nblk * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  unsigned epoch = 0;
  for (int mode = 0; mode < 3; ++mode) {
    float best = 1e9f;
    for (int rep = 0; rep < 10; ++rep) {
      ++epoch;
      CK(hipMemset(ticket, 0, 4));
      CK(hipEventRecord(e0));
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(nblk), dim3(256), 0, 0, flags, data, ticket, epoch);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(nblk), dim3(256), 0, 0, flags, data, ticket, epoch);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(nblk), dim3(256), 0, 0, flags, data, ticket, epoch);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    printf("mode %d (%s): %u blocks, best %.1f us\n", mode,
           mode == 0 ? "plain flag store" : (mode == 1 ? "release fence + flag" : "release + serial acquire look-back"),
           nblk, best * 1e3f);
  }
  return 0;
}
