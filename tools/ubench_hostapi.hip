// Host-side cost of the HIP calls a stage flush makes (the batcher's per-flush
// uploads, launches and events): microseconds per call on the calling thread, with
// the device idle and with a large H2D in flight on another stream.
//   hipcc --offload-arch=gfx950 -O2 tools/ubench_hostapi.hip -o /tmp/ubench_hostapi
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__global__ void k_pull(const uint4* __restrict__ src, uint4* __restrict__ dst, unsigned n16) {
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x) dst[i] = src[i];
}

__global__ void k_touch(const unsigned* p, unsigned* q, unsigned n) {
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) q[i] = p[i] + 1;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t s, big;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&big, hipStreamNonBlocking));
  const size_t MAXB = 8u << 20, BIG = 256u << 20;
  void *hp, *dp, *hbig, *dbig;
  CK(hipHostMalloc(&hp, MAXB, 0));
  CK(hipMalloc(&dp, MAXB));
  CK(hipHostMalloc(&hbig, BIG, 0));
  CK(hipMalloc(&dbig, BIG));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const size_t sizes[] = {256, 4096, 65536, 262144, 1u << 20, 4u << 20};
  for (int busy = 0; busy < 2; ++busy) {
    for (size_t sz : sizes) {
      const int R = 50;
      CK(hipStreamSynchronize(s));
      if (busy) CK(hipMemcpyAsync(dbig, hbig, BIG, hipMemcpyHostToDevice, big));  // ~4.5 ms of DMA
      double t0 = now_us();
      for (int r = 0; r < R; ++r) CK(hipMemcpyAsync(dp, hp, sz, hipMemcpyHostToDevice, s));
      double t1 = now_us();
      CK(hipStreamSynchronize(s));
      double t2 = now_us();
      for (int r = 0; r < R; ++r) CK(hipMemcpyAsync(hp, dp, sz, hipMemcpyDeviceToHost, s));
      double t3 = now_us();
      CK(hipStreamSynchronize(s));
      CK(hipStreamSynchronize(big));
      printf("%s H2D %8zu B: %7.1f us/call (+%7.1f us to drain)   D2H: %7.1f us/call\n", busy ? "busy" : "idle", sz,
             (t1 - t0) / R, (t2 - t1), (t3 - t2) / R);
    }
    const int R = 200;
    if (busy) CK(hipMemcpyAsync(dbig, hbig, BIG, hipMemcpyHostToDevice, big));
    double t0 = now_us();
    for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_touch, dim3(64), dim3(256), 0, s, (const unsigned*)dp, (unsigned*)dp + 65536, 16384u);
    double t1 = now_us();
    for (int r = 0; r < R; ++r) CK(hipEventRecord(ev, s));
    double t2 = now_us();
    CK(hipStreamSynchronize(s));
    double t3 = now_us();
    for (int r = 0; r < R; ++r) (void)hipEventQuery(ev);
    double t4 = now_us();
    CK(hipStreamSynchronize(big));
    printf("%s launch %.1f us/call, eventRecord %.1f us/call, eventQuery %.2f us/call\n", busy ? "busy" : "idle",
           (t1 - t0) / R, (t2 - t1) / R, (t4 - t3) / R);
  }
  // per call: hipMemcpyAsync H2D (pinned source) against a kernel that pulls the same
  // bytes over PCIe from the mapped pinned buffer; host us per call (median / max of 40)
  // and the device time to drain all 40
  void* hmap = nullptr;
  CK(hipHostGetDevicePointer(&hmap, hp, 0));
  const size_t sz2[] = {16384, 65536, 212992, 327680};
  for (size_t sz : sz2) {
    for (int mode = 0; mode < 2; ++mode) {
      const int R = 40;
      double c[R];
      CK(hipStreamSynchronize(s));
      const double tb = now_us();
      for (int r = 0; r < R; ++r) {
        const double a = now_us();
        if (mode == 0) CK(hipMemcpyAsync(dp, hp, sz, hipMemcpyHostToDevice, s));
        else hipLaunchKernelGGL(k_pull, dim3(64), dim3(256), 0, s, (const uint4*)hmap, (uint4*)dp, (unsigned)(sz / 16));
        c[r] = now_us() - a;
      }
      const double te = now_us();
      CK(hipStreamSynchronize(s));
      const double td = now_us();
      for (int i = 0; i < R; ++i)
        for (int j = i + 1; j < R; ++j)
          if (c[j] < c[i]) { double t = c[i]; c[i] = c[j]; c[j] = t; }
      printf("%-8s %7zu B: host median %6.1f max %8.1f us; 40 calls %8.1f us + drain %8.1f us\n",
             mode ? "kernel" : "memcpy", sz, c[R / 2], c[R - 1], te - tb, td - te);
    }
  }
  return 0;
}
