// Does a big H2D on one stream overlap a big D2H on another?  Measured with 0..7 other
// streams created first (the runtime spreads streams over GPU_MAX_HW_QUEUES hardware
// queues), for plain streams, CU-mask streams and high-priority streams.
//   hipcc --offload-arch=gfx950 -O2 tools/ubench_queues.hip -o tools/bin/ubench_queues
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static hipStream_t make(int kind) {
  hipStream_t s;
  if (kind == 0) {
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  } else if (kind == 1) {
    static const uint32_t all[16] = {~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u};
    CK(hipExtStreamCreateWithCUMask(&s, 16, all));
  } else {
    int lo, hi;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
  }
  return s;
}

int main() {
  const size_t B = 64u << 20;
  void *h1, *h2, *d1, *d2;
  CK(hipHostMalloc(&h1, B, 0));
  CK(hipHostMalloc(&h2, B, 0));
  CK(hipMalloc(&d1, B));
  CK(hipMalloc(&d2, B));
  const char* kinds[] = {"plain", "cumask", "highprio"};
  for (int kind = 0; kind < 3; ++kind) {
    for (int extra = 0; extra < 8; ++extra) {
      std::vector<hipStream_t> ex;
      for (int i = 0; i < extra; ++i) ex.push_back(make(0));
      hipStream_t a = make(kind), b = make(kind);
      double best_h = 1e9, best_d = 1e9, best_both = 1e9;
      for (int r = 0; r < 4; ++r) {
        double t0 = now_ms();
        CK(hipMemcpyAsync(d1, h1, B, hipMemcpyHostToDevice, a));
        CK(hipStreamSynchronize(a));
        double t1 = now_ms();
        CK(hipMemcpyAsync(h2, d2, B, hipMemcpyDeviceToHost, b));
        CK(hipStreamSynchronize(b));
        double t2 = now_ms();
        CK(hipMemcpyAsync(d1, h1, B, hipMemcpyHostToDevice, a));
        CK(hipMemcpyAsync(h2, d2, B, hipMemcpyDeviceToHost, b));
        CK(hipStreamSynchronize(a));
        CK(hipStreamSynchronize(b));
        double t3 = now_ms();
        if (r) {
          best_h = std::min(best_h, t1 - t0);
          best_d = std::min(best_d, t2 - t1);
          best_both = std::min(best_both, t3 - t2);
        }
      }
      printf("%-8s extra %d: H2D %.2f ms, D2H %.2f ms, both %.2f ms (overlap %.0f%%)\n", kinds[kind], extra, best_h,
             best_d, best_both, 100.0 * (best_h + best_d - best_both) / std::min(best_h, best_d));
      CK(hipStreamDestroy(a));
      CK(hipStreamDestroy(b));
      for (auto s : ex) CK(hipStreamDestroy(s));
    }
  }
  return 0;
}
