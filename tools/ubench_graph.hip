// Inter-kernel gap of a dependent launch chain on one stream: plain launches,
// plain launches with an event pair around one kernel, and the same chain replayed
// as a captured hipGraph (with and without event record nodes in it).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_small(unsigned* p, unsigned n) {  // a few us of work
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 3u + 1u;
}

static void chain(hipStream_t s, unsigned* p, unsigned n, hipEvent_t e0, hipEvent_t e1, bool ev) {
  hipLaunchKernelGGL(k_small, dim3((n + 255) / 256), dim3(256), 0, s, p, n);
  hipLaunchKernelGGL(k_small, dim3((n + 255) / 256), dim3(256), 0, s, p, n);
  if (ev) CK(hipEventRecord(e0, s));
  hipLaunchKernelGGL(k_small, dim3((n + 255) / 256), dim3(256), 0, s, p, n);
  if (ev) CK(hipEventRecord(e1, s));
  hipLaunchKernelGGL(k_small, dim3((n + 255) / 256), dim3(256), 0, s, p, n);
}

// a streaming copy shaped like k_piecesN: one 64-lane workgroup per KiB
__global__ __launch_bounds__(64) void k_big(const uint4* __restrict__ in, uint4* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  out[i] = in[i];
}

static float time_ms(hipStream_t s, hipEvent_t t0, hipEvent_t t1, int R, void (*body)(hipStream_t, void*), void* arg) {
  for (int w = 0; w < 5; ++w) body(s, arg);
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(t0, s));
  for (int r = 0; r < R; ++r) body(s, arg);
  CK(hipEventRecord(t1, s));
  CK(hipStreamSynchronize(s));
  float ms; CK(hipEventElapsedTime(&ms, t0, t1));
  return ms / R;
}
struct BigArgs { uint4* in; uint4* out; unsigned nblk; unsigned* p; unsigned n; };
static void big_only(hipStream_t s, void* v) {
  BigArgs* a = (BigArgs*)v;
  hipLaunchKernelGGL(k_big, dim3(a->nblk), dim3(64), 0, s, a->in, a->out);
}
static void small_only(hipStream_t s, void* v) {
  BigArgs* a = (BigArgs*)v;
  hipLaunchKernelGGL(k_small, dim3((a->n + 255) / 256), dim3(256), 0, s, a->p, a->n);
}
static void big_chain(hipStream_t s, void* v) {
  BigArgs* a = (BigArgs*)v;
  small_only(s, v); small_only(s, v); big_only(s, v); small_only(s, v);
}

int main() {
  const unsigned n = 1u << 20;
  unsigned* p;
  CK(hipMalloc(&p, n * 4));
  CK(hipMemset(p, 0, n * 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1, t0, t1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&t0)); CK(hipEventCreate(&t1));
  const int R = 2000;
  for (int mode = 0; mode < 4; ++mode) {
    const bool ev = mode & 1, graph = mode >= 2;
    hipGraphExec_t ex = nullptr;
    if (graph) {
      hipGraph_t g;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
      chain(s, p, n, e0, e1, ev);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    }
    for (int w = 0; w < 50; ++w) { if (graph) CK(hipGraphLaunch(ex, s)); else chain(s, p, n, e0, e1, ev); }
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(t0, s));
    for (int r = 0; r < R; ++r) { if (graph) CK(hipGraphLaunch(ex, s)); else chain(s, p, n, e0, e1, ev); }
    CK(hipEventRecord(t1, s));
    CK(hipStreamSynchronize(s));
    float ms; CK(hipEventElapsedTime(&ms, t0, t1));
    float kms = 0; if (ev) CK(hipEventElapsedTime(&kms, e0, e1));
    printf("%-22s %8.2f us per 4-kernel chain  (event pair around kernel 3: %.2f us)\n",
           graph ? (ev ? "graph + event nodes" : "graph") : (ev ? "launches + events" : "launches"), 1000.f * ms / R, 1000.f * kms);
  }
  // one kernel alone, back to back (no dependency chain difference on one stream)
  CK(hipEventRecord(t0, s));
  for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_small, dim3((n + 255) / 256), dim3(256), 0, s, p, n);
  CK(hipEventRecord(t1, s));
  CK(hipStreamSynchronize(s));
  float ms; CK(hipEventElapsedTime(&ms, t0, t1));
  printf("%-22s %8.2f us per kernel\n", "single launches", 1000.f * ms / R);
  // a 1 GiB streaming copy between small kernels: does its boundary cost more?
  BigArgs ba;
  ba.nblk = 1u << 20;  // 1 GiB
  CK(hipMalloc(&ba.in, (size_t)ba.nblk * 1024));
  CK(hipMalloc(&ba.out, (size_t)ba.nblk * 1024));
  CK(hipMemset(ba.in, 1, (size_t)ba.nblk * 1024));
  ba.p = p; ba.n = n;
  const float tb = time_ms(s, t0, t1, 50, big_only, &ba), ts = time_ms(s, t0, t1, 500, small_only, &ba),
              tc = time_ms(s, t0, t1, 50, big_chain, &ba);
  printf("big copy alone %.2f us, small alone %.2f us, [small small big small] %.2f us: %.2f us beyond the parts\n",
         1000.f * tb, 1000.f * ts, 1000.f * tc, 1000.f * (tc - tb - 3 * ts));
  return 0;
}
