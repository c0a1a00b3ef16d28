// ubench_unmask.hip — kernel-level microbenchmark for the decode hot kernel.
// Builds the full decode pipeline once on a synthetic batch in HBM, then times
// k_pieces / k_piecesN variants and a plain 16-B copy of the same byte
// count (the streaming ceiling of this chip), interleaved in one process.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I.. tools/ubench_unmask.hip \
//         benchsupport/csrc/synth.hip -o /tmp/ubench
//   /tmp/ubench [frames] [payload] [text]
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../include/wsbench.h"

#include "../snf4j_amd/csrc/decode.hip"

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

__global__ __launch_bounds__(256) void k_copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) dst[i] = src[i];
}

int main(int argc, char** argv) {
  const uint64_t F = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 20);
  const uint32_t P = argc > 2 ? atoi(argv[2]) : 4096;
  const int text = argc > 3 ? atoi(argv[3]) : 1;
  const uint32_t fps = 1024;
  const uint32_t hl = 2 + (P > 0xffff ? 8 : P > 125 ? 2 : 0) + 4;
  const uint64_t flen = hl + P, wire_len = F * flen;
  const uint32_t S = (uint32_t)((F + fps - 1) / fps);
  uint8_t *wire, *payload;
  uint64_t* off;
  uint32_t* sf;
  CK(hipMalloc(&wire, wire_len + 64));
  CK(hipMalloc(&payload, wire_len + 16 * F + 64));
  CK(hipMalloc(&off, (F + 1) * 8));
  CK(hipMalloc(&sf, (S + 1) * 4));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  wsb_synth_uniform(0, st, 0x5EED, F, P, fps, text ? 1 : 2, 1, text, wire, off, sf);
  ws::DecodeArgs a{};
  a.wire = wire; a.wire_len = wire_len; a.frame_off = off; a.n_frames = F; a.session_first = sf; a.n_sessions = S;
  a.client_mode = 0; a.allow_ext = 0; a.validate = text; a.max_payload = 65536;
  CK(hipMalloc(&a.state, S * 8)); CK(hipMemset(a.state, 0, S * 8));
  a.payload_out = payload;
  CK(hipMalloc(&a.desc, F * 16)); CK(hipMalloc(&a.result, S * 16));
  a.nblk = (uint32_t)((F + ws::DBLOCK - 1) / ws::DBLOCK);
  CK(hipMalloc(&a.rec, F * sizeof(ws::FrameRec))); CK(hipMalloc(&a.vflag, F)); CK(hipMalloc(&a.slink, 3 * S * 4));
  CK(hipMalloc(&a.edge, 2 * F * 4));
  CK(hipMalloc(&a.blk_sum, a.nblk * 8)); CK(hipMalloc(&a.blk_max, 4 * a.nblk * 4)); CK(hipMalloc(&a.chunk_sum, (a.nblk / ws::SCAN_CHUNK + 1) * 8)); CK(hipMalloc(&a.chunk_max, (a.nblk / ws::SCAN_CHUNK + 1) * 16));
  CK(hipMalloc(&a.sess_err, S * 8)); CK(hipMalloc(&a.total, 8));
  const uint64_t npb = ws::piece_bound(wire_len, F);
  a.n_pieces = npb;
  CK(hipMalloc(&a.pieces, (npb + 8) * sizeof(ws::PieceDesc)));
  CK(hipMemsetAsync(a.sess_err, 0xff, S * 8, st));
  ws::launch_parse(a, st); ws::launch_scan(a, st); ws::launch_link(a, st);
  ws::launch_pieces(a, st, npb); ws::launch_final(a, st);
  CK(hipStreamSynchronize(st));
  std::vector<uint8_t> res(S * 16);
  CK(hipMemcpy(res.data(), a.result, S * 16, hipMemcpyDeviceToHost));
  uint64_t delivered = 0; int errs = 0;
  for (uint32_t s = 0; s < S; ++s) { delivered += *(uint32_t*)&res[16 * s]; errs += *(uint16_t*)&res[16 * s + 4] != 0; }
  printf("frames %llu payload %u text %d: delivered %llu errors %d\n", (unsigned long long)F, P, text,
         (unsigned long long)delivered, errs);

  const double alg = (double)wire_len + (double)F * P;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  struct V { const char* name; int kind; uint32_t grid; };
  std::vector<V> vs = {
      {"copy16 g=8192", 0, 8192}, {"pieces nt W1", 13, 0}, {"pieces nt W1 xcd", 14, 0},
      {"piecesN2 xcd", 18, 0}, {"piecesN4 xcd", 19, 0}, {"piecesN3 xcd", 24, 0}, {"piecesN4", 25, 0},
      {"parse", 20, 0}, {"scan", 23, 0}, {"link", 21, 0},  // pipeline order
  };
  std::vector<double> best(vs.size(), 1e30), sum(vs.size(), 0);
  const int rounds = 8;
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipEventRecord(e0, st));
      if (vs[i].kind == 0) {
        const uint64_t n16 = (uint64_t)(wire_len / 16);
        hipLaunchKernelGGL(k_copy16, dim3(vs[i].grid), dim3(256), 0, st, (const uint4*)wire, (uint4*)payload, n16);
      } else if (vs[i].kind == 10) {
        hipLaunchKernelGGL((ws::k_pieces<1, 4, 0>), dim3((uint32_t)((npb + 3) / 4)), dim3(256), 0, st, a);
      } else if (vs[i].kind == 13) {
        hipLaunchKernelGGL((ws::k_pieces<1, 1, 0>), dim3((uint32_t)npb), dim3(64), 0, st, a);
      } else if (vs[i].kind == 14) {
        hipLaunchKernelGGL((ws::k_pieces<1, 1, 1>), dim3((uint32_t)npb), dim3(64), 0, st, a);
      } else if (vs[i].kind == 15) {
        hipLaunchKernelGGL((ws::k_pieces<0, 1, 1>), dim3((uint32_t)npb), dim3(64), 0, st, a);
      } else if (vs[i].kind == 16) {
        hipLaunchKernelGGL((ws::k_pieces<1, 4, 1>), dim3((uint32_t)((npb + 3) / 4)), dim3(256), 0, st, a);
      } else if (vs[i].kind == 18) {
        hipLaunchKernelGGL((ws::k_piecesN<1, 1, 2>), dim3((uint32_t)((npb + 1) / 2)), dim3(64), 0, st, a);
      } else if (vs[i].kind == 19) {
        hipLaunchKernelGGL((ws::k_piecesN<1, 1, 4>), dim3((uint32_t)((npb + 3) / 4)), dim3(64), 0, st, a);
      } else if (vs[i].kind == 24) {
        hipLaunchKernelGGL((ws::k_piecesN<1, 1, 3>), dim3((uint32_t)((npb + 2) / 3)), dim3(64), 0, st, a);
      } else if (vs[i].kind == 25) {
        hipLaunchKernelGGL((ws::k_piecesN<1, 0, 4>), dim3((uint32_t)((npb + 3) / 4)), dim3(64), 0, st, a);
      } else if (vs[i].kind == 20) {
        ws::launch_parse(a, st);
      } else if (vs[i].kind == 21) {
        ws::launch_link(a, st);
      } else if (vs[i].kind == 23) {
        ws::launch_scan(a, st);
      }
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0) { best[i] = ms < best[i] ? ms : best[i]; sum[i] += ms; }
    }
  }
  for (size_t i = 0; i < vs.size(); ++i) {
    const double bytes = vs[i].kind == 0 ? 2.0 * (double)(wire_len / 16 * 16) : alg;
    if (vs[i].kind >= 20) { printf("%-22s best %.4f ms\n", vs[i].name, best[i]); continue; }
    printf("%-22s best %.4f ms  avg %.4f ms  %.1f GB/s (best)  %.1f%% of 8 TB/s\n", vs[i].name, best[i],
           sum[i] / (rounds - 1), bytes / best[i] / 1e6, bytes / best[i] / 1e6 / 80.0);
  }
  return 0;
}
