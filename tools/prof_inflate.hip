// Phase profile of k_inflate: the kernel compiled with WSG_INFLATE_PROF (clock64 per
// phase, summed over sessions) over a batch written by tools/make_inflate_input.py.
// Diagnostic only; not part of the library.
#ifndef NO_PROF
#define WSG_INFLATE_PROF 1
#endif
#include "../snf4j_amd/csrc/inflate.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  FILE* f = fopen(argc > 1 ? argv[1] : "gpurun_out/infl_in.bin", "rb");
  if (!f) { printf("no input\n"); return 1; }
  uint64_t hdr[4];  // n_frames, n_sessions, payload_len, cap per session
  if (fread(hdr, 8, 4, f) != 4) return 1;
  const uint64_t n = hdr[0], ns = hdr[1], pl = hdr[2], cap = hdr[3];
  std::vector<wsg_frame_desc> desc(n);
  std::vector<uint32_t> sf(ns + 1);
  std::vector<uint8_t> payload(pl);
  if (fread(desc.data(), sizeof(wsg_frame_desc), n, f) != n) return 1;
  if (fread(sf.data(), 4, ns + 1, f) != ns + 1) return 1;
  if (fread(payload.data(), 1, pl, f) != pl) return 1;
  fclose(f);
  std::vector<uint64_t> off(ns + 1);
  for (uint64_t i = 0; i <= ns; ++i) off[i] = i * cap;
  ws::InflArgs a{};
  wsg_frame_desc *d_desc, *d_odesc;
  uint32_t *d_sf, *d_rf;
  uint8_t *d_pl, *d_win, *d_out;
  uint64_t* d_off;
  wsg_inflate_state* d_st;
  wsg_session_result* d_res;
  CK(hipMalloc(&d_desc, n * sizeof(wsg_frame_desc)));
  CK(hipMalloc(&d_odesc, n * sizeof(wsg_frame_desc)));
  CK(hipMalloc(&d_sf, (ns + 1) * 4));
  CK(hipMalloc(&d_rf, ns * 4));
  CK(hipMalloc(&d_pl, pl));
  CK(hipMalloc(&d_win, ns * 32768));
  CK(hipMalloc(&d_out, ns * cap));
  CK(hipMalloc(&d_off, (ns + 1) * 8));
  CK(hipMalloc(&d_st, ns * sizeof(wsg_inflate_state)));
  CK(hipMalloc(&d_res, ns * sizeof(wsg_session_result)));
  CK(hipMemcpy(d_desc, desc.data(), n * sizeof(wsg_frame_desc), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_sf, sf.data(), (ns + 1) * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_pl, payload.data(), pl, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_off, off.data(), (ns + 1) * 8, hipMemcpyHostToDevice));
  a.no_context = 0; a.desc = d_desc; a.n_frames = n; a.session_first = d_sf; a.n_sessions = (uint32_t)ns;
  a.payload = d_pl; a.payload_len = pl; a.state = d_st; a.window = d_win; a.out = d_out; a.out_off = d_off;
  a.out_desc = d_odesc; a.result = d_res; a.replay_from = d_rf;
  unsigned long long z[24] = {};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemset(d_st, 0, ns * sizeof(wsg_inflate_state)));
#ifdef WSG_INFLATE_PROF
    CK(hipMemcpyToSymbol(HIP_SYMBOL(ws::g_infl_prof), z, sizeof(z)));
#endif
    CK(hipEventRecord(e0));
    ws::launch_inflate(a, 0);
    CK(hipEventRecord(e1));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long p[24] = {};
#ifdef WSG_INFLATE_PROF
    CK(hipMemcpyFromSymbol(p, HIP_SYMBOL(ws::g_infl_prof), sizeof(p)));
#endif
    std::vector<wsg_session_result> r(ns);
    CK(hipMemcpy(r.data(), d_res, ns * sizeof(wsg_session_result), hipMemcpyDeviceToHost));
    uint64_t errs = 0;
    for (auto& x : r) errs += x.error != 0;
    const char* names[24] = {"total", "carry_in", "fast_loop", "header_iters", "len_iters(incl fast)", "done_iters",
                             "flush", "commit", "frame_setup", "fast_literals", "fast_matches", "fast_match_bytes",
                             "restages", "slow_len_iters", "blocks", "frames", "lit_path", "long_lit_canon",
                             "long_lit_count", "long_dist_count", "len+dist decode", "dist extra+copy", "whole match sym"};
    printf("rep %d: %.3f ms, %llu sessions with error\n", rep, ms, (unsigned long long)errs);
    for (int i = 0; i < 23; ++i)
      printf("  %-22s %14.1f per session%s\n", names[i], (double)p[i] / ns, i < 9 ? " cycles" : "");
  }
  return 0;
}
