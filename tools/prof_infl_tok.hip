// Phase profile of k_infl_tok (the message-parallel pre-decode): the kernel compiled
// with WSG_INFLATE_TOK_PROF (clock64 per phase, summed over lanes) over a batch
// written by tools/make_inflate_input.py.  Diagnostic only; not part of the library.
#define WSG_INFLATE_TOK_PROF 1
#ifndef INFL_SRC  // (-DINFL_SRC='"path"': an experiment copy of inflate.hip)
#define INFL_SRC "../snf4j_amd/csrc/inflate.hip"
#endif
#include INFL_SRC
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  FILE* f = fopen(argc > 1 ? argv[1] : "gpurun_out/infl_in.bin", "rb");
  if (!f) { printf("no input\n"); return 1; }
  const uint32_t max_lanes = argc > 2 ? (uint32_t)atoi(argv[2]) : 262144u;
  const int use_lds = argc > 3 ? atoi(argv[3]) : 1;
  const int use_order = argc > 4 ? atoi(argv[4]) : 1;
  const int pairs = argc > 5 ? atoi(argv[5]) : 0;  // 1: the split-lane decode (two lanes a frame)
  uint64_t hdr[4];  // n_frames, n_sessions, payload_len, cap per session
  if (fread(hdr, 8, 4, f) != 4) return 1;
  const uint64_t n = hdr[0], ns = hdr[1], pl = hdr[2];
  std::vector<wsg_frame_desc> desc(n);
  std::vector<uint32_t> sf(ns + 1);
  std::vector<uint8_t> payload(pl);
  if (fread(desc.data(), sizeof(wsg_frame_desc), n, f) != n) return 1;
  if (fread(sf.data(), 4, ns + 1, f) != ns + 1) return 1;
  if (fread(payload.data(), 1, pl, f) != pl) return 1;
  fclose(f);
  const uint64_t want = pairs ? 2 * n : n;
  const uint32_t lanes = (uint32_t)(want < max_lanes ? ((want + 63) / 64) * 64 : max_lanes);
  ws::InflArgs a{};
  wsg_frame_desc* d_desc;
  uint32_t *d_sf, *d_tok;
  uint8_t *d_pl, *d_lit, *d_tab;
  ws::InflTokStat* d_stat;
  CK(hipMalloc(&d_desc, n * sizeof(wsg_frame_desc)));
  CK(hipMalloc(&d_sf, (ns + 1) * 4));
  CK(hipMalloc(&d_pl, pl));
  CK(hipMalloc(&d_tok, ws::infl_tok_words(pl, n) * 4));
  CK(hipMalloc(&d_lit, ws::infl_lit_bytes(pl, n)));
  CK(hipMalloc(&d_stat, n * sizeof(ws::InflTokStat)));
  CK(hipMalloc(&d_tab, (uint64_t)lanes * ws::infl_tab_bytes()));
  CK(hipMemcpy(d_desc, desc.data(), n * sizeof(wsg_frame_desc), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_sf, sf.data(), (ns + 1) * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_pl, payload.data(), pl, hipMemcpyHostToDevice));
  const uint64_t cap = hdr[3];
  wsg_inflate_state* d_state;
  uint8_t *d_win, *d_out, *d_fast;
  wsg_frame_desc* d_odesc;
  wsg_session_result* d_res;
  uint32_t* d_rf;
  uint64_t* d_off;
  std::vector<uint64_t> ooff(ns + 1);
  for (uint64_t i = 0; i <= ns; ++i) ooff[i] = i * cap;
  CK(hipMalloc(&d_state, ns * sizeof(wsg_inflate_state)));
  CK(hipMalloc(&d_win, ns * 32768));
  CK(hipMalloc(&d_out, ns * cap));
  CK(hipMalloc(&d_fast, ns));
  CK(hipMalloc(&d_odesc, n * sizeof(wsg_frame_desc)));
  CK(hipMalloc(&d_res, ns * sizeof(wsg_session_result)));
  CK(hipMalloc(&d_rf, ns * 4));
  CK(hipMalloc(&d_off, (ns + 1) * 8));
  CK(hipMemcpy(d_off, ooff.data(), (ns + 1) * 8, hipMemcpyHostToDevice));
  a.state = d_state; a.window = d_win; a.out = d_out; a.out_off = d_off; a.out_desc = d_odesc; a.result = d_res;
  a.replay_from = d_rf; a.fast_done = d_fast;
  a.desc = d_desc; a.n_frames = n; a.session_first = d_sf; a.n_sessions = (uint32_t)ns;
  a.payload = d_pl; a.payload_len = pl;
  a.tok = d_tok; a.lit = d_lit; a.lit_len = ws::infl_lit_bytes(pl, n); a.tstat = d_stat; a.tab = d_tab; a.n_lanes = lanes;
  a.n_tab = lanes;  // (a block per lane: d_tab holds lanes tables)
  CK(hipMalloc(&a.tab_cnt, 4));
  CK(hipMemset(a.tab_cnt, 0, 4));
  a.tok_lds = use_lds;
  a.split = pairs;
  if (pairs) {
    CK(hipMalloc(&a.tok2, ws::infl_tok_words(pl, n) * 4));
    CK(hipMalloc(&a.lit2, ws::infl_lit_bytes(pl, n)));
  }
  CK(hipMalloc(&a.split_cnt, 8));
  if (use_order) {
    CK(hipMalloc(&a.order, ws::infl_ord_words(n) * 4));
    a.ord_cnt = a.order + n;
  }
  unsigned long long z[8] = {};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemcpyToSymbol(HIP_SYMBOL(ws::g_tok_prof), z, sizeof(z)));
    CK(hipEventRecord(e0));
    CK(hipMemsetAsync(a.tab_cnt, 0, 4, 0));
    CK(hipMemsetAsync(a.split_cnt, 0, 8, 0));
    ws::launch_infl_tok(a, 0);
    CK(hipEventRecord(e1));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long p[8] = {};
    CK(hipMemcpyFromSymbol(p, HIP_SYMBOL(ws::g_tok_prof), sizeof(p)));
    std::vector<ws::InflTokStat> st(n);
    CK(hipMemcpy(st.data(), d_stat, n * sizeof(ws::InflTokStat), hipMemcpyDeviceToHost));
    uint64_t ok = 0;
    for (auto& x : st) ok += x.ok != 0;
    unsigned long long nsplit = 0;
    CK(hipMemcpy(&nsplit, a.split_cnt, 8, hipMemcpyDeviceToHost));
    const double m = p[6] ? (double)p[6] : 1.0;
    // then the parallel replay of the sessions, its phase clocks
    CK(hipMemset(d_state, 0, ns * sizeof(wsg_inflate_state)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(ws::g_fast_prof), z, sizeof(z)));
    CK(hipEventRecord(e0));
    ws::launch_infl_fast(a, 0);
    CK(hipEventRecord(e1));
    CK(hipDeviceSynchronize());
    float fms = 0;
    CK(hipEventElapsedTime(&fms, e0, e1));
    unsigned long long fp[8] = {};
    CK(hipMemcpyFromSymbol(fp, HIP_SYMBOL(ws::g_fast_prof), sizeof(fp)));
    printf("fast replay %.3f ms: per session cycles: expand %.0f chase %.0f gather %.0f store %.0f total %.0f\n", fms,
           (double)fp[0] / ns, (double)fp[1] / ns, (double)fp[2] / ns, (double)fp[3] / ns, (double)fp[4] / ns);
    printf("rep %d: %.3f ms, %u lanes, %llu lane-messages, %llu ok, %llu split\n", rep, ms, lanes,
           (unsigned long long)p[6], (unsigned long long)ok, nsplit);
#ifdef SPLIT_DBG
    {
      unsigned long long g[12] = {};
      CK(hipMemcpyFromSymbol(g, HIP_SYMBOL(ws::g_split_dbg), sizeof(g)));
      printf("  split: opened %llu, not opened %llu, tail failed %llu, head quit: tail marking %llu, tail failed %llu, "
             "window unmarked %llu, block ended %llu; restarts %llu\n", g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7]);
      printf("  symbol loops (wave-level) %llu, wave iterations %.1f avg, lane steps %.1f avg per loop-lane\n", g[9],
             g[9] ? (double)g[8] / g[9] : 0.0, g[9] ? (double)g[10] / (64.0 * g[9]) : 0.0);
      unsigned long long z12[12] = {};
      CK(hipMemcpyToSymbol(HIP_SYMBOL(ws::g_split_dbg), z12, sizeof(z12)));
    }
#endif
    const char* names[8] = {"message total", "header+tables", "tables (dynamic)", "symbol loop", "steps", "blocks", "messages", "lds bail-outs"};
    for (int i = 0; i < 8; ++i) printf("  %-18s %12.1f per message%s\n", names[i], (double)p[i] / m, i < 4 ? " cycles" : "");
  }
  return 0;
}
