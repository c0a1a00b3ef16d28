#!/bin/bash
# Diagnostic binaries for k_inflate (phase clocks and a plain runner for counters).
set -e
cd "$(dirname "$0")/.."
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Isnf4j_amd/csrc"
$H tools/prof_inflate.hip -o tools/prof_inflate
$H -DNO_PROF tools/prof_inflate.hip -o tools/run_inflate
$H tools/prof_infl_tok.hip -o tools/prof_infl_tok
[ -n "$TOK_EXP" ] && $H $TOK_EXP tools/prof_infl_tok.hip -o tools/prof_infl_tok_exp
