#!/bin/bash
# k_infl_fast variants after the row-resolved expansion: tokens a thread a round (TPT) and
# a branch-free chase; inflate GPU tests on each variant first, then a same-box A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in snf4j_amd/libwsgpu.so "$@"; do
  WSG_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r04_xscan_tests.log 2>&1 || { echo "$lib"; tail -30 gpurun_out/r04_xscan_tests.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/r04_xscan_tests.log)"
done
bash scripts/ab_line.sh inflate snf4j_amd/libwsgpu.so "$@"
