#!/bin/bash
# k_infl_fast row-resolved expansion: inflate GPU tests, then same-box A/B against the
# thread-per-token expansion (WSG_FAST_XSCAN=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r04_xscan_tests.log 2>&1 || { tail -30 gpurun_out/r04_xscan_tests.log; exit 1; }
tail -3 gpurun_out/r04_xscan_tests.log
bash scripts/ab_line.sh inflate snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_bg0.so snf4j_amd/_ab/libwsgpu_xs0.so
