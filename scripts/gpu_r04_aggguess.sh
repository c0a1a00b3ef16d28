#!/bin/bash
# the aggregator plan's session search from an interpolated guess (k_agg_a, WSG_SESSION_GUESS=1
# in aggregate.hip): aggregator GPU tests on it, then a same-box A/B on the aggregator line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
WSG_LIB=snf4j_amd/_ab/libwsgpu_ag1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_aggregate.py tests/test_gpu_stages.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04_ag1_tests.log 2>&1 || { tail -20 gpurun_out/r04_ag1_tests.log; exit 1; }
tail -1 gpurun_out/r04_ag1_tests.log
bash scripts/ab_agg.sh snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_ag1.so
