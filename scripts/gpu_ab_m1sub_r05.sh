#!/bin/bash
# Round 5: the one-step match through the distance sub-tables too (WSG_TOK_MATCH1_SUB=1)
# — inflate + stage tests on it, then the inflate line against the current build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WSG_LIB=snf4j_amd/_ab/libwsgpu_m1sub.so timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_stages.py \
  -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05ar_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05ar_tests.log; [ $rc -eq 0 ] || exit $rc
LINES=inflate bash scripts/ab_stages.sh snf4j_amd/_ab/libwsgpu_cur.so snf4j_amd/_ab/libwsgpu_m1sub.so | tee gpurun_out/r05ar_ab_m1sub.txt
