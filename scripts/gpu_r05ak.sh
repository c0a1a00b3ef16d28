#!/bin/bash
# Round 5, run ak: the lane decoder refilling its bit buffer to 57-64 bits every step
# (WSG_TOK_EAGER=1, k_infl_tok) — inflate + stage tests on it, then the inflate line
# and the burst / steady stage lines against the current build, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WSG_LIB=snf4j_amd/_ab/libwsgpu_eager.so timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_stages.py \
  -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05ak_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05ak_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  for lib in cur eager; do
    WSG_LIB=snf4j_amd/_ab/libwsgpu_$lib.so timeout -k 10 240 python bench.py --only inflate --extra-steps 10 \
      > gpurun_out/abin.json 2> gpurun_out/abin.err || { tail -5 gpurun_out/abin.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abin.json'));print('inflate $lib', d['value'], d['ms_per_step'], d.get('pipeline_ms'))"
    for line in e2e_stages e2e_stages_steady; do
      WSG_LIB=snf4j_amd/_ab/libwsgpu_$lib.so timeout -k 10 240 python bench.py --only $line \
        --extra-steps 3 > gpurun_out/abst.json 2> gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('$line $lib', d['value'], d.get('ms_per_batch'))"
    done
  done
done | tee gpurun_out/r05ak_ab_eager.txt
echo R05AJ_DONE
