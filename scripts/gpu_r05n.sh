#!/bin/bash
# Round 5, run n: flushes in flight (3, 4) x the two-phase inflate's pre-decode
# contexts (2, 3) on the burst / steady stage lines; the stage tests on the 3-context
# builds first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in d3t3 d4t3; do
  WSG_LIB=snf4j_amd/_ab/libwsgpu_$lib.so timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py \
    tests/test_gpu_loop.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05n_tests_$lib.log 2>&1
  rc=$?; tail -2 gpurun_out/r05n_tests_$lib.log; [ $rc -eq 0 ] || exit $rc
done
for round in 1 2 3; do
  for cfg in "d3t2 3" "d3t3 3" "d4t2 4" "d4t3 4"; do
    set -- $cfg
    for line in e2e_stages e2e_stages_steady; do
      WSG_LIB=snf4j_amd/_ab/libwsgpu_$1.so WSG_BENCH_INFLIGHT=$2 timeout -k 10 240 python bench.py --only $line \
        --extra-steps 3 > gpurun_out/abst.json 2> gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('$line $1', d['value'], d.get('ms_per_batch'), d.get('feed_ms'), d.get('wait_ms'))"
    done
  done
done | tee gpurun_out/r05n_ab_depth_tokctx.txt
echo R05N_DONE
