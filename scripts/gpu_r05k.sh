#!/bin/bash
# Round 5, run k: lazy stage collection (WSG_STAGE_LAZY: wsg_batcher_wait blocks on its
# own flush only; flush_async collects a finished chain and begins the next) — its
# stage tests, then the burst and steady stage lines and the aggregate line against
# the eager build, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WSG_LIB=snf4j_amd/_ab/libwsgpu_lazy.so timeout -k 10 900 python -u -m pytest tests/test_gpu_stages.py \
  tests/test_gpu_loop.py tests/test_gpu_session.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r05k_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05k_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  for lib in early lazy; do
    for line in e2e_stages e2e_stages_steady; do
      WSG_LIB=snf4j_amd/_ab/libwsgpu_$lib.so timeout -k 10 240 python bench.py --only $line \
        --extra-steps 3 > gpurun_out/abst.json 2> gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('$line $lib', d['value'], d['ms_per_batch'], d.get('feed_ms'), d.get('wait_ms'))"
    done
  done
done | tee gpurun_out/r05k_ab_lazy.txt
echo R05K_DONE
