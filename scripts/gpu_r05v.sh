#!/bin/bash
# Round 5, run v: the download stream at high priority (now the default) with the stage
# context's stream at high priority too (stprio), stage tests on both, then the burst /
# steady / aggregator stage lines interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_jni.py tests/test_gpu_loop.py \
  tests/test_gpu_session.py tests/test_gpu_aggregate.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r05v_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05v_tests.log; [ $rc -eq 0 ] || exit $rc
WSG_LIB=snf4j_amd/_ab/libwsgpu_stprio.so timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py \
  -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05v_tests_stprio.log 2>&1
rc=$?; tail -2 gpurun_out/r05v_tests_stprio.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  for lib in sprio stprio; do
    for line in e2e_stages e2e_stages_steady e2e_aggregate; do
      WSG_LIB=snf4j_amd/_ab/libwsgpu_$lib.so timeout -k 10 240 python bench.py --only $line \
        --extra-steps 3 > gpurun_out/abst.json 2> gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('$line $lib', d['value'], d.get('ms_per_batch'), d.get('feed_ms'), d.get('wait_ms'))"
    done
  done
done | tee gpurun_out/r05v_ab_stprio.txt
echo R05V_DONE
