#!/bin/bash
# Round 5, run f: two-phase inflate in the stage chain (a flush's pre-decode on its own
# context, ahead of the previous flush's replay): tests, the stage line at two and
# three flushes in flight against the round-5 run-d build, the stage profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_inflate.py tests/test_gpu_jni.py \
  tests/test_gpu_loop.py tests/test_gpu_session.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r05f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05f_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  for cfg in "async2 2" "cur 2" "cur 3"; do
    set -- $cfg
    WSG_LIB=snf4j_amd/_ab/libwsgpu_$1.so WSG_BENCH_INFLIGHT=$2 timeout -k 10 240 python bench.py --only e2e_stages \
      --extra-steps 3 > gpurun_out/abst.json 2> gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('stages $1 depth $2', d['value'], d['ms_per_batch'], d.get('feed_ms'), d.get('wait_ms'))"
  done
done | tee gpurun_out/r05f_ab_stages.txt
bash scripts/gpu_stageprof.sh r05f || exit 1
echo R05F_DONE
