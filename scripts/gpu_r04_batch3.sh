#!/bin/bash
# Round-4 batch 3: tests after the stage-worker revert; same-box A/B of the stage chain in
# wsg_batcher_wait (default) against the worker-thread build (stworker) on both stage lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_jni.py tests/test_gpu_loop.py \
  tests/test_gpu_decode.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04d_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do for lib in snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_stworker.so; do
  for line in e2e_stages e2e_aggregate; do
    WSG_LIB=$lib timeout -k 10 240 python bench.py --only $line --extra-steps 3 > gpurun_out/abw.json 2>gpurun_out/abw.err || { tail -5 gpurun_out/abw.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abw.json'));print('$line', '$(basename $lib)', d['value'], d.get('ms_per_batch'), d.get('feed_ms'), d.get('wait_ms'))"
  done
done; done | tee gpurun_out/r04_ab_stageworker2.txt
echo BATCH_DONE
