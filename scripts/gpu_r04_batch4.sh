#!/bin/bash
# Round-4 batch 4: the stage chain begun in the previous flush's wait (inflate overlapping
# the caller's feeds): tests of the batcher paths, then same-box A/B against the previous
# build (stprev) on both stage lines, then the stage-phase profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_jni.py tests/test_gpu_loop.py \
  tests/test_gpu_decode.py tests/test_gpu_inflate.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04e_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04e_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do for lib in snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_stprev.so; do
  for line in e2e_stages e2e_aggregate; do
    WSG_LIB=$lib timeout -k 10 240 python bench.py --only $line --extra-steps 3 > gpurun_out/abw.json 2>gpurun_out/abw.err || { tail -5 gpurun_out/abw.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abw.json'));print('$line', '$(basename $lib)', d['value'], d.get('ms_per_batch'), d.get('feed_ms'), d.get('wait_ms'))"
  done
done; done | tee gpurun_out/r04_ab_stagebegin.txt
WSG_LIB=snf4j_amd/_ab/libwsgpu_stageprof.so timeout -k 10 240 python bench.py --only e2e_stages --extra-steps 3 \
  > gpurun_out/stageprof.json 2> gpurun_out/stageprof.err || exit 1
grep "stage prof" gpurun_out/stageprof.err | head -20
echo BATCH_DONE
