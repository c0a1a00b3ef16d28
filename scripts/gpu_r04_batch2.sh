#!/bin/bash
# Round-4 batch 2: tests of the changed paths, aggregator fold bound A/B (3072 vs round 3's
# 2048), stage-worker blocking vs spinning event waits A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_aggregate.py tests/test_gpu_stages.py tests/test_gpu_jni.py \
  tests/test_gpu_loop.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04c_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_agg.sh snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_agg2048.so > gpurun_out/r04_ab_aggfold3072.txt 2>&1 || exit 1
cat gpurun_out/r04_ab_aggfold3072.txt
bash scripts/ab_stages.sh snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_stspin.so > gpurun_out/r04_ab_stageblocking.txt 2>&1 || exit 1
cat gpurun_out/r04_ab_stageblocking.txt
WSG_LIB=snf4j_amd/_ab/libwsgpu_stageprof.so timeout -k 10 240 python bench.py --only e2e_stages --extra-steps 3 \
  > gpurun_out/stageprof.json 2> gpurun_out/stageprof.err || exit 1
grep "stage prof" gpurun_out/stageprof.err | head -20
echo BATCH_DONE
