#!/bin/bash
# Round 5, run ai: the stage output laid out on the device (k_stage_layout) and its
# gather queued right behind the validator, against the host-laid-out build
# (WSG_AB_NO_DEV_LAYOUT): stage tests first, then the burst / steady stage lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_jni.py tests/test_gpu_loop.py \
  tests/test_gpu_session.py tests/test_gpu_aggregate.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r05ai_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05ai_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  for lib in nodevlay devlay; do
    for line in e2e_stages e2e_stages_steady; do
      WSG_LIB=snf4j_amd/_ab/libwsgpu_$lib.so timeout -k 10 240 python bench.py --only $line \
        --extra-steps 3 > gpurun_out/abst.json 2> gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('$line $lib', d['value'], d.get('ms_per_batch'), d.get('feed_ms'), d.get('wait_ms'))"
    done
  done
done | tee gpurun_out/r05ai_ab_devlayout.txt
echo R05AI_DONE
