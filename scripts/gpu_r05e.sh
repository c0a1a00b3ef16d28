#!/bin/bash
# Round 5, run e: three flushes in flight (each wait collects the next flush's chain and
# begins the one after): tests, then the stage and decode lines, interleaved against the
# begin-one-early build with two in flight, and the stage profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_jni.py tests/test_gpu_loop.py \
  tests/test_gpu_session.py tests/test_gpu_decode.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r05e_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05e_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  for cfg in "async2 2" "cur 2" "cur 3"; do
    set -- $cfg
    WSG_LIB=snf4j_amd/_ab/libwsgpu_$1.so WSG_BENCH_INFLIGHT=$2 timeout -k 10 240 python bench.py --only e2e_stages \
      --extra-steps 3 > gpurun_out/abst.json 2> gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('stages $1 depth $2', d['value'], d['ms_per_batch'], d.get('feed_ms'), d.get('wait_ms'))"
  done
done | tee gpurun_out/r05e_ab_stages_depth.txt
for round in 1 2; do
  for cfg in "async2 2" "cur 3"; do
    set -- $cfg
    WSG_LIB=snf4j_amd/_ab/libwsgpu_$1.so WSG_BENCH_INFLIGHT=$2 timeout -k 10 300 python bench.py --steps 5 --warmup 2 \
      --no-extras --no-cpu-baseline --e2e > gpurun_out/abe2e.json 2> gpurun_out/abe2e.err || { tail -5 gpurun_out/abe2e.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abe2e.json'));e=d['e2e_pinned'];print('e2e $1 depth $2', e['native_batcher']['GiB_per_s'], e['drop_in_loop']['GiB_per_s'], e.get('native_batcher_stages',{}).get('value'))"
  done
done | tee gpurun_out/r05e_ab_e2e_depth.txt
bash scripts/gpu_stageprof.sh r05e || exit 1
echo R05E_DONE
