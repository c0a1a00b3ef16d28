#!/bin/bash
# Round 5, run d: the asynchronous stage chain (next flush's inflate begun in the
# previous wait): its tests, a same-box A/B against the synchronous chain, the
# split-lane decode on stage-sized launches, and the stage profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/ab_batch.sh r05d "tests/test_gpu_stages.py tests/test_gpu_inflate.py tests/test_gpu_jni.py tests/test_gpu_loop.py tests/test_gpu_session.py" \
  ab_stages.sh stages_async snf4j_amd/_ab/libwsgpu_stsync.so snf4j_amd/_ab/libwsgpu_cur.so -- || exit 1
bash scripts/ab_env.sh WSG_TUNE_INFLATE_SPLIT "0 1" "d['value'], d['ms_per_batch'], d['wait_ms']" --only e2e_stages \
  > gpurun_out/r05d_ab_split_stages.txt 2>&1 || { tail -5 gpurun_out/r05d_ab_split_stages.txt; exit 1; }
cat gpurun_out/r05d_ab_split_stages.txt
bash scripts/gpu_stageprof.sh r05d || exit 1
echo R05D_DONE
