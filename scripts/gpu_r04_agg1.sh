#!/bin/bash
# Round-4: the single-pass aggregator plan (k_agg_plan1) — the release cost microbenchmark,
# aggregator parity with both plans, then same-box A/B of WSG_TUNE_AGG_PLAN on configs[2].
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 tools/ubench_release 2128 | tee gpurun_out/r04_ubench_release.txt || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_aggregate.py -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/r04g_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04g_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_env.sh WSG_TUNE_AGG_PLAN "0 1" "(d['aggregate']['value'], {k:v for k,v in d['aggregate'].get('pipeline_ms',{}).items() if 'agg' in k})" --only configs2 \
  | tee gpurun_out/r04_ab_aggplan1.txt
echo BATCH_DONE
