#!/bin/bash
# Round-4 split-lane inflate: parity tests, then same-box A/Bs of WSG_TUNE_INFLATE_SPLIT
# (0: a lane a message, 1: auto) on the stage-chain line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_stages.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/r04s_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04s_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do for v in 0 1; do
  WSG_TUNE_INFLATE_SPLIT=$v timeout -k 10 240 python bench.py --only e2e_stages --extra-steps 3 > gpurun_out/abst.json 2>gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('stages split=$v', d['value'], d['ms_per_batch'], d.get('feed_ms'), d.get('wait_ms'))"
done; done | tee gpurun_out/r04_ab_split_stages.txt
echo SPLIT_DONE
