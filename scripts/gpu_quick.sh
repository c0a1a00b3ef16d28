#!/bin/bash
# Quick GPU pass during development: given pytest files, then bench.py --only lines.
#   scripts/gpu_quick.sh "tests/test_a.py tests/test_b.py" "inflate e2e_stages"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$1" ]; then
  timeout -k 10 600 python -u -m pytest $1 -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/quick_tests.log 2>&1
  rc=$?; tail -4 gpurun_out/quick_tests.log; [ $rc = 0 ] || exit $rc
fi
for l in $2; do
  timeout -k 10 300 python bench.py --only $l --extra-steps ${STEPS:-5} > gpurun_out/quick_$l.log 2>&1
  rc=$?; tail -1 gpurun_out/quick_$l.log | cut -c1-900; [ $rc = 0 ] || exit $rc
done
echo QUICK_DONE
