#!/bin/bash
# GPU validation pass: parity tests, smoke, bench.  Every GPU step has its own
# time limit; the script stops at the first fault/abort/timeout (exit >= 2 or signal).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "--- $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  return $rc
}
step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider; rc=$?; ok $rc || exit $rc
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; ok $rc || exit $rc
step bench_small 300 python bench.py --frames 262144 --steps 5 --warmup 2 --no-cpu-baseline; rc=$?; ok $rc || exit $rc
step bench 600 python bench.py --e2e; rc=$?; ok $rc || exit $rc
echo ALL_DONE
