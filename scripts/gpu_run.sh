#!/bin/bash
# A GPU pass: parity tests, smoke, the default bench line (each step time-limited,
# stops at the first failure).  scripts/gpu_run.sh <tag> [tests-only|bench-only]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-run}
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_$name.log" 2>&1
  local rc=$?
  echo "--- $name rc=$rc"; tail -n 15 "gpurun_out/${tag}_$name.log"
  return $rc
}
if [ "$2" != bench-only ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread || exit $?
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
[ "$2" = tests-only ] && { echo ALL_DONE; exit 0; }
step bench 600 python bench.py || exit $?
echo ALL_DONE
