#!/bin/bash
# GPU validation pass: parity tests, smoke, the N=2 launcher rehearsal, bench.
# Every GPU step has its own time limit; the script stops at the first failure.
#   scripts/gpu_check.sh [quick]   (quick: no full bench)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "--- $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  return $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread || exit $?
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
# N=2 through bench.py's own launcher, both ranks on device 0 (a rehearsal, not a number)
WSG_BENCH_ONE_DEVICE=1 step bench_n2_rehearsal 300 python bench.py --gpus 2 --frames 262144 --steps 5 --warmup 2 --cpu-seconds 2 || exit $?
step bench_config3 300 python bench.py --config 3 --steps 5 --warmup 2 --no-extras --no-cpu-baseline || exit $?
[ "$1" = quick ] && { echo ALL_DONE; exit 0; }
step bench 600 python bench.py --e2e || exit $?
echo ALL_DONE
