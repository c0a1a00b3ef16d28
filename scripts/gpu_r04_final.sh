#!/bin/bash
# Round-4 closing run, part 1: the GPU test suite, smoke(), the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/r04_final_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r04_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r04_bench_full.json 2> gpurun_out/r04_bench_full.err
rc=$?; tail -c 600 gpurun_out/r04_bench_full.json; exit $rc
