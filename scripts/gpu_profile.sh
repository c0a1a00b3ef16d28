#!/bin/bash
# rocprofv3 evidence for the bench workload: kernel trace + stats, then one PMC
# pass per counter group (FETCH_SIZE and WRITE_SIZE do not fit one pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-extras $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o fetch --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras $* > gpurun_out/prof_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o write --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras $* > gpurun_out/prof_write.log 2>&1 || exit $?
find gpurun_out/prof_kt gpurun_out/prof_fetch gpurun_out/prof_write -type f | head -20
