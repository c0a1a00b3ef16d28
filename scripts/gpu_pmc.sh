#!/bin/bash
# rocprofv3 evidence for one bench invocation:
#   scripts/gpu_pmc.sh TAG [bench args...]
# kernel trace + stats, then one PMC pass per counter group (FETCH_SIZE and
# WRITE_SIZE do not fit one pass; at most 8 SQ counters a pass).  Every pass has
# its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/prof/$tag
mkdir -p "$out"
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --extra-steps 5 $*"
PARGS="--steps 3 --warmup 1 --no-cpu-baseline --extra-steps 2 $*"
run() {  # run <name> <rocprofv3 args...>
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 "$@" -d "$out/$name" -o "$name" --output-format csv -- python3 bench.py $PARGS \
    > "$out/$name.log" 2>&1 || { echo "pass $name failed"; tail -5 "$out/$name.log"; exit 1; }
}
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$out/kt" -o kt --output-format csv -- python3 bench.py $ARGS \
  > "$out/kt.log" 2>&1 || { echo "kernel trace failed"; tail -5 "$out/kt.log"; exit 1; }
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sq2 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH
echo "profiled $tag"
