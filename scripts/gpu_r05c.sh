#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/ab_batch.sh r05c - ab_line.sh "inflate_tok" inflate snf4j_amd/_ab/libwsgpu_tokold.so snf4j_amd/_ab/libwsgpu_cur.so -- \
  ab_stages.sh "stages_tok" snf4j_amd/_ab/libwsgpu_tokold.so snf4j_amd/_ab/libwsgpu_cur.so -- || exit 1
for lib in tokold cur; do
  (cd /tmp && WSG_LIB=$GRAFT_REPO_ROOT/snf4j_amd/_ab/libwsgpu_$lib.so timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/r05c_w_$lib -o w --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --only inflate --steps 3 --warmup 1 --no-cpu-baseline --extra-steps 2 > $GRAFT_REPO_ROOT/gpurun_out/r05c_w_$lib.log 2>&1) || { echo "pmc $lib failed"; exit 1; }
done
bash scripts/gpu_stageprof.sh r05c || exit 1
echo R05C_DONE
