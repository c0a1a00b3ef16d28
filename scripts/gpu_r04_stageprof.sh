#!/bin/bash
# The stage chain's per-flush host phases (WSG_STAGE_PROF build) and its device timeline
# (rocprofv3 kernel + memory-copy trace of the e2e_stages line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WSG_LIB=snf4j_amd/_ab/libwsgpu_stageprof.so timeout -k 10 240 python bench.py --only e2e_stages --extra-steps 3 \
  > gpurun_out/stageprof.json 2> gpurun_out/stageprof.err || exit 1
grep "stage prof" gpurun_out/stageprof.err | head -20
cat gpurun_out/stageprof.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_st -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --only e2e_stages --extra-steps 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_st.log 2>&1 || exit 1
echo DONE
