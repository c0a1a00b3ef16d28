#!/bin/bash
# The stage chain's per-flush host phases (a WSG_STAGE_PROF build: scripts/build_variant.sh
# stageprof batcher.hip -DWSG_STAGE_PROF) and its device timeline (rocprofv3 kernel +
# memory-copy trace of the e2e_stages line, summarised by tools/rocpd_stats.py).
#   scripts/gpu_stageprof.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05}
WSG_LIB=snf4j_amd/_ab/libwsgpu_stageprof.so timeout -k 10 240 python bench.py --only e2e_stages --extra-steps 3 \
  > gpurun_out/${tag}_stageprof.json 2> gpurun_out/${tag}_stageprof.err || exit 1
grep "stage prof" gpurun_out/${tag}_stageprof.err | head -20
cat gpurun_out/${tag}_stageprof.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof_st -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --only e2e_stages --extra-steps 2 > $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof_st.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && db=$(find gpurun_out/${tag}_prof_st -name '*.db' | head -1) && \
  python tools/rocpd_stats.py "$db" > gpurun_out/${tag}_stage_kernels.txt && cat gpurun_out/${tag}_stage_kernels.txt
echo DONE
