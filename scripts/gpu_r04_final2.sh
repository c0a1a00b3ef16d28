#!/bin/bash
# Round-4 closing run after the replay rework: GPU tests, smoke(), the default bench line,
# and the inflate line's rocprofv3 kernel stats + PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_r04_final.sh || exit 1
bash scripts/gpu_profiles.sh r04z inflate
