#!/bin/bash
# Round 5, run aa: the encode batcher's streams on hardware queues of their own (CU-mask
# streams: enccum) against the current build, through scripts/seq_probe.py (the
# encode line alone, then after the stage line, where the runtime's placement of its
# streams on hardware queues had cost it a quarter).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in cur enccum cur enccum; do
  echo "== $lib"
  WSG_LIB=snf4j_amd/_ab/libwsgpu_$lib.so timeout -k 10 300 python scripts/seq_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/r05aa_ab_encprio.txt
echo R05AA_DONE
