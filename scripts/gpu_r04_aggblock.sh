#!/bin/bash
# Round-4: the aggregator plan's frames per block (WSG_AGG_BLOCK 256 / 512 / 1024): parity of
# each build, then same-box A/B on configs[2].
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in snf4j_amd/_ab/libwsgpu_ab512.so snf4j_amd/_ab/libwsgpu_ab1024.so; do
  WSG_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_aggregate.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/r04h_tests.log 2>&1
  rc=$?; echo "$lib tests rc=$rc"; tail -2 gpurun_out/r04h_tests.log; [ $rc -eq 0 ] || exit $rc
done
bash scripts/ab_agg.sh snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_ab512.so snf4j_amd/_ab/libwsgpu_ab1024.so > gpurun_out/r04_ab_aggblock.txt 2>&1 || { cat gpurun_out/r04_ab_aggblock.txt; exit 1; }
cat gpurun_out/r04_ab_aggblock.txt
echo BATCH_DONE
