#!/bin/bash
# Round-4: decode parse/link blocks of 512 frames (WSG_DBLOCK) — parity of that build, then
# same-box A/B of the headline and the validator line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WSG_LIB=snf4j_amd/_ab/libwsgpu_db512.so timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_validate.py \
  tests/test_gpu_mixed.py tests/test_gpu_scan_chunks.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04j_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04j_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_lib.sh snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_db512.so > gpurun_out/r04_ab_dblock.txt 2>&1 || { cat gpurun_out/r04_ab_dblock.txt; exit 1; }
cat gpurun_out/r04_ab_dblock.txt
bash scripts/ab_line.sh validator snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_db512.so > gpurun_out/r04_ab_dblock_val.txt 2>&1 || { cat gpurun_out/r04_ab_dblock_val.txt; exit 1; }
cat gpurun_out/r04_ab_dblock_val.txt
echo BATCH_DONE
