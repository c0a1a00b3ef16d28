#!/bin/bash
# session search from an interpolated guess (WSG_SESSION_GUESS): decode / aggregate /
# encode / validate / mixed GPU tests, then same-box A/B of the headline, configs[1] and
# the aggregator line against the plain binary search (libwsgpu_sg0.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_aggregate.py tests/test_gpu_encode.py tests/test_gpu_validate.py tests/test_gpu_mixed.py tests/test_gpu_scan_chunks.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r04_sguess_tests.log 2>&1 || { tail -30 gpurun_out/r04_sguess_tests.log; exit 1; }
tail -1 gpurun_out/r04_sguess_tests.log
echo "# headline"; bash scripts/ab_lib.sh snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_sg0.so || exit 1
echo "# configs1"; bash scripts/ab_line.sh configs1 snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_sg0.so || exit 1
echo "# configs2 (aggregator)"; bash scripts/ab_line.sh configs2 snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_sg0.so
