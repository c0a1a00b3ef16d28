#!/bin/bash
# validator by LDS-DMA (k_vpieces_lds): the validator / decode GPU tests on the new build,
# then a same-box A/B of the validator line against the register-load kernel (WSG_VLDS=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_validate.py tests/test_gpu_stages.py tests/test_gpu_inflate.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r04_vlds_tests.log 2>&1 || { tail -30 gpurun_out/r04_vlds_tests.log; exit 1; }
tail -1 gpurun_out/r04_vlds_tests.log
bash scripts/ab_line.sh validator snf4j_amd/libwsgpu.so "$@"
