#!/bin/bash
# Round 5, run ad: the encode batcher's kernels writing the wire straight into pinned
# host memory (encdirect: no runtime D2H) — encode tests, then scripts/seq_probe.py
# (the encode line alone and after the stage line) against the current build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WSG_LIB=snf4j_amd/_ab/libwsgpu_encdirect.so timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_jni.py \
  tests/test_gpu_loop.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05ad_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05ad_tests.log; [ $rc -eq 0 ] || exit $rc
for lib in cur encdirect cur encdirect; do
  echo "== $lib"
  WSG_LIB=snf4j_amd/_ab/libwsgpu_$lib.so timeout -k 10 300 python scripts/seq_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/r05ad_ab_encdirect.txt
echo R05AD_DONE
