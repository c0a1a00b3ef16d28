#!/bin/bash
# Round-4: the stage output gather with 16-B stores for unaligned sources (current), against
# the dword version (cpprev) and 24 workgroups (cp24): stage tests, then same-box A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_jni.py -x -q -p no:cacheprovider --timeout 200 \
  --timeout-method thread > gpurun_out/r04k_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04k_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do for lib in snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_cpprev.so snf4j_amd/_ab/libwsgpu_cp24.so; do
  for line in e2e_stages e2e_aggregate; do
    WSG_LIB=$lib timeout -k 10 240 python bench.py --only $line --extra-steps 3 > gpurun_out/abw.json 2>gpurun_out/abw.err || { tail -5 gpurun_out/abw.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abw.json'));print('$line', '$(basename $lib)', d['value'], d.get('ms_per_batch'))"
  done
done; done | tee gpurun_out/r04_ab_stagecopy.txt
echo BATCH_DONE
