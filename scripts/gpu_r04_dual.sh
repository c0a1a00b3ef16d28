#!/bin/bash
# Round-4: the lane decoder's two-literal step — inflate parity tests, then same-box A/B of the
# inflate and stage lines against the previous build (tokprev).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_stages.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04f_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do for lib in snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_tokprev.so; do
  WSG_LIB=$lib timeout -k 10 240 python bench.py --inflate-only --extra-steps 5 > gpurun_out/abin.json 2>gpurun_out/abin.err || { tail -5 gpurun_out/abin.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abin.json'));print('inflate', '$(basename $lib)', d['value'], d['roofline']['avg_launch_ms'], d.get('pipeline_ms'))"
  WSG_LIB=$lib timeout -k 10 240 python bench.py --only e2e_stages --extra-steps 3 > gpurun_out/abw.json 2>gpurun_out/abw.err || { tail -5 gpurun_out/abw.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abw.json'));print('e2e_stages', '$(basename $lib)', d['value'], d.get('ms_per_batch'))"
done; done | tee gpurun_out/r04_ab_dual.txt
echo BATCH_DONE
