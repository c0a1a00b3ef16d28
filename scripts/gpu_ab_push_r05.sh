cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_jni.py tests/test_gpu_loop.py tests/test_gpu_session.py \
  -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05ao_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05ao_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_stages.sh snf4j_amd/_ab/libwsgpu_rtd2h.so snf4j_amd/_ab/libwsgpu_push.so | tee gpurun_out/r05ao_ab_push.txt || exit 1
bash scripts/gpu_stageprof.sh r05ao > /dev/null 2>&1; grep "stage prof" gpurun_out/r05ao_stageprof.err | head -20
