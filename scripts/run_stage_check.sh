mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_decode.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_stages.log 2>&1; rc=$?; tail -5 gpurun_out/t_stages.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --only e2e_stages --extra-steps 3 > gpurun_out/e2e_stages_after.log 2>&1; rc=$?; tail -2 gpurun_out/e2e_stages_after.log; exit $rc
