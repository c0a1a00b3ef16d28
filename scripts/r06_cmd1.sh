mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_encode.py tests/test_gpu_stages.py tests/test_gpu_loop.py tests/test_gpu_session.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r06f_encdefl.log 2>&1 || exit 1
for fs in 1 0 1 0; do WSG_TUNE_FUSED_SCAN=$fs timeout -k 10 200 python -u bench.py --no-extras --no-e2e --no-cpu-baseline --steps 20 > gpurun_out/r06f_north_fs$fs.json 2>>gpurun_out/r06f_north.err || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06f_north_fs$fs.json; done
