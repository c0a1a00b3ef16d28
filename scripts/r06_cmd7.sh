mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_deflate.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r06zg_deflate.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --only deflate --extra-steps 5 > gpurun_out/r06zg_deflate.json 2>gpurun_out/r06zg.err || exit 1
