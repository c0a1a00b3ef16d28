mkdir -p gpurun_out
timeout -k 10 120 tools/bin/ubench_d2h > gpurun_out/r06g_d2h.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --only e2e_stages --extra-steps 5 > gpurun_out/r06g_stages.json 2>gpurun_out/r06g.err || exit 1
timeout -k 10 400 python -u bench.py --only e2e_stages_multi --extra-steps 5 > gpurun_out/r06g_multi.json 2>>gpurun_out/r06g.err || exit 1
timeout -k 10 400 python -u bench.py --only deflate --extra-steps 5 > gpurun_out/r06g_deflate.json 2>>gpurun_out/r06g.err || exit 1
