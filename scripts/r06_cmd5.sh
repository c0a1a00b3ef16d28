mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_deflate.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r06i_deflate.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --only deflate --extra-steps 5 > gpurun_out/r06i_deflate.json 2>gpurun_out/r06i.err || exit 1
bash scripts/ab_line.sh validator snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_vp2.so snf4j_amd/_ab/libwsgpu_vminw6.so snf4j_amd/_ab/libwsgpu_vminw8.so > gpurun_out/r06h_ab_validator2.txt 2>&1 || exit 1
