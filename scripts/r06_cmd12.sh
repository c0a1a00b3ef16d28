# branch-light parse: deflate tests, then same-box A/B of the deflate line against variants
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_deflate.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r06z_deflate.log 2>&1 || { tail -5 gpurun_out/r06z_deflate.log; exit 1; }
bash scripts/ab_line.sh deflate snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_pold.so snf4j_amd/_ab/libwsgpu_lb4.so snf4j_amd/_ab/libwsgpu_emit128.so snf4j_amd/_ab/libwsgpu_ring16.so > gpurun_out/r06z_ab_deflate.txt 2>&1 || exit 1
echo done
