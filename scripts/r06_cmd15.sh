# deferred refills in the LDS walk: deflate tests on the default (8), then the same-box A/B
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_deflate.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r06zd_deflate.log 2>&1 || { tail -5 gpurun_out/r06zd_deflate.log; exit 1; }
bash scripts/ab_line.sh deflate snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_rf1.so snf4j_amd/_ab/libwsgpu_rf4.so snf4j_amd/_ab/libwsgpu_rf16.so > gpurun_out/r06zd_ab_refill.txt 2>&1 || exit 1
echo done
