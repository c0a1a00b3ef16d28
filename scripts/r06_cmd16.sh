# deferred refills: committed (immediate) against 16 / 24 / 32 idle lanes, same box
mkdir -p gpurun_out
bash scripts/ab_line.sh deflate snf4j_amd/_ab/libwsgpu_cmt.so snf4j_amd/_ab/libwsgpu_rf16.so snf4j_amd/_ab/libwsgpu_rf24.so snf4j_amd/_ab/libwsgpu_rf32.so > gpurun_out/r06ze_ab_refill.txt 2>&1 || exit 1
echo done
