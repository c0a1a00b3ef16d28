# same-box A/B of the deflate line: symbol ring, emit width, link batch, half-wave parse
mkdir -p gpurun_out
bash scripts/ab_line.sh deflate snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_ring64.so snf4j_amd/_ab/libwsgpu_ring48.so snf4j_amd/_ab/libwsgpu_emit512.so snf4j_amd/_ab/libwsgpu_lb12.so snf4j_amd/_ab/libwsgpu_pt32.so > gpurun_out/r06za_ab_deflate.txt 2>&1 || exit 1
echo done
