mkdir -p gpurun_out
bash scripts/ab_line.sh validator snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_vp2.so snf4j_amd/_ab/libwsgpu_vminw6.so snf4j_amd/_ab/libwsgpu_vminw8.so > gpurun_out/r06h_ab_validator2.txt 2>&1 || exit 1
