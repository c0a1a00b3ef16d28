# validator-bound experiments: dispatch floor and read stream at the
# validator's grid shape, then the validator line with 4 / 8 / 16 KiB a wave (same box)
mkdir -p gpurun_out
timeout -k 10 120 tools/bin/ubench_grid > gpurun_out/r06h_grid.jsonl 2>&1 || exit 1
bash scripts/ab_line.sh validator snf4j_amd/libwsgpu.so snf4j_amd/_ab/libwsgpu_vp8.so snf4j_amd/_ab/libwsgpu_vp16.so > gpurun_out/r06h_ab_validator.txt 2>&1 || exit 1
