# PMC of the deflate line's kernels (issue counters)
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
out=gpurun_out/prof/r06_dl4; mkdir -p $out
A="--steps 3 --warmup 1 --no-cpu-baseline --extra-steps 2 --only deflate"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $out/sq1 -o sq1 --output-format csv -- python3 bench.py $A > $out/sq1.log 2>&1 || { echo sq1 failed; tail -3 $out/sq1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH -d $out/sq2 -o sq2 --output-format csv -- python3 bench.py $A > $out/sq2.log 2>&1 || { echo sq2 failed; tail -3 $out/sq2.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR -d $out/sq3 -o sq3 --output-format csv -- python3 bench.py $A > $out/sq3.log 2>&1 || { echo sq3 failed; tail -3 $out/sq3.log; exit 1; }
echo done
