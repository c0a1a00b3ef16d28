#!/bin/bash
# k_inflate instruction-mix counters over the bench batch (run on the GPU box from the repo root).
export TMPDIR=/tmp
mkdir -p gpurun_out
python tools/make_inflate_input.py gpurun_out/infl_in.bin ${1:-1024} || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d gpurun_out/pmc_infl -o pmc --output-format csv -- ./tools/run_inflate gpurun_out/infl_in.bin > gpurun_out/pmc_infl.log 2>&1
rc=$?
rm -f gpurun_out/infl_in.bin
exit $rc
