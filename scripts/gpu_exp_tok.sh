#!/bin/bash
# k_infl_tok split-lane experiments (tools/exp/tok_*: tools/prof_infl_tok.hip over experiment
# copies of inflate.hip): one lane a message vs lane pairs, on the bench batch and a
# stage-chain-sized one.   scripts/gpu_exp_tok.sh "<variants>" [tests]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_stages.py -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > gpurun_out/exp_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/exp_tests.log; [ $rc -eq 0 ] || exit $rc
fi
python tools/make_inflate_input.py /tmp/infl_full.bin 8192 && python tools/make_inflate_input.py /tmp/infl_stage.bin 819 || exit 1
for inp in stage full; do
  for v in $1; do for pairs in 0 1; do
    echo "== $inp $v pairs=$pairs"
    timeout -k 10 120 tools/exp/tok_$v /tmp/infl_$inp.bin 262144 1 1 $pairs > gpurun_out/exp_one.txt 2>&1 || { cat gpurun_out/exp_one.txt; exit 1; }
    grep -A10 "rep 2" gpurun_out/exp_one.txt | grep -v "blocks\|messages  \|bail"
  done; done
done
