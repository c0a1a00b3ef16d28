#!/bin/bash
# Round 5, run q: the stage output gathered on the device and downloaded by one
# runtime D2H (WSG_AB_SDMA_OUT) instead of the gather kernel's PCIe stores — its
# stage tests, the burst / steady stage lines against the current build, and its
# device timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WSG_LIB=snf4j_amd/_ab/libwsgpu_sdma.so timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py \
  -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05q_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05q_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  for lib in d4t3 sdma; do
    for line in e2e_stages e2e_stages_steady; do
      WSG_LIB=snf4j_amd/_ab/libwsgpu_$lib.so timeout -k 10 240 python bench.py --only $line \
        --extra-steps 3 > gpurun_out/abst.json 2> gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('$line $lib', d['value'], d.get('ms_per_batch'), d.get('feed_ms'), d.get('wait_ms'))"
    done
  done
done | tee gpurun_out/r05q_ab_sdma.txt
cd /tmp && WSG_LIB=$GRAFT_REPO_ROOT/snf4j_amd/_ab/libwsgpu_sdma.so timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace \
  -d $GRAFT_REPO_ROOT/gpurun_out/r05q_prof_st -o run -- python $GRAFT_REPO_ROOT/bench.py --only e2e_stages --extra-steps 2 \
  > $GRAFT_REPO_ROOT/gpurun_out/r05q_prof_st.log 2>&1 || exit 1
echo R05Q_DONE
