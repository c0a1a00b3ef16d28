#!/bin/bash
# Round 5, run u: the output gather's priority — its waves at s_setprio 3 (gprio), its
# stream at the highest stream priority (sprio), both (gsprio) — against the current
# build on the burst / steady stage lines, interleaved; and the replay taking the
# pre-decode's device list as it is when nothing is held (samex).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in gsprio samex; do
  WSG_LIB=snf4j_amd/_ab/libwsgpu_$lib.so timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_inflate.py \
    -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05u_tests_$lib.log 2>&1
  rc=$?; tail -2 gpurun_out/r05u_tests_$lib.log; [ $rc -eq 0 ] || exit $rc
done
for round in 1 2 3; do
  for lib in pull gprio sprio gsprio samex; do
    for line in e2e_stages e2e_stages_steady; do
      WSG_LIB=snf4j_amd/_ab/libwsgpu_$lib.so timeout -k 10 240 python bench.py --only $line \
        --extra-steps 3 > gpurun_out/abst.json 2> gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('$line $lib', d['value'], d.get('ms_per_batch'), d.get('feed_ms'), d.get('wait_ms'))"
    done
  done
done | tee gpurun_out/r05u_ab_prio.txt
echo R05U_DONE
