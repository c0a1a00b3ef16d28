#!/bin/bash
# Round 5, run o: the full GPU suite at four flushes in flight (three pre-decode
# contexts), then the stage lines against the three-in-flight build and the output
# gather at 24 and 48 workgroups, and the decode-only host lines at 3 and 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r05o_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05o_tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  for cfg in "d3t2 3" "d4t3 4" "g24 4" "g48 4"; do
    set -- $cfg
    for line in e2e_stages e2e_stages_steady; do
      WSG_LIB=snf4j_amd/_ab/libwsgpu_$1.so WSG_BENCH_INFLIGHT=$2 timeout -k 10 240 python bench.py --only $line \
        --extra-steps 3 > gpurun_out/abst.json 2> gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('$line $1', d['value'], d.get('ms_per_batch'), d.get('feed_ms'), d.get('wait_ms'))"
    done
  done
  for cfg in "d3t2 3" "d4t3 4"; do
    set -- $cfg
    WSG_LIB=snf4j_amd/_ab/libwsgpu_$1.so WSG_BENCH_INFLIGHT=$2 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-extras \
      --no-cpu-baseline --e2e > gpurun_out/abe2e.json 2> gpurun_out/abe2e.err || { tail -5 gpurun_out/abe2e.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abe2e.json'));e=d['e2e_pinned'];print('e2e $1', e['native_batcher']['GiB_per_s'], e['drop_in_loop']['GiB_per_s'], e['drop_in_loop']['collected_blocking'])"
  done
done | tee gpurun_out/r05o_ab.txt
echo R05O_DONE
