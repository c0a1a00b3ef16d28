#!/bin/bash
# Round 5, run h: the stage chain streaming (the steady line: 4x longer session streams,
# ~20 flushes a pass) at two and three flushes in flight, two-phase inflate against the
# run-d build, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for round in 1 2 3; do
  for cfg in "async2 2" "cur 2" "cur 3"; do
    set -- $cfg
    WSG_LIB=snf4j_amd/_ab/libwsgpu_$1.so WSG_BENCH_INFLIGHT=$2 timeout -k 10 240 python bench.py --only e2e_stages_steady \
      --extra-steps 3 > gpurun_out/abst.json 2> gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('steady $1 depth $2', d['value'], d['ms_per_batch'], d.get('feed_ms'), d.get('wait_ms'), d['rounds'])"
  done
done | tee gpurun_out/r05h_ab_steady.txt
echo R05H_DONE
