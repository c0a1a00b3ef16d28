#!/bin/bash
# Round 5, run g: the stage chain's streams on more hardware queues (GPU_MAX_HW_QUEUES:
# HIP's default is 4 a process, and the chain uses the batcher context's three streams,
# the stage stream, the download stream and two pre-decode streams).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for round in 1 2 3; do
  for cfg in "async2 2 4" "async2 2 8" "cur 2 8" "cur 3 8" "cur 3 16"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$3 WSG_LIB=snf4j_amd/_ab/libwsgpu_$1.so WSG_BENCH_INFLIGHT=$2 timeout -k 10 240 python bench.py --only e2e_stages \
      --extra-steps 3 > gpurun_out/abst.json 2> gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('stages $1 depth $2 hwq $3', d['value'], d['ms_per_batch'], d.get('feed_ms'), d.get('wait_ms'))"
  done
done | tee gpurun_out/r05g_ab_hwq.txt
echo R05G_DONE
