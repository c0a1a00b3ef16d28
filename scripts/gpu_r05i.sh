#!/bin/bash
# Round 5, run i: the decode-only host paths (native batcher, drop-in loop) at two and
# three flushes in flight, same build, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for round in 1 2 3; do
  for d in 2 3; do
    WSG_BENCH_INFLIGHT=$d timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline --e2e \
      > gpurun_out/abe2e.json 2> gpurun_out/abe2e.err || { tail -5 gpurun_out/abe2e.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abe2e.json'));e=d['e2e_pinned'];print('e2e depth $d', e['native_batcher']['GiB_per_s'], e['drop_in_loop']['GiB_per_s'], e['drop_in_loop']['collected_blocking'])"
  done
done | tee gpurun_out/r05i_ab_e2e_depth.txt
echo R05I_DONE
