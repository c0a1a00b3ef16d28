#!/bin/bash
# A/B of libwsgpu.so builds on the host-to-host stage-chain line (batcher -> inflate -> validator),
# interleaved:  scripts/ab_stages.sh <lib_a.so> <lib_b.so> [...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2 3; do for lib in "$@"; do
  WSG_LIB=$lib timeout -k 10 240 python bench.py --only e2e_stages --extra-steps 3 > gpurun_out/abst.json 2>gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('$(basename $lib)', d['value'], d['ms_per_batch'], d.get('feed_ms'), d.get('wait_ms'))"
done; done
