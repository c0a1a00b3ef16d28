#!/bin/bash
# A/B of the aggregator line (inside bench --only configs2) for builds of libwsgpu.so:
#   scripts/ab_agg.sh <lib_a.so> <lib_b.so> [...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2 3; do for lib in "$@"; do
  WSG_LIB=$lib timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --extra-steps 10 --only configs2 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'))['aggregate'];r=d['roofline'];print('$(basename $lib)', d['value'], r['achieved'], r.get('frac'), d.get('pipeline_ms'))"
done; done
