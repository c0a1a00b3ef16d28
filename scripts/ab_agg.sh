#!/bin/bash
# A/B of libwsgpu.so builds on the aggregator line (configs[2] decode + aggregate), interleaved:
#   scripts/ab_agg.sh <lib_a.so> <lib_b.so> [...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2 3; do for lib in "$@"; do
  WSG_LIB=$lib timeout -k 10 180 python bench.py --only configs2 --no-cpu-baseline --extra-steps 10 > gpurun_out/abagg.json 2>gpurun_out/abagg.err || { tail -5 gpurun_out/abagg.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abagg.json'));a=d['aggregate'];print('$(basename $lib)', a['value'], a['ms_per_step'], a['roofline'].get('avg_launch_ms'), {k:v for k,v in a.get('pipeline_ms',{}).items() if 'agg' in k})"
done; done
