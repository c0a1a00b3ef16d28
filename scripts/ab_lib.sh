#!/bin/bash
# A/B of two builds of libwsgpu.so on the same box, interleaved:
#   scripts/ab_lib.sh <lib_a.so> <lib_b.so> [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=$1; B=$2; shift 2
for round in 1 2 3; do for lib in "$A" "$B"; do
  WSG_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-extras --no-cpu-baseline --extra-steps 10 "$@" > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$(basename $lib)', d['value'], d['ms_per_step'], r['avg_launch_ms'], r.get('frac_of_copy_ceiling'), d.get('pipeline_ms'))"
done; done
