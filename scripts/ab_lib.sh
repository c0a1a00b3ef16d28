#!/bin/bash
# A/B of builds of libwsgpu.so on the same box, interleaved:
#   scripts/ab_lib.sh <lib_a.so> <lib_b.so> [<lib_c.so> ...] [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS=()
while [[ "$1" == *.so ]]; do LIBS+=("$1"); shift; done
for round in 1 2 3; do for lib in "${LIBS[@]}"; do
  WSG_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-extras --no-cpu-baseline --extra-steps 10 "$@" > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$(basename $lib)', d['value'], d['ms_per_step'], r['avg_launch_ms'], r.get('frac_of_copy_ceiling'), d.get('pipeline_ms'))"
done; done
