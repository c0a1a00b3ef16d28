#!/bin/bash
# A/B of libwsgpu.so builds on one secondary bench line, interleaved (3 rounds):
#   scripts/ab_line.sh <line> <lib_a.so> <lib_b.so> [...]     (line: bench.py --only names)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LINE=$1; shift
for round in 1 2 3; do for lib in "$@"; do
  WSG_LIB=$lib timeout -k 10 240 python bench.py --only "$LINE" --no-cpu-baseline --extra-steps 10 > gpurun_out/abline.json 2>gpurun_out/abline.err || { tail -5 gpurun_out/abline.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abline.json'));print('$(basename $lib)', d['value'], d['ms_per_step'], d.get('pipeline_ms'))"
done; done
