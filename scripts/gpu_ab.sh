#!/bin/bash
# A/B of a decode switch on one bench line: scripts/gpu_ab.sh ENVVAR [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
var=$1; shift
for v in 1 0 1 0; do
  env $var=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-extras --no-cpu-baseline --extra-steps 10 "$@" > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$var=$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['pipeline_ms'])"
done
