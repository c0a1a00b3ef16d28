#!/bin/bash
# A/B of an environment switch on one build, interleaved:
#   scripts/ab_env.sh WSG_TUNE_<NAME> "v1 v2 ..." (bench.py apply_tuning) <python expr over d (the JSON line)> [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAR=$1; VALS=$2; EXPR=$3; shift 3
for round in 1 2 3; do for v in $VALS; do
  env "$VAR=$v" timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --extra-steps 10 "$@" > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$VAR=$v', $EXPR)"
done; done
