#!/bin/bash
# A/B of libwsgpu.so builds on the host-to-host stage-chain lines (batcher -> inflate ->
# validator), interleaved over 3 rounds:
#   scripts/ab_stages.sh <lib_a.so[:depth]> <lib_b.so[:depth]> [...]
# `depth` = the flushes the bench keeps in flight with that build (WSG_BENCH_INFLIGHT:
# builds made with another WSG_AB_INFLIGHT); LINES overrides the lines (default: the
# burst and the steady stage lines; e2e_aggregate and inflate are others).  Variant
# builds: scripts/build_variant.sh <tag> batcher.hip|inflate.hip -D<switch> (the
# WSG_AB_* / WSG_TOK_* switches in the sources; profiles/r05_ab/ holds round 5's runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LINES=${LINES:-"e2e_stages e2e_stages_steady"}
for round in 1 2 3; do
  for spec in "$@"; do
    lib=${spec%%:*}
    depth=${spec#*:}
    [ "$depth" = "$spec" ] && depth=""
    for line in $LINES; do
      steps=3
      [ "$line" = inflate ] && steps=10
      ( [ -n "$depth" ] && export WSG_BENCH_INFLIGHT=$depth
        WSG_LIB=$lib timeout -k 10 240 python bench.py --only "$line" --no-cpu-baseline --extra-steps $steps \
          > gpurun_out/abst.json 2> gpurun_out/abst.err ) || { tail -5 gpurun_out/abst.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('$line $(basename $lib)${depth:+ depth $depth}', d['value'], d.get('ms_per_batch', d.get('ms_per_step')), d.get('feed_ms'), d.get('wait_ms'))"
    done
  done
done
