#!/bin/bash
# Round 5, run t: no stage advance in flush_async (the feed's side job and wait move the
# chains: flush_async returns at once, so the next upload starts sooner) against the
# current build, burst / steady stage lines, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for round in 1 2 3 4; do
  for lib in pull noflushadv; do
    for line in e2e_stages e2e_stages_steady; do
      WSG_LIB=snf4j_amd/_ab/libwsgpu_$lib.so timeout -k 10 240 python bench.py --only $line \
        --extra-steps 3 > gpurun_out/abst.json 2> gpurun_out/abst.err || { tail -5 gpurun_out/abst.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/abst.json'));print('$line $lib', d['value'], d.get('ms_per_batch'), d.get('feed_ms'), d.get('wait_ms'))"
    done
  done
done | tee gpurun_out/r05t_ab_flushadv.txt
echo R05T_DONE
