#!/bin/bash
# A/B of libwsgpu.so builds on the PCIe-inclusive paths (bench.py --e2e), interleaved:
#   scripts/ab_e2e.sh <lib_a.so> <lib_b.so> [...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2 3; do for lib in "$@"; do
  WSG_LIB=$lib timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-extras --no-cpu-baseline --e2e > gpurun_out/abe2e.json 2>gpurun_out/abe2e.err || { tail -5 gpurun_out/abe2e.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abe2e.json'))['e2e_pinned'];n=d['native_batcher'];print('$(basename $lib)', 'pipelined', d['pipelined']['GiB_per_s'], 'native', n['GiB_per_s'], 'feed', n['feed_GiB_per_s'])"
done; done
