#!/bin/bash
# rocprofv3 evidence for bench lines: scripts/gpu_profiles.sh ROUND [line ...]
# lines: north configs1 configs2 configs3 encode validator inflate handshake
# (default: all).  Per line a scripts/gpu_pmc.sh run, then its pmc_report JSON
# and the kernel-trace stats copied to gpurun_out/prof/ROUND_<line>_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
round=$1; shift
lines=${*:-north configs1 configs2 configs3 encode validator inflate handshake hs_client}
for l in $lines; do
  echo "[$(date +%T)] profiling $l"
  if [ "$l" = north ]; then args="--no-extras"; else args="--only $l"; fi
  bash scripts/gpu_pmc.sh "$l" $args || exit 1
  python3 scripts/pmc_report.py "gpurun_out/prof/$l" --json "gpurun_out/prof/${round}_${l}_pmc.json" > /dev/null || exit 1
  cp gpurun_out/prof/$l/kt/*kernel_stats.csv "gpurun_out/prof/${round}_${l}_kernel_stats.csv" || exit 1
done
echo "profiles done"
