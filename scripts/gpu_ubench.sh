#!/bin/bash
# kernel microbenchmarks (text 4 KiB, binary 4 KiB, binary 1 KiB, text 64 KiB, text 100 B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "1048576 4096 1" "1048576 4096 0" "4194304 1024 0" "65536 65536 1" "16777216 100 1"; do
  echo "=== ubench $cfg"
  timeout -k 10 120 ./tools/ubench_unmask $cfg || exit $?
done
