#!/bin/bash
# A batch of GPU steps for one call: the tests of the changed paths, then A/B runs of
# library builds (scripts/build_variant.sh) through the ab_*.sh drivers, each step
# time-limited, stopping at the first failure.  Replaces round 4's one-off
# gpu_r04_*.sh scripts (git history keeps them).
#   scripts/ab_batch.sh <tag> "<pytest files or ->" [<driver> <out-name> <lib.so>... --] ...
# e.g.
#   scripts/ab_batch.sh r05c "tests/test_gpu_stages.py tests/test_gpu_inflate.py" \
#     ab_stages.sh stagecopy snf4j_amd/_ab/libwsgpu_old.so snf4j_amd/_ab/libwsgpu_new.so --
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1; tests=$2; shift 2
if [ "$tests" != - ]; then
  timeout -k 10 900 python -u -m pytest $tests -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "gpurun_out/${tag}_tests.log" 2>&1
  rc=$?; tail -3 "gpurun_out/${tag}_tests.log"; [ $rc -eq 0 ] || exit $rc
fi
while [ $# -gt 0 ]; do
  driver=$1 name=$2; shift 2
  libs=()
  while [ $# -gt 0 ] && [ "$1" != -- ]; do libs+=("$1"); shift; done
  shift
  timeout -k 10 900 bash "scripts/$driver" "${libs[@]}" > "gpurun_out/${tag}_ab_${name}.txt" 2>&1 || \
    { tail -20 "gpurun_out/${tag}_ab_${name}.txt"; exit 1; }
  cat "gpurun_out/${tag}_ab_${name}.txt"
done
echo BATCH_DONE
