# rocprofv3 kernel stats of the deflate line on the committed build
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
T=${TAG:-r06y}
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${T}_deflate -o k --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --extra-steps 2 --only deflate > gpurun_out/prof/${T}_deflate.log 2>&1 || exit 1
echo done
