# round-6 checkpoint: every GPU test, smoke, the default bench line, deflate kernel stats
mkdir -p gpurun_out
T=${TAG:-r06y}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests_all.log 2>&1 || { tail -5 gpurun_out/${T}_gpu_tests_all.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${T}_deflate -o k --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --extra-steps 2 --only deflate > gpurun_out/prof/${T}_deflate.log 2>&1 || exit 1
echo done
