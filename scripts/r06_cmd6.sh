# rocprofv3 kernel stats + PMC of the deflate line (round 6)
bash scripts/gpu_pmc.sh r06_deflate --only deflate || exit 1
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof/r06_deflate/tcc -o tcc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --extra-steps 2 --only deflate > gpurun_out/prof/r06_deflate/tcc.log 2>&1 || { echo "tcc pass failed"; exit 1; }
