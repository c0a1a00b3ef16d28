# final tree: every GPU test and smoke
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06zh_gpu_tests_all.log 2>&1 || { tail -5 gpurun_out/r06zh_gpu_tests_all.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06zh_smoke.log 2>&1 || exit 1
echo done
