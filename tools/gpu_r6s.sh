set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6s_pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r6s_pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/r6s_pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6s_smoke.log 2>&1 || { tail -5 gpurun_out/r6s_smoke.log; exit 1; }
tail -1 gpurun_out/r6s_smoke.log
