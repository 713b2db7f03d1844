set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_table.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6n_pytest.txt 2>&1 || { tail -30 gpurun_out/r6n_pytest.txt; exit 1; }
tail -2 gpurun_out/r6n_pytest.txt
timeout -k 10 200 python tools/bench_table.py --iters 10 > gpurun_out/r6n_bench_table.json 2> gpurun_out/r6n_bench_table.err || { tail -5 gpurun_out/r6n_bench_table.err; exit 1; }
cat gpurun_out/r6n_bench_table.json
