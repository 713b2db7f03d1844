set -u
# round 5 session u: table kernels copying straight from global; stagger A/B.
mkdir -p gpurun_out
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_table.py tests/test_lcdb_integration.py -k "not c5" > gpurun_out/r5u_table_tests.txt 2>&1 || { tail -40 gpurun_out/r5u_table_tests.txt; exit 1; }
tail -2 gpurun_out/r5u_table_tests.txt
timeout -k 10 300 python tools/bench_table.py > gpurun_out/r5u_table.json 2>&1 || { tail -20 gpurun_out/r5u_table.json; exit 1; }
grep -v amdgpu.ids gpurun_out/r5u_table.json
bash tools/gpu_r5t.sh
