set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_table.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6m_pytest.txt 2>&1 || { tail -30 gpurun_out/r6m_pytest.txt; exit 1; }
tail -2 gpurun_out/r6m_pytest.txt
VARIANTS="base sepcopy base2" bash tools/gpu_r6l.sh
