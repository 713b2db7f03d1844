set -u
# round 5 session g: GPU tests on the round-5 decoder; trip phases again; replay probe exact.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r5g_pytest.txt 2>&1 || { tail -30 gpurun_out/r5g_pytest.txt; exit 1; }
tail -2 gpurun_out/r5g_pytest.txt
timeout -k 10 300 python tools/ring_phases.py probes/ringph.so lcdb_amd/liblcdb_gpu_snappy.so > gpurun_out/r5g_phases.json 2> gpurun_out/r5g_phases.err || { tail -20 gpurun_out/r5g_phases.err; exit 1; }
cat gpurun_out/r5g_phases.json
PROBE_CHECK=1 timeout -k 10 300 python tools/probe_ab.py probes/replay.so > gpurun_out/r5g_replay.txt 2>&1 || { tail -20 gpurun_out/r5g_replay.txt; exit 1; }
cat gpurun_out/r5g_replay.txt
