set -u
mkdir -p gpurun_out
timeout -k 10 120 tools/dropin_latency 4000 > gpurun_out/r6d_dropin_c.json 2> gpurun_out/r6d_dropin_c.err || { tail -5 gpurun_out/r6d_dropin_c.err; exit 1; }
cat gpurun_out/r6d_dropin_c.json
timeout -k 10 120 python tools/bench_dropin_latency.py > gpurun_out/r6d_dropin_py.json 2> gpurun_out/r6d_dropin_py.err || { tail -5 gpurun_out/r6d_dropin_py.err; exit 1; }
cat gpurun_out/r6d_dropin_py.json
