set -u
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r6y_bench.json 2> gpurun_out/r6y_bench.err || { tail -5 gpurun_out/r6y_bench.err; exit 1; }
grep '^{' gpurun_out/r6y_bench.json | tail -1 | head -c 300; echo
timeout -k 10 120 tools/dropin_latency 4000 > gpurun_out/r6y_dropin_c.json 2>&1 || { tail -5 gpurun_out/r6y_dropin_c.json; exit 1; }
cat gpurun_out/r6y_dropin_c.json
