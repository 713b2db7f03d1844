set -u
# round 5 session a: ring-decoder trip phases; encoder first-batch width A/B.
mkdir -p gpurun_out
timeout -k 10 300 python tools/ring_phases.py probes/ringph.so lcdb_amd/liblcdb_gpu_snappy.so > gpurun_out/r5a_phases.json 2> gpurun_out/r5a_phases.err || { tail -20 gpurun_out/r5a_phases.err; exit 1; }
cat gpurun_out/r5a_phases.json
PROBE_CHECK=1 timeout -k 10 600 python tools/probe_ab.py probes/base.so probes/e14.so probes/e30.so probes/e8.so probes/base.so probes/e14.so probes/e30.so probes/e8.so > gpurun_out/r5a_encw.txt 2>&1 || { tail -20 gpurun_out/r5a_encw.txt; exit 1; }
cat gpurun_out/r5a_encw.txt
