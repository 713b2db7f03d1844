set -u
# round 5 session b: decoder reads-first / exact far loads; encoder first-batch width.
mkdir -p gpurun_out
PROBE_CHECK=1 timeout -k 10 700 python tools/probe_ab.py probes/rbase.so probes/rf.so probes/fx.so probes/rffx.so probes/e8.so probes/e14.so probes/e30.so probes/rbase.so probes/rf.so probes/fx.so probes/rffx.so probes/e8.so probes/e14.so probes/e30.so > gpurun_out/r5b_ab.txt 2>&1 || { tail -20 gpurun_out/r5b_ab.txt; exit 1; }
cat gpurun_out/r5b_ab.txt
