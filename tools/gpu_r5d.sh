set -u
# round 5 session d: dword-aligned ring LDS accesses (exact) and an aligned-piece probe.
mkdir -p gpurun_out
PROBE_CHECK=1 timeout -k 10 700 python tools/probe_ab.py probes/d0.so probes/dw.so probes/pdw.so probes/wdw.so probes/alp.so probes/d0.so probes/dw.so probes/pdw.so probes/wdw.so probes/alp.so > gpurun_out/r5d_ab.txt 2>&1 || { tail -20 gpurun_out/r5d_ab.txt; exit 1; }
cut -c1-60,100-400 gpurun_out/r5d_ab.txt
