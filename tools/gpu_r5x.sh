set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/cu_mask_probe.py 86 128 64 170 > gpurun_out/r5x_cumask.json 2> gpurun_out/r5x_cumask.err || { tail -5 gpurun_out/r5x_cumask.err; exit 1; }
cat gpurun_out/r5x_cumask.json
