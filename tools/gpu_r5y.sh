set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/cu_mask_map.py > gpurun_out/r5y_cumap.json 2> gpurun_out/r5y_cumap.err || { tail -5 gpurun_out/r5y_cumap.err; exit 1; }
cat gpurun_out/r5y_cumap.json
