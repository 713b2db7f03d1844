set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/cu_mask_probe.py > gpurun_out/r5z2_cuprobe.json 2> gpurun_out/r5z2_cuprobe.err || { tail -5 gpurun_out/r5z2_cuprobe.err; exit 1; }
cat gpurun_out/r5z2_cuprobe.json
timeout -k 10 400 python bench.py > gpurun_out/r5z2_bench.json 2> gpurun_out/r5z2_bench.err || { tail -5 gpurun_out/r5z2_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r5z2_bench.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d.get('pipelined')))"
