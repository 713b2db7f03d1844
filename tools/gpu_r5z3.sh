set -u
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/r5z3_bench.json 2> gpurun_out/r5z3_bench.err || { tail -5 gpurun_out/r5z3_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r5z3_bench.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d.get('pipelined')))"
