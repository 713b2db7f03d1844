set -u
mkdir -p gpurun_out
: > gpurun_out/r6r_ab.txt
for r in 1 2; do
  for v in 0 2 5 10; do
    LGS_VERIFY_EARLY=$v timeout -k 10 120 python tools/bench_table.py --iters 10 > gpurun_out/r6r_$v.json 2> gpurun_out/r6r_$v.err || { tail -5 gpurun_out/r6r_$v.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r6r_$v.json').read().strip().splitlines()[-1]); print('$r early=$v', round(d['write_ms']*1e3,1), round(d['read_ms']*1e3,1), d['parity'])" >> gpurun_out/r6r_ab.txt
  done
done
cat gpurun_out/r6r_ab.txt
