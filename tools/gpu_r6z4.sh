set -u
mkdir -p gpurun_out
: > gpurun_out/r6z4_ab.txt
for r in 1 2 3; do
  for v in tbase tilp; do
    timeout -k 10 120 python tools/bench_table.py --iters 10 --lib probes/$v.so > gpurun_out/r6z4_$v.json 2> gpurun_out/r6z4_$v.err || { tail -5 gpurun_out/r6z4_$v.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r6z4_$v.json').read().strip().splitlines()[-1]); print('$r $v', round(d['write_ms']*1e3,1), round(d['read_ms']*1e3,1), round(d['crc_ms']*1e3,1), d['parity'])" >> gpurun_out/r6z4_ab.txt
  done
done
cat gpurun_out/r6z4_ab.txt
