set -u
mkdir -p gpurun_out
: > gpurun_out/r6l_ab.txt
for r in 1 2; do
  for v in ${VARIANTS:-base nolds nostore noload}; do
    timeout -k 10 120 python tools/bench_table.py --iters 5 --lib probes/$v.so > gpurun_out/r6l_$v.json 2> gpurun_out/r6l_$v.err; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$v rc=$rc"; tail -5 gpurun_out/r6l_$v.err; exit 1; fi
    python -c "
import json; d=json.loads(open('gpurun_out/r6l_$v.json').read().strip().splitlines()[-1]); print('$r', '$v', round(d['write_ms']*1e3,1), round(d['read_ms']*1e3,1), round(d['crc_ms']*1e3,1))" >> gpurun_out/r6l_ab.txt
  done
done
cat gpurun_out/r6l_ab.txt
