set -u
mkdir -p gpurun_out
: > gpurun_out/r6j_ab.txt
for r in 1 2; do
  for v in late early fused; do
    case $v in late) E="LGS_VERIFY_EARLY=0";; early) E="LGS_VERIFY_EARLY=1";; fused) E="LGS_VERIFY_OVERLAP=0";; esac
    env $E timeout -k 10 120 python tools/bench_table.py --iters 10 > gpurun_out/r6j_$v.json 2> gpurun_out/r6j_$v.err || { tail -5 gpurun_out/r6j_$v.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r6j_$v.json').read().strip().splitlines()[-1]); print('$r $v', round(d['write_ms']*1e3,1), round(d['read_ms']*1e3,1), d['parity'])" >> gpurun_out/r6j_ab.txt
  done
done
cat gpurun_out/r6j_ab.txt
