set -u
mkdir -p gpurun_out
: > gpurun_out/r6o.txt
for ov in 1 0; do
  LGS_VERIFY_OVERLAP=$ov timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-pipelined --no-cpu-baseline --no-c3 > gpurun_out/r6o_bench_$ov.json 2> gpurun_out/r6o_bench_$ov.err || { tail -5 gpurun_out/r6o_bench_$ov.err; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/r6o_bench_$ov.json') if l.startswith('{')][-1]); t=d['table']; print('bench overlap=$ov', round(t['write_ms']*1e3,1), round(t['read_ms']*1e3,1), round(t['read_noverify_ms']*1e3,1), round(d['kernels']['decode']['avg_ms']*1e3,1))" >> gpurun_out/r6o.txt
  LGS_VERIFY_OVERLAP=$ov timeout -k 10 120 python tools/bench_table.py --iters 10 > gpurun_out/r6o_bt_$ov.json 2> gpurun_out/r6o_bt_$ov.err || { tail -5 gpurun_out/r6o_bt_$ov.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r6o_bt_$ov.json').read().strip().splitlines()[-1]); print('bench_table overlap=$ov', round(d['write_ms']*1e3,1), round(d['read_ms']*1e3,1))" >> gpurun_out/r6o.txt
done
cat gpurun_out/r6o.txt
