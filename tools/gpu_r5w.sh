set -u
# round 5 session w: CU-partitioned encode || decode with the split balanced by decoder generations.
mkdir -p gpurun_out
for k in 1 2; do
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c3 --no-table > gpurun_out/r5w_bench_$k.json 2> gpurun_out/r5w_bench_$k.err || { tail -5 gpurun_out/r5w_bench_$k.err; exit 1; }
python -c "
import json; d=json.loads([l for l in open('gpurun_out/r5w_bench_$k.json') if l.startswith('{')][-1])
print({k: d.get(k) for k in ('value','ms_per_step')}); print(d.get('pipelined'))"
done
