set -u
# round 5 session k: parity + contract with the service on; table paths; bench with table/CU-partition fields.
mkdir -p gpurun_out
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
LGS_DIE_EXIT=3 timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_dropin_contract.py > gpurun_out/r5k_parity.txt 2>&1 || { tail -40 gpurun_out/r5k_parity.txt; exit 1; }
tail -2 gpurun_out/r5k_parity.txt
timeout -k 10 300 python tools/bench_table.py > gpurun_out/r5k_table.json 2>&1 || { tail -20 gpurun_out/r5k_table.json; exit 1; }
grep -v amdgpu.ids gpurun_out/r5k_table.json
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c3 > gpurun_out/r5k_bench.json 2> gpurun_out/r5k_bench.err || { tail -5 gpurun_out/r5k_bench.err; exit 1; }
python -c "
import json; d=json.loads([l for l in open('gpurun_out/r5k_bench.json') if l.startswith('{')][-1])
print({k: d.get(k) for k in ('value','ms_per_step','parity')}); print(d.get('pipelined')); print(d.get('table')); print({k: round(v['avg_ms']*1e3,1) for k, v in d['kernels'].items()})"
