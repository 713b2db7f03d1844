set -u
# round 5 session j: the drop-in service (fixed arena address), latency on/off; table paths.
mkdir -p gpurun_out
LGS_DIE_EXIT=3 timeout -k 10 120 python -u tools/svc_smoke.py > gpurun_out/r5j_smoke.txt 2>&1 || { grep -v amdgpu.ids gpurun_out/r5j_smoke.txt | tail; exit 1; }
grep -v amdgpu.ids gpurun_out/r5j_smoke.txt | tail -4
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
LGS_DIE_EXIT=3 timeout -k 10 300 $T tests/test_gpu_service.py > gpurun_out/r5j_service.txt 2>&1 || { tail -40 gpurun_out/r5j_service.txt; exit 1; }
tail -2 gpurun_out/r5j_service.txt
LGS_DROPIN_SERVICE=1 NO_TDB=1 REPS=2000 timeout -k 10 300 python tools/bench_dropin_latency.py > gpurun_out/r5j_dropin_svc.json 2>&1 || { tail -20 gpurun_out/r5j_dropin_svc.json; exit 1; }
grep -v amdgpu.ids gpurun_out/r5j_dropin_svc.json | head -c 900; echo
LGS_DROPIN_SERVICE=0 NO_TDB=1 REPS=2000 timeout -k 10 300 python tools/bench_dropin_latency.py > gpurun_out/r5j_dropin_launch.json 2>&1 || { tail -20 gpurun_out/r5j_dropin_launch.json; exit 1; }
grep -v amdgpu.ids gpurun_out/r5j_dropin_launch.json | head -c 900; echo
LGS_DIE_EXIT=3 timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_dropin_contract.py > gpurun_out/r5j_parity.txt 2>&1 || { tail -40 gpurun_out/r5j_parity.txt; exit 1; }
tail -2 gpurun_out/r5j_parity.txt
timeout -k 10 300 python tools/bench_table.py > gpurun_out/r5j_table.json 2>&1 || { tail -20 gpurun_out/r5j_table.json; exit 1; }
grep -v amdgpu.ids gpurun_out/r5j_table.json
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c3 > gpurun_out/r5j_bench.json 2> gpurun_out/r5j_bench.err || { tail -5 gpurun_out/r5j_bench.err; exit 1; }
python -c "
import json; d=json.loads([l for l in open('gpurun_out/r5j_bench.json') if l.startswith('{')][-1])
print({k: d.get(k) for k in ('value','ms_per_step','parity')}); print(d.get('pipelined')); print(d.get('table')); print({k: round(v['avg_ms']*1e3,1) for k, v in d['kernels'].items()})"
