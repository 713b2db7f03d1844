set -u
# round 4 session i: the chain decoder's parity and latency; quad narrowing probes.
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_parity.py -k "small_batch or dropin or variants_golden or runahead" > gpurun_out/r4i_chain.txt 2>&1 || { tail -30 gpurun_out/r4i_chain.txt; exit 1; }
tail -2 gpurun_out/r4i_chain.txt
NO_TDB=1 REPS=1000 timeout -k 10 300 python tools/bench_dropin_latency.py > gpurun_out/r4i_dropin.json 2>&1 || exit 1
REPS=300 timeout -k 10 200 python tools/dropin_breakdown.py > gpurun_out/r4i_breakdown.json 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r4i_dropin.json | head -c 420; echo
grep -v amdgpu.ids gpurun_out/r4i_breakdown.json
timeout -k 10 500 $T tests/test_gpu_parity.py tests/test_dropin_contract.py tests/test_gpu_probe_decoders.py > gpurun_out/r4i_parity.txt 2>&1 || { tail -30 gpurun_out/r4i_parity.txt; exit 1; }
tail -2 gpurun_out/r4i_parity.txt
for q in q1 q1a q1b q1c q0; do LGS_DECODE_KERNEL=quad timeout -k 10 200 python tools/quad_diag.py probes/$q.so 1 > gpurun_out/r4i_diag_$q.txt 2>&1; grep -v amdgpu.ids gpurun_out/r4i_diag_$q.txt | head -1; done
timeout -k 10 200 python tools/pipe_ab.py 20 > gpurun_out/r4i_pipe.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r4i_pipe.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c3 > gpurun_out/r4i_bench.json 2> gpurun_out/r4i_bench.err || { tail -5 gpurun_out/r4i_bench.err; exit 1; }
python -c "
import json; d=json.loads([l for l in open('gpurun_out/r4i_bench.json') if l.startswith('{')][-1])
print({k: d.get(k) for k in ('value','ms_per_step')}, d.get('pipelined'), {k: d.get(k) for k in ('encode_ms','decode_ms')})"
