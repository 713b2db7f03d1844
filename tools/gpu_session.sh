set -u
# round 4 session h: the workgroup decoder's parity, then its timings.
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_parity.py -k "group" > gpurun_out/r4h_group.txt 2>&1 || { tail -30 gpurun_out/r4h_group.txt; exit 1; }
tail -2 gpurun_out/r4h_group.txt
timeout -k 10 500 $T tests/test_gpu_parity.py tests/test_dropin_contract.py > gpurun_out/r4h_parity.txt 2>&1 || { tail -30 gpurun_out/r4h_parity.txt; exit 1; }
tail -2 gpurun_out/r4h_parity.txt
PROBE_CHECK=1 timeout -k 10 400 python tools/probe_ab.py probes/cur.so probes/patsrc.so probes/sinkmirror.so probes/both.so probes/cur.so probes/patsrc.so > gpurun_out/r4h_ring_ab.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r4h_ring_ab.txt
NO_TDB=1 REPS=1000 timeout -k 10 300 python tools/bench_dropin_latency.py > gpurun_out/r4h_dropin.json 2>&1 || exit 1
REPS=300 timeout -k 10 200 python tools/dropin_breakdown.py > gpurun_out/r4h_breakdown.json 2>&1 || exit 1
timeout -k 10 300 python tools/bench_mixed.py --iters 10 > gpurun_out/r4h_mixed_walk.json 2>&1 || exit 1
LGS_WIDE_DECODER=group timeout -k 10 300 python tools/bench_mixed.py --iters 10 > gpurun_out/r4h_mixed_group.json 2>&1 || exit 1
timeout -k 10 200 python tools/pipe_ab.py 20 > gpurun_out/r4h_pipe.txt 2>&1 || exit 1
LGS_DECODE_KERNEL=quad timeout -k 10 200 python tools/quad_diag.py probes/q1.so 6 > gpurun_out/r4h_quad_diag.txt 2>&1
for f in r4h_mixed_walk r4h_mixed_group; do python -c "
import json; d=json.load(open('gpurun_out/$f.json'))
print('$f', {k:(round(v['encode_GiBps'],1), round(v['decode_GiBps'],1)) for k,v in d['classes'].items()}, 'mix', round(d['mixed_one_launch']['encode_GiBps'],1), round(d['mixed_one_launch']['decode_GiBps'],1), d['parity'])"; done
tail -c 400 gpurun_out/r4h_dropin.json; echo
grep -v amdgpu.ids gpurun_out/r4h_breakdown.json
grep -v amdgpu.ids gpurun_out/r4h_quad_diag.txt | head -8
grep -v amdgpu.ids gpurun_out/r4h_pipe.txt
timeout -k 10 120 python tools/ring_trips.py probes/tripcount.so > gpurun_out/r4h_trips.json 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r4h_trips.json
PASSES="sqA sqB fetch write" bash tools/profile.sh r4h_ring --blocks 65536 --iters 2 --which decode > /dev/null 2>&1 || exit 1
PASSES="fetch" bash tools/profile.sh r4h_refill --blocks 65536 --iters 2 --which decode --lib probes/nofarflush.so > /dev/null 2>&1 || exit 1
python tools/pmc_summary.py gpurun_out/prof_r4h_ring > gpurun_out/r4h_ring_pmc.txt 2>&1
python tools/pmc_summary.py gpurun_out/prof_r4h_refill > gpurun_out/r4h_refill_pmc.txt 2>&1
tail -5 gpurun_out/r4h_ring_pmc.txt gpurun_out/r4h_refill_pmc.txt
