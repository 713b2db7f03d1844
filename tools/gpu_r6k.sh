set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_table.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6k_pytest.txt 2>&1 || { tail -30 gpurun_out/r6k_pytest.txt; exit 1; }
tail -2 gpurun_out/r6k_pytest.txt
: > gpurun_out/r6k_ab.txt
for r in 1 2; do
  for v in overlap fused; do
    case $v in overlap) E="LGS_VERIFY_OVERLAP=1";; fused) E="LGS_VERIFY_OVERLAP=0";; esac
    env $E timeout -k 10 120 python tools/bench_table.py --iters 10 > gpurun_out/r6k_$v.json 2> gpurun_out/r6k_$v.err || { tail -5 gpurun_out/r6k_$v.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r6k_$v.json').read().strip().splitlines()[-1]); print('$r $v', round(d['write_ms']*1e3,1), round(d['read_ms']*1e3,1), d['parity'])" >> gpurun_out/r6k_ab.txt
  done
done
cat gpurun_out/r6k_ab.txt

