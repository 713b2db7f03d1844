set -u
mkdir -p gpurun_out
LGS_FRAME_OVERLAP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_table.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6t_pytest.txt 2>&1 || { tail -30 gpurun_out/r6t_pytest.txt; exit 1; }
tail -1 gpurun_out/r6t_pytest.txt
: > gpurun_out/r6t_ab.txt
for r in 1 2 3; do
  for v in 0 1; do
    LGS_FRAME_OVERLAP=$v timeout -k 10 120 python tools/bench_table.py --iters 10 > gpurun_out/r6t_$v.json 2> gpurun_out/r6t_$v.err || { tail -5 gpurun_out/r6t_$v.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r6t_$v.json').read().strip().splitlines()[-1]); print('$r frame_overlap=$v', round(d['write_ms']*1e3,1), round(d['read_ms']*1e3,1), d['parity'])" >> gpurun_out/r6t_ab.txt
  done
done
cat gpurun_out/r6t_ab.txt
