set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "wide or c3 or golden or runahead or split" > gpurun_out/wide_pytest.log 2>&1 || { tail -n 40 gpurun_out/wide_pytest.log; exit 1; }
tail -n 3 gpurun_out/wide_pytest.log
for w in walk trips walk trips; do
  LGS_WIDE_DECODER=$w timeout -k 10 200 python tools/bench_mixed.py --iters 10 > gpurun_out/wide_mixed_$w.json
  python -c "
import json; d=json.load(open('gpurun_out/wide_mixed_$w.json'))
print('$w', {k:(round(v['encode_GiBps'],1), round(v['decode_GiBps'],1)) for k,v in d['classes'].items()}, 'mix', round(d['mixed_one_launch']['decode_GiBps'],1), d['parity'])"
done
