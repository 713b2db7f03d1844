set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6x2_pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r6x2_pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/r6x2_pytest_gpu.txt
PROBE_CHECK=1 timeout -k 10 600 python tools/probe_ab.py probes/noilp.so probes/split.so probes/noilp.so probes/split.so probes/noilp.so probes/split.so probes/noilp.so probes/split.so > gpurun_out/r6x2_ab.txt 2> gpurun_out/r6x2_ab.err || { tail -5 gpurun_out/r6x2_ab.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r6x2_ab.txt'):
    if l.startswith('{'):
        d=json.loads(l); print(d['lib'], round(d['encode_us'],1), round(d['decode_us'],1), d.get('encode_exact'), d.get('decode_exact'))"
: > gpurun_out/r6x2_lat.txt
for r in 1 2 3; do
  for v in split noilp; do
    if [ $v = noilp ]; then L="LD_LIBRARY_PATH=probes/noilp"; else L="X=1"; fi
    env $L timeout -k 10 120 tools/dropin_latency 4000 > gpurun_out/r6x2_$v.json 2>&1 || { tail -5 gpurun_out/r6x2_$v.json; exit 1; }
    echo "$r $v $(cat gpurun_out/r6x2_$v.json)" >> gpurun_out/r6x2_lat.txt
  done
done
cat gpurun_out/r6x2_lat.txt
