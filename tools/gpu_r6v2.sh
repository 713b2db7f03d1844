set -u
mkdir -p gpurun_out
PROBE_CHECK=1 timeout -k 10 800 python tools/probe_ab.py probes/sbase.so probes/smaxilp.so probes/smaxmem.so probes/sbase.so probes/smaxilp.so probes/smaxmem.so probes/sbase.so probes/smaxilp.so probes/smaxmem.so probes/sbase.so probes/smaxilp.so probes/smaxmem.so > gpurun_out/r6v2_ab.txt 2> gpurun_out/r6v2_ab.err || { tail -5 gpurun_out/r6v2_ab.err; exit 1; }
cat gpurun_out/r6v2_ab.txt | python -c "
import sys,json
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(d['lib'], round(d['encode_us'],1), round(d['decode_us'],1), d.get('encode_exact'), d.get('decode_exact'))"
