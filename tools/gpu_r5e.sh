set -u
# round 5 session e: 4-lanes-per-job flush.
mkdir -p gpurun_out
PROBE_CHECK=1 timeout -k 10 700 python tools/probe_ab.py probes/d0.so probes/pdw.so probes/f4.so probes/d0.so probes/pdw.so probes/f4.so probes/d0.so probes/pdw.so probes/f4.so > gpurun_out/r5e_ab.txt 2>&1 || { tail -20 gpurun_out/r5e_ab.txt; exit 1; }
python - <<'P'
import json
for l in open('gpurun_out/r5e_ab.txt'):
    if l.startswith('{'):
        d=json.loads(l); print(d['lib'], round(d['decode_us'],1), round(d['encode_us'],1), d['encode_exact'], d['decode_exact'])
P
