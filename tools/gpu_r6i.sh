set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r6i -o r6i --output-format csv -- python3 tools/bench_table.py --iters 3 ${BT_ARGS:-} > gpurun_out/r6i.log 2>&1 || { tail -20 gpurun_out/r6i.log; exit 1; }
f=$(find gpurun_out/prof_r6i -name '*kernel_trace.csv' | head -1); cp "$f" gpurun_out/r6i_trace.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r6i_trace.csv')))
rows=[r for r in rows if any(k in r['Kernel_Name'] for k in ('verify_kernel','check_kernel','decode_ring','merge_kernel'))]
rows.sort(key=lambda r:int(r['Start_Timestamp']))
t0=int(rows[0]['Start_Timestamp'])
for r in rows[-12:]:
    n=r['Kernel_Name'].split('(')[0].replace('void ','').replace('lgs::(anonymous namespace)::','')
    print(n[:40], (int(r['Start_Timestamp'])-t0)/1e3, (int(r['End_Timestamp'])-t0)/1e3, (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
PY
