set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6b -o r6b --output-format csv -- python3 tools/bench_table.py --iters 5 > gpurun_out/r6b.log 2>&1 || { tail -20 gpurun_out/r6b.log; exit 1; }
f=$(find gpurun_out/prof_r6b -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/r6b_kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r6b_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], r['AverageNs'])"
