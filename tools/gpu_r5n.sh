set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r5n
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5n -o tbl --output-format csv -- python3 tools/bench_table.py --iters 5 > gpurun_out/prof_r5n/log.txt 2>&1 || { tail -5 gpurun_out/prof_r5n/log.txt; exit 1; }
f=$(find gpurun_out/prof_r5n -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -20
