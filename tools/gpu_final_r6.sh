set -u
# Final measurements of the round on one MI355X: the -m gpu suite, smoke, the
# bench line, its rocprof kernel summary, the PMC passes of the two codec
# kernels (traffic keyed to the kernel sources), the table kernels' rocprof
# summary and the C-level drop-in latency.  Each GPU step has its own limit;
# stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6z}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${P}_pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/${P}_pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/${P}_pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.log 2>&1 || { tail -5 gpurun_out/${P}_smoke.log; exit 1; }
tail -1 gpurun_out/${P}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { tail -5 gpurun_out/${P}_bench.err; exit 1; }
grep '^{' gpurun_out/${P}_bench.json | tail -1 | head -c 400; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${P}_bench -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-pipelined --no-cpu-baseline --no-c3 --no-table > gpurun_out/${P}_bench_under_rocprof.json 2> gpurun_out/${P}_bench_under_rocprof.err || { tail -5 gpurun_out/${P}_bench_under_rocprof.err; exit 1; }
PASSES="fetch write sqA sqB lds2" bash tools/profile.sh ${P} --blocks 65536 --iters 2 > /dev/null 2>&1 || { echo profile failed; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_${P} > gpurun_out/${P}_pmc.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${P}_table -o table --output-format csv -- python3 tools/bench_table.py --iters 5 > gpurun_out/${P}_table_under_rocprof.json 2>&1 || { tail -5 gpurun_out/${P}_table_under_rocprof.json; exit 1; }
timeout -k 10 120 tools/dropin_latency 4000 > gpurun_out/${P}_dropin_c.json 2>&1 || { tail -5 gpurun_out/${P}_dropin_c.json; exit 1; }
echo done
