set -u
# Round-4 final measurements on one MI355X: the GPU test suite, the bench
# line, its rocprof kernel summary, and the PMC passes of the two codec
# kernels (traffic + instruction counts).  Each GPU step has its own limit;
# the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r4z}
T="python -u -m pytest -q -p no:cacheprovider --timeout 400 --timeout-method thread"
timeout -k 10 900 $T tests -m gpu > gpurun_out/${P}_pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/${P}_pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/${P}_pytest_gpu.txt
NO_TDB=1 REPS=1000 timeout -k 10 300 python tools/bench_dropin_latency.py > gpurun_out/${P}_dropin.json 2>&1 || exit 1
REPS=300 timeout -k 10 200 python tools/dropin_breakdown.py > gpurun_out/${P}_breakdown.json 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/${P}_dropin.json | head -c 300; echo
timeout -k 10 600 python bench.py > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { tail -5 gpurun_out/${P}_bench.err; exit 1; }
grep '^{' gpurun_out/${P}_bench.json | tail -1 | head -c 1500; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${P}_bench -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-pipelined --no-cpu-baseline --no-c3 > gpurun_out/${P}_bench_under_rocprof.json 2> gpurun_out/${P}_bench_under_rocprof.err || { tail -5 gpurun_out/${P}_bench_under_rocprof.err; exit 1; }
PASSES="fetch write sqA sqB" bash tools/profile.sh ${P} --blocks 65536 --iters 2 > /dev/null 2>&1 || { echo profile failed; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_${P} > gpurun_out/${P}_pmc.txt 2>&1
grep -v amdgpu.ids gpurun_out/${P}_pmc.txt | head -60
