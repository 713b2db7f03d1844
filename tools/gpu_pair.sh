set -u
# Wave decoder with paired tag steps: parity first, then the single-block
# latency, the drop-in, and the bench line with its C3 classes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r4p}
T="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_dropin_contract.py > gpurun_out/${P}_parity.txt 2>&1 || { tail -30 gpurun_out/${P}_parity.txt; exit 1; }
tail -2 gpurun_out/${P}_parity.txt
REPS=300 timeout -k 10 200 python tools/dropin_breakdown.py > gpurun_out/${P}_breakdown.json 2>&1 || exit 1
grep '^{' gpurun_out/${P}_breakdown.json
NO_TDB=1 REPS=1000 timeout -k 10 300 python tools/bench_dropin_latency.py > gpurun_out/${P}_dropin.json 2>&1 || exit 1
grep '^{' gpurun_out/${P}_dropin.json | head -c 400; echo
timeout -k 10 500 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { tail -5 gpurun_out/${P}_bench.err; exit 1; }
grep '^{' gpurun_out/${P}_bench.json | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j.get('c3'))"
