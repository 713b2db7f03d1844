set -u
# round 5 session r: full GPU suite (C5 through the drop-in service), refreshed
# bloom / PCIe / host-API / drop-in numbers.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=r5r
T="python -u -m pytest -q -p no:cacheprovider --timeout 400 --timeout-method thread"
timeout -k 10 1000 $T tests -m gpu > gpurun_out/${P}_pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/${P}_pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/${P}_pytest_gpu.txt
cp gpurun_out/c5_result.json gpurun_out/${P}_c5_result.json
timeout -k 10 300 python tools/bench_bloom.py > gpurun_out/${P}_bloom.json 2>&1 || { tail -5 gpurun_out/${P}_bloom.json; exit 1; }
timeout -k 10 300 python tools/bench_pcie.py > gpurun_out/${P}_pcie.json 2>&1 || { tail -5 gpurun_out/${P}_pcie.json; exit 1; }
timeout -k 10 400 python tools/bench_host_api.py > gpurun_out/${P}_host_api.json 2>&1 || { tail -5 gpurun_out/${P}_host_api.json; exit 1; }
NO_TDB=1 REPS=2000 timeout -k 10 300 python tools/bench_dropin_latency.py > gpurun_out/${P}_dropin.json 2>&1 || exit 1
LGS_DROPIN_SERVICE=0 REPS=300 timeout -k 10 200 python tools/dropin_breakdown.py > gpurun_out/${P}_breakdown.json 2>&1 || exit 1
for f in bloom pcie host_api dropin breakdown; do echo "== $f"; grep -v amdgpu.ids gpurun_out/${P}_$f.json | tail -2 | head -c 1500; echo; done
