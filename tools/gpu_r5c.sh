set -u
# round 5 session c: GPU tests on the exact-far decoder; PMC of the codec kernels.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r5c_pytest.txt 2>&1 || { tail -30 gpurun_out/r5c_pytest.txt; exit 1; }
tail -3 gpurun_out/r5c_pytest.txt
PASSES="trace sqA sqB lds2 fetch write" bash tools/profile.sh r5c || exit 1
python tools/pmc_summary.py gpurun_out/prof_r5c > gpurun_out/r5c_pmc.txt 2>&1; tail -70 gpurun_out/r5c_pmc.txt
