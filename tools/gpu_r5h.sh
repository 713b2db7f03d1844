set -u
# round 5 session h: the drop-in service -- tests, latency on/off.
mkdir -p gpurun_out
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_service.py > gpurun_out/r5h_service.txt 2>&1 || { tail -40 gpurun_out/r5h_service.txt; exit 1; }
tail -2 gpurun_out/r5h_service.txt
LGS_DROPIN_SERVICE=1 NO_TDB=1 REPS=2000 timeout -k 10 300 python tools/bench_dropin_latency.py > gpurun_out/r5h_dropin_svc.json 2>&1 || { tail -20 gpurun_out/r5h_dropin_svc.json; exit 1; }
grep -v amdgpu.ids gpurun_out/r5h_dropin_svc.json | head -c 700; echo
LGS_DROPIN_SERVICE=0 NO_TDB=1 REPS=2000 timeout -k 10 300 python tools/bench_dropin_latency.py > gpurun_out/r5h_dropin_launch.json 2>&1 || { tail -20 gpurun_out/r5h_dropin_launch.json; exit 1; }
grep -v amdgpu.ids gpurun_out/r5h_dropin_launch.json | head -c 700; echo
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_dropin_contract.py > gpurun_out/r5h_parity.txt 2>&1 || { tail -40 gpurun_out/r5h_parity.txt; exit 1; }
tail -2 gpurun_out/r5h_parity.txt
