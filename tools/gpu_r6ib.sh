set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_service.py tests/test_dropin_contract.py tests/test_lcdb_integration.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6ib_pytest.txt 2>&1 || { tail -30 gpurun_out/r6ib_pytest.txt; exit 1; }
tail -1 gpurun_out/r6ib_pytest.txt
: > gpurun_out/r6ib_lat.txt
for r in 1 2 3; do
  for v in 1 0; do
    LGS_SERVICE_INBOX=$v timeout -k 10 120 tools/dropin_latency 4000 > gpurun_out/r6ib_$v.json 2>&1 || { tail -5 gpurun_out/r6ib_$v.json; exit 1; }
    echo "$r inbox=$v $(cat gpurun_out/r6ib_$v.json)" >> gpurun_out/r6ib_lat.txt
  done
done
cat gpurun_out/r6ib_lat.txt
