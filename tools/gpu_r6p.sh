set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py tests/test_dropin_contract.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6p_pytest.txt 2>&1 || { tail -30 gpurun_out/r6p_pytest.txt; exit 1; }
tail -1 gpurun_out/r6p_pytest.txt
: > gpurun_out/r6p_ab.txt
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then L="LD_LIBRARY_PATH=probes/svc_old"; else L="X=1"; fi
    env $L timeout -k 10 120 tools/dropin_latency 4000 > gpurun_out/r6p_$v.json 2>&1 || { tail -5 gpurun_out/r6p_$v.json; exit 1; }
    echo "$r $v $(cat gpurun_out/r6p_$v.json)" >> gpurun_out/r6p_ab.txt
  done
done
cat gpurun_out/r6p_ab.txt
