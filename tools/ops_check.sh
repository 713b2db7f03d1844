#!/usr/bin/env bash
# tools/ops_check.sh -- GPU session for the two-pass decoder: its parity
# tests, then C2 timings (ring vs ops, alternating processes, bytes checked),
# then a kernel-trace of one ops child.  Stops at a crash or time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIB=lcdb_amd/liblcdb_gpu_snappy.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 \
    --timeout-method thread -k "${OPS_K:-ops}" -p no:cacheprovider > gpurun_out/ops_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/ops_pytest.log | tail -n 20
[ $rc -ge 2 ] && [ $rc -ne 5 ] && { tail -n 40 gpurun_out/ops_pytest.log; exit $rc; }
PROBE_CHECK=1 timeout -k 10 300 python tools/probe_ab.py $LIB@ring $LIB@ops $LIB@ring $LIB@ops \
    || exit $?
LGS_DECODE_KERNEL=ops timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ops_prof \
    -o run --output-format csv -- python tools/probe_ab.py --child $LIB > gpurun_out/ops_prof.log 2>&1 || exit $?
find gpurun_out/ops_prof -name "*kernel_stats.csv" -exec cut -c1-160 {} \;
exit $rc
