#!/usr/bin/env bash
# tools/iter.sh -- one kernel-iteration check on the GPU box: the GPU parity
# tests that cover the codec kernels (fast subset), then an A/B timing of
# the product library against probes/base.so (the previous build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_table.py -m gpu -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/iter_pytest.log 2>&1
rc=$?
tail -n 3 gpurun_out/iter_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/probe_ab.py probes/base.so lcdb_amd/liblcdb_gpu_snappy.so \
    probes/base.so lcdb_amd/liblcdb_gpu_snappy.so
