#!/usr/bin/env bash
# tools/ab_run.sh -- scratch GPU session for a candidate kernel change: the
# codec parity tests on the product library, then A/B timings of
# probes/base.so (previous build) against probes/new.so (this build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || exit $rc
export PROBE_CHECK=1
timeout -k 10 300 python tools/probe_ab.py probes/base.so probes/new.so probes/base.so probes/new.so || exit $?
for lib in probes/base.so probes/new.so; do
  timeout -k 10 300 python tools/bench_mixed.py --lib $lib --iters 10 > gpurun_out/ab_mixed_$(basename $lib .so).json || exit $?
  python -c "
import json,sys; d=json.load(open('gpurun_out/ab_mixed_$(basename $lib .so).json'))
print('$lib', {k:(round(v['encode_GiBps'],1), round(v['decode_GiBps'],1)) for k,v in d['classes'].items()}, 'mix', round(d['mixed_one_launch']['encode_GiBps'],1), round(d['mixed_one_launch']['decode_GiBps'],1), d['parity'])"
done
