#!/usr/bin/env bash
# tools/ab_run.sh -- scratch GPU session for a candidate kernel change: the
# codec parity tests on the product library, then A/B timings of
# probes/base.so (previous build) against probes/new.so (this build).
# Fails (non-zero exit, message on stderr) unless the parity gate actually
# ran and passed: a pytest that errors, selects nothing or skips is a failure.
set -euo pipefail
die() { echo "ab_run.sh: $*" >&2; exit 1; }
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 \
    || { tail -n 20 gpurun_out/ab_pytest.log >&2; die "parity gate failed"; }
tail -n 3 gpurun_out/ab_pytest.log
grep -Eq '^[0-9]+ passed' gpurun_out/ab_pytest.log || die "parity gate ran no tests"
! grep -Eq '[0-9]+ (skipped|failed|error)' gpurun_out/ab_pytest.log || die "parity gate skipped or failed tests"
export PROBE_CHECK=1
timeout -k 10 300 python tools/probe_ab.py probes/base.so probes/new.so probes/base.so probes/new.so \
    || die "probe_ab failed"
for lib in probes/base.so probes/new.so; do
  timeout -k 10 300 python tools/bench_mixed.py --lib $lib --iters 10 \
      > gpurun_out/ab_mixed_$(basename $lib .so).json || die "bench_mixed failed on $lib"
  python -c "
import json,sys; d=json.load(open('gpurun_out/ab_mixed_$(basename $lib .so).json'))
print('$lib', {k:(round(v['encode_GiBps'],1), round(v['decode_GiBps'],1)) for k,v in d['classes'].items()}, 'mix', round(d['mixed_one_launch']['encode_GiBps'],1), round(d['mixed_one_launch']['decode_GiBps'],1), d['parity']); sys.exit(0 if d['parity'] == 'round trips exact' else 1)" \
      || die "bench_mixed parity failed on $lib"
done
