#!/usr/bin/env bash
# tools/ab_table.sh TAG LIB... -- the table GPU tests on the current library,
# then tools/bench_table.py over the current library and each LIB, twice,
# alternating (A/B of table-kernel builds).  A LIB of the form env:NAME=VALUE
# runs the current library with that environment variable instead.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=$1; shift
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $T -m gpu tests/test_gpu_table.py > gpurun_out/${P}_table_tests.txt 2>&1 || { tail -30 gpurun_out/${P}_table_tests.txt; exit 1; }
tail -1 gpurun_out/${P}_table_tests.txt
for r in 1 2; do
  for lib in cur "$@"; do
    arg=""; envv=""; tag=$(basename $lib .so)
    case $lib in
      cur) ;;
      env:*) envv=${lib#env:}; tag=${envv//=/_} ;;
      *) arg="--lib $lib" ;;
    esac
    timeout -k 10 300 env $envv python tools/bench_table.py --iters 10 $arg > gpurun_out/${P}_bt_${tag}_$r.json 2>&1 || { tail -5 gpurun_out/${P}_bt_${tag}_$r.json; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/${P}_bt_${tag}_$r.json') if l.startswith('{')][-1])
print('$tag $r', {k: round(d[k]*1000,1) for k in ('write_ms','read_ms','read_noverify_ms','crc_ms') if k in d}, d['parity'][:30])"
  done
done
