#!/usr/bin/env bash
# Run bench.py once per decode-kernel variant (LGS_DECODE_KERNEL) for A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${*:-wave lane64 lane32}; do
  LGS_DECODE_KERNEL=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
     > gpurun_out/bench_$v.log 2>&1 || { echo "bench $v failed rc=$?"; tail -5 gpurun_out/bench_$v.log; exit 3; }
  echo "$v: $(grep -o '"value": [0-9.]*\|"encode_GiBps": [0-9.]*\|"decode_GiBps": [0-9.]*\|"parity": "[^"]*"' gpurun_out/bench_$v.log | tr '\n' ' ')"
done
