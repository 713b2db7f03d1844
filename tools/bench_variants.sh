#!/usr/bin/env bash
# A/B: run bench.py once per environment setting, e.g.
#   tools/bench_variants.sh LGS_DECODE_KERNEL=ring LGS_DECODE_KERNEL=wave
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  tag=$(echo "$v" | tr '=,' '__')
  env ${v//,/ } timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
     > "gpurun_out/bench_$tag.log" 2>&1 || { echo "bench $v failed rc=$?"; tail -5 "gpurun_out/bench_$tag.log"; exit 3; }
  echo "$v: $(grep -o '"value": [0-9.]*\|"encode_GiBps": [0-9.]*\|"decode_GiBps": [0-9.]*\|"parity": "[^"]*"' "gpurun_out/bench_$tag.log" | tr '\n' ' ')"
done
