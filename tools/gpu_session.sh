#!/usr/bin/env bash
# tools/gpu_session.sh -- the one GPU session script (replaces the per-session
# gpu_r*.sh of rounds 5-6).  Runs the steps named in STEPS, in this order,
# each under its own time limit, and stops at the first failure; outputs go
# to gpurun_out/${P}_*.  Usage on the box:
#   P=r7a STEPS="tests smoke bench" bash tools/gpu_session.sh
# Steps:
#   tests     the whole -m gpu suite (K="-k expr" narrows it)
#   service   the service / drop-in / lcdb-integration tests only
#   smoke     __graft_entry__.smoke()
#   bench     python bench.py (BENCH_ARGS)
#   rocprof   rocprofv3 --kernel-trace --stats of the bench's codec kernels
#   pmc       PMC passes of the codec kernels (tools/profile.sh, PASSES)
#   table     rocprofv3 summary of the table kernels (tools/bench_table.py)
#   latency   the drop-in's per-call latency from C (tools/dropin_latency)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-s}
STEPS=${STEPS:-tests smoke bench}
K=${K:-}
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
want() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }
step() {  # name, limit, output file, command...
  local name=$1 lim=$2 out=$3; shift 3
  echo "== $name"
  timeout -k 10 "$lim" "$@" > "$out" 2>&1
  local rc=$?
  tail -n 3 "$out" | grep -v amdgpu.ids
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; exit $rc; fi
}
want tests && step tests 1000 gpurun_out/${P}_pytest_gpu.txt $T -m gpu $K tests
want service && step service 600 gpurun_out/${P}_pytest_service.txt $T -m gpu \
    tests/test_gpu_service.py tests/test_dropin_contract.py tests/test_lcdb_integration.py \
    tests/test_gpu_parity.py -k "dropin or service or lcdb or c5"
want smoke && step smoke 300 gpurun_out/${P}_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
if want bench; then
  echo "== bench"
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err \
    || { tail -5 gpurun_out/${P}_bench.err; exit 1; }
  grep '^{' gpurun_out/${P}_bench.json | tail -1 | head -c 600; echo
fi
if want rocprof; then
  echo "== rocprof"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${P}_bench -o bench \
      --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-pipelined \
      --no-cpu-baseline --no-c3 --no-table > gpurun_out/${P}_bench_under_rocprof.json \
      2> gpurun_out/${P}_bench_under_rocprof.err \
    || { tail -5 gpurun_out/${P}_bench_under_rocprof.err; exit 1; }
  find gpurun_out/prof_${P}_bench -name '*kernel_stats.csv' -exec cp {} gpurun_out/${P}_kernel_stats.csv \;
  head -5 gpurun_out/${P}_kernel_stats.csv | cut -c1-160
fi
if want pmc; then
  echo "== pmc"
  PASSES="${PASSES:-fetch write sqA sqB lds2}" bash tools/profile.sh ${P} --blocks 65536 --iters 2 \
      > gpurun_out/${P}_profile.log 2>&1 || { tail -5 gpurun_out/${P}_profile.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/prof_${P} > gpurun_out/${P}_pmc.txt 2>&1
  head -40 gpurun_out/${P}_pmc.txt
fi
if want table; then
  echo "== table"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${P}_table -o table \
      --output-format csv -- python3 tools/bench_table.py --iters 5 \
      > gpurun_out/${P}_table_under_rocprof.json 2>&1 \
    || { tail -5 gpurun_out/${P}_table_under_rocprof.json; exit 1; }
  find gpurun_out/prof_${P}_table -name '*kernel_stats.csv' -exec cp {} gpurun_out/${P}_table_kernel_stats.csv \;
  grep -v amdgpu.ids gpurun_out/${P}_table_under_rocprof.json | tail -3
fi
want latency && step latency 120 gpurun_out/${P}_dropin_c.json tools/dropin_latency 4000
echo "== done"
