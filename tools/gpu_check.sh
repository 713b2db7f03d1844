#!/usr/bin/env bash
# tools/gpu_check.sh -- one GPU-box session: gpu tests, smoke, bench, profile.
# Each GPU step has its own time limit.  An ordinary test failure (pytest
# exit 1) does not stop the session; a crash, abort, signal or time limit
# (exit >= 2) ends it before anything else touches the GPU.
#   usage: tools/gpu_check.sh [tests] [smoke] [bench] [prof] [latency] [pmc:TAG] [traffic:TAG]
#          (default: tests smoke bench prof)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
steps="${*:-tests smoke bench prof}"
run() {   # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/session.log
  local t0=$SECONDS
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($((SECONDS - t0))s)" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 2 ]; then echo "== stopping: $name exit $rc" | tee -a gpurun_out/session.log; exit $rc; fi
  return 0
}
for s in $steps; do
  case $s in
    tests) run pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider ;;
    alltests) run pytest_gpu 1100 python -m pytest tests -m gpu -q -p no:cacheprovider --durations=15 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 3 ;;
    prof)  run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run \
             --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pipelined --no-c3 ;;
    latency) run latency 600 python tools/bench_dropin_latency.py ;;
    pmc:*) run "pmc_${s#pmc:}" 900 bash tools/profile.sh "${s#pmc:}" ;;
    # CPU only: profiles/traffic_latest.json from that PMC run, so a later
    # bench step in the same session reports it (copy it back from the log)
    traffic:*) run "traffic_${s#traffic:}" 120 python tools/traffic_json.py "gpurun_out/prof_${s#traffic:}" "${s#traffic:}" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
