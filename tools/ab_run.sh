#!/usr/bin/env bash
# tools/ab_run.sh -- scratch GPU step for A/B timing of probe builds
# (tools/probe_ab.py); edited per experiment, output under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PROBE_CHECK=1
timeout -k 10 500 python tools/probe_ab.py "$@" > gpurun_out/ab.log 2>&1
rc=$?; cat gpurun_out/ab.log; exit $rc
