#!/usr/bin/env bash
# tools/profile.sh TAG -- rocprofv3 kernel trace + PMC passes of the codec
# kernels (tools/prof_kernels.py), one counter group per run, outputs under
# gpurun_out/prof_TAG/.  Stops at the first run that crashes or times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r1}
shift || true
args="${*:---blocks 65536 --iters 3}"
out=gpurun_out/prof_$tag
mkdir -p "$out"
pass() {  # name, then rocprofv3 options
  local name=$1; shift
  echo "== $name" | tee -a "$out/passes.log"
  timeout -k 10 300 rocprofv3 "$@" -d "$out/$name" -o "$name" --output-format csv \
      -- python3 tools/prof_kernels.py $args > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$out/passes.log"
  tail -n 3 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
passes="${PASSES:-trace sqA sqB tcp fetch write}"
want() { case " $passes " in *" $1 "*) return 0;; esac; return 1; }
want trace && pass trace --kernel-trace --stats
want sqA && pass sqA --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
want sqB && pass sqB --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
want tcp && pass tcp --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr
want lds && pass lds --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
want lds2 && pass lds2 --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE
want occ && pass occ --pmc MeanOccupancyPerCU
want fetch && pass fetch --pmc FETCH_SIZE
want write && pass write --pmc WRITE_SIZE
exit 0
