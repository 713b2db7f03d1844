set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/prof_r5q; mkdir -p $out
pass() { local name=$1; shift; timeout -k 10 240 rocprofv3 "$@" -d $out/$name -o $name --output-format csv -- python3 tools/bench_table.py --iters 3 > $out/$name.log 2>&1 || { tail -3 $out/$name.log; exit 1; }; }
pass sqA --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
pass sqB --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
pass lds --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE
python tools/pmc_summary.py $out > gpurun_out/r5q_pmc.txt 2>&1; grep -A40 "crc_kernel" gpurun_out/r5q_pmc.txt | head -45
