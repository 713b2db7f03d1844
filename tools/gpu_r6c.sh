set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/prof_r6c/a -o a --output-format csv -- python3 tools/bench_table.py --iters 2 > gpurun_out/r6c_a.log 2>&1 || { tail -5 gpurun_out/r6c_a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_ANY -d gpurun_out/prof_r6c/b -o b --output-format csv -- python3 tools/bench_table.py --iters 2 > gpurun_out/r6c_b.log 2>&1 || { tail -5 gpurun_out/r6c_b.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/prof_r6c > gpurun_out/r6c_pmc.txt 2>&1 || true
ls gpurun_out/prof_r6c/*
