#!/bin/bash
# SQ counter passes over one bench step of k_stack_hist, per debug mode
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc3
i=0
for d in 0 3; do
for grp in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE" "SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS_ATOMIC SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  SG_HIST_DBG=$d timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc3/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc3/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmc3/p$i.log; exit 3; }
  echo "== dbg $d pass $i"
  grep k_stack_hist gpurun_out/pmc3/p$i/run_counter_collection.csv | awk -F, '{print $(NF-3), $(NF-2)}'
done
done
