#!/bin/bash
# VALU / issue counters of k_stack_hist per debug mode
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc4
for d in 0 13 2 3; do
  SG_HIST_DBG=$d timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc4/d$d -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc4/d$d.log 2>&1 || { echo "dbg $d failed"; tail -3 gpurun_out/pmc4/d$d.log; exit 3; }
  echo "== dbg $d"; grep k_stack_hist gpurun_out/pmc4/d$d/run_counter_collection.csv | awk -F, '{print $(NF-3), $(NF-2)}'
done
