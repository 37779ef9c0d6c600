#!/bin/bash
# counter passes over one bench step of the hist kernel (full and SG_HIST_DBG variants)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
i=0
for dbg in 0 3; do
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM"; do
  i=$((i+1))
  SG_HIST_DBG=$dbg timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc2/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc2/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmc2/p$i.log; }
  python3 - $i $dbg <<'PY'
import csv,sys
i,dbg=sys.argv[1],sys.argv[2]
try:
    for r in csv.DictReader(open(f'gpurun_out/pmc2/p{i}/run_counter_collection.csv')):
        if 'k_stack_hist' in r['Kernel_Name']:
            print('dbg',dbg,r['Counter_Name'],r['Counter_Value'])
except Exception as e: print('parse fail',i,e)
PY
done
done
