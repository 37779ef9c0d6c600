#!/bin/bash
# Diagnosis of k_stack_hist: A/B debug modes, SQ counters, FETCH_SIZE calibration
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
rocprofv3 -L > gpurun_out/diag/counters_list.txt 2>&1 || true
for d in 0 2 3 5; do
  SG_HIST_DBG=$d timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/diag/ab$d.log 2>&1 || { echo "ab $d failed"; tail -5 gpurun_out/diag/ab$d.log; exit 3; }
  python3 -c "import json;d=json.loads(open('gpurun_out/diag/ab$d.log').read().splitlines()[-1]);print('dbg $d', d['kernel_ms'], d['ms_per_step'])"
done
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD" "GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/diag/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/diag/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/diag/p$i.log; }
  grep k_stack_hist gpurun_out/diag/p$i/run_counter_collection.csv | awk -F, '{print $(NF-3), $(NF-2)}'
done
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/diag/probe -o run -- ./tools/bw_probe > gpurun_out/diag/probe.log 2>&1 || { echo "probe pmc failed"; tail -3 gpurun_out/diag/probe.log; exit 4; }
cat gpurun_out/diag/probe.log | grep -v amdgpu.ids
grep k_probe gpurun_out/diag/probe/run_counter_collection.csv | awk -F, '{print $9, $10, $(NF-2)}'
