#!/bin/bash
# LDS / VALU counters of the registration FFT kernels (register-mean, configs[1], one step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcr
i=0
for grp in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES" "SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FLOPS_FP64 SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_VMEM SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcr/p$i -o run -- python3 bench.py --workload register-mean --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcr/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmcr/p$i.log; exit 3; }
  echo "== pass $i ok"
done
