#!/bin/bash
# instruction-cache and instruction-mix counters of k_stack_hist, SIGMA (configs[2]) and
# WINSORIZED (configs[4]) workloads, one bench step each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc5
i=0
for wl in sigma winsorized-rgb; do
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc5/p$i -o run -- python3 bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc5/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmc5/p$i.log; exit 3; }
  echo "== $wl pass $i"
  grep k_stack_hist gpurun_out/pmc5/p$i/run_counter_collection.csv | awk -F, '{print $(NF-3), $(NF-2)}'
done
done
