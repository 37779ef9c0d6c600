#!/bin/bash
# SQ counters of k_stack_hist (one bench step) for the tile widths and with / without the finish
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_r2}
mkdir -p $O
i=0
for cfg in "2 0" "2 2" "1 0" "1 2"; do
  set -- $cfg
  for grp in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_ANY"; do
    i=$((i+1))
    SG_HIST_NI=$1 SG_HIST_DBG=$2 timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; exit 3; }
    echo "== NI=$1 dbg=$2"
    grep k_stack_hist $O/p$i/run_counter_collection.csv | awk -F, '{print $(NF-3), $(NF-2)}' | sort -u
  done
done
