#!/bin/bash
# k_stack_replay timing on configs[4] (SG_HIST_DBG=12)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4s}
mkdir -p $O
SG_HIST_DBG=12 timeout -k 10 300 python bench.py --workload winsorized-rgb --steps 1 --warmup 0 --no-cpu-baseline > $O/replay_prof_wins.log 2>&1 || { echo "probe failed"; tail -20 $O/replay_prof_wins.log; exit 3; }
grep -a "replay\|sg why" $O/replay_prof_wins.log | tail -6
