#!/bin/bash
# k_stack_replay timing only (SG_HIST_DBG=12)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4f}
mkdir -p $O
SG_HIST_DBG=12 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/replay_prof.log 2>&1 || { echo "replay prof failed"; tail -20 $O/replay_prof.log; exit 3; }
grep -a "replay" $O/replay_prof.log | tail -4
