#!/bin/bash
# k_stack_replay timing (SG_HIST_DBG=12: per-pixel cycles, fp80 sd recomputations, reason
# counters), then configs[1] / configs[4] / normalised benches at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4c}
mkdir -p $O
SG_HIST_DBG=12 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/replay_prof.log 2>&1 || { echo "replay prof failed"; tail -20 $O/replay_prof.log; exit 3; }
grep -a "replay:\|sg why" $O/replay_prof.log | tail -4
timeout -k 10 300 python bench.py --workload register-mean --steps 10 --warmup 2 --no-cpu-baseline > $O/register_mean.log 2>&1 || { echo "register-mean failed"; tail -20 $O/register_mean.log; exit 3; }
timeout -k 10 300 python bench.py --workload winsorized-rgb --steps 5 --warmup 1 --no-cpu-baseline > $O/winsorized_rgb.log 2>&1 || { echo "winsorized failed"; tail -20 $O/winsorized_rgb.log; exit 3; }
timeout -k 10 300 python bench.py --normalize additive-scaling --steps 10 --warmup 2 --no-cpu-baseline > $O/sigma_additive.log 2>&1 || { echo "additive failed"; tail -20 $O/sigma_additive.log; exit 3; }
for f in register_mean winsorized_rgb sigma_additive; do echo "$f $(grep '^{' $O/$f.log | cut -c1-400)"; done
