#!/bin/bash
# replay fast path from registers (no LDS reads per pass / Winsorize iteration, ballot ORs):
# GPU tests, replay probe on configs[4], configs[4] and configs[2] under rocprofv3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4t}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
SG_HIST_DBG=12 timeout -k 10 300 python bench.py --workload winsorized-rgb --steps 1 --warmup 0 --no-cpu-baseline > $O/replay_prof_wins.log 2>&1 || { echo "probe failed"; tail -20 $O/replay_prof_wins.log; exit 3; }
grep -a "replay" $O/replay_prof_wins.log | tail -2
for w in winsorized-rgb sigma; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_$w.log 2>&1 || { echo "prof $w failed"; tail -20 $O/prof_$w.log; exit 3; }
  echo "$w $(grep '^{' $O/prof_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("stage_ms"), d.get("kernel_ms"))')"
  grep -h "replay" $O/prof_$w/run_kernel_stats.csv | cut -c1-120
done
