#!/bin/bash
# Winsorize fast iterations with the median / inner sums cached between clamps: GPU tests,
# configs[4] under rocprofv3 (replay time)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4w}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload winsorized-rgb --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 3; }
echo "wins $(grep '^{' $O/prof.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms"])')"
grep -h "replay" $O/prof/run_kernel_stats.csv | cut -c1-120
