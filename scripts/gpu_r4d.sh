#!/bin/bash
# k_stack_replay SIGMA fast passes (prefix sums on the sorted stack): GPU tests, replay timing
# (SG_HIST_DBG=12), bench x3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4d}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 3; }
tail -2 $O/pytest_gpu.log
SG_HIST_DBG=12 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/replay_prof.log 2>&1 || { echo "replay prof failed"; tail -20 $O/replay_prof.log; exit 3; }
grep -a "replay" $O/replay_prof.log | tail -4
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/new_$rep.log 2>&1 || { echo "bench failed"; tail -20 $O/new_$rep.log; exit 3; }
  echo "new_$rep $(grep '^{' $O/new_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
done
