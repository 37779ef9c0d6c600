#!/bin/bash
# WINSORIZED passes on the replay's fast path (replay_winsor_inner): GPU tests, then configs[4]
# A/B against lib_wf0 (-DSG_REPLAY_WFAST=0) with a kernel trace of the replay
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4q}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
L=$PWD/siril-0.9_amd
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload winsorized-rgb --steps 3 --warmup 1 --no-cpu-baseline > $O/new_$rep.log 2>&1 || { echo "bench failed"; tail -20 $O/new_$rep.log; exit 3; }
  echo "new_$rep $(grep '^{' $O/new_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms"], d["redo_pixels"])')"
  SG_LIB_PATH=$L/lib_wf0/libsirilgpu.so timeout -k 10 300 python bench.py --workload winsorized-rgb --steps 3 --warmup 1 --no-cpu-baseline > $O/old_$rep.log 2>&1 || { echo "bench failed"; tail -20 $O/old_$rep.log; exit 3; }
  echo "old_$rep $(grep '^{' $O/old_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms"], d["redo_pixels"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload winsorized-rgb --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 3; }
grep -h "replay\|literal\|k_stack_hist\|k_stack_sorted" $O/prof/run_kernel_stats.csv | cut -c1-160
