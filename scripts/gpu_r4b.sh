#!/bin/bash
# step overhead: one packed H2D of the call's inputs, one counter read-back (no mid-step round
# trip), register bitonic sort in k_stack_replay; A/B against lib_ab3 (HEAD before), then a
# rocprofv3 kernel trace of the new default; frame-load cache policy A/B (lib_auxN: sc0 / nt / both)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4b}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 3; }
tail -2 $O/pytest_gpu.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 3; }
  echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
}
L=$PWD/siril-0.9_amd
for rep in 1 2 3; do
  run new_$rep
  run old_$rep SG_LIB_PATH=$L/lib_ab3/libsirilgpu.so
  for a in 1 2 3; do run aux${a}_$rep SG_LIB_PATH=$L/lib_aux$a/libsirilgpu.so; done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 3; }
find $O/prof -name "*.csv" | head
