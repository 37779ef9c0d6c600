#!/bin/bash
# round 2, session 3: GPU tests at the new default (builtin packed binning, two frames
# interleaved), then A/B: lib_ab1 = round-2 inline-asm binning, lib_ab2 = builtins, one frame
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4a}
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
  run asm_$rep SG_LIB_PATH=$L/lib_ab1/libsirilgpu.so
  run b1_$rep SG_LIB_PATH=$L/lib_ab2/libsirilgpu.so
done
