#!/bin/bash
# build-phase A/B modes compiled out of the production steady loop (SGH_DBG_MODES=0) vs the
# probe build with them (lib_dbg): GPU stack tests, 3 alternating bench rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4v}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 3; }
  echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"])')"
}
L=$PWD/siril-0.9_amd
for rep in 1 2 3; do
  run new_$rep
  run dbg_$rep SG_LIB_PATH=$L/lib_dbg/libsirilgpu.so
done
