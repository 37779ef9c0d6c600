#!/bin/bash
# finish sensitivity: +800 VALU per wave (lib_ab1), +s_sleep 30 / 90 (~1.9k / 5.8k cycles) per
# wave at the start of the finish (lib_ab2 / lib_ab3), against HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r2w}
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 3; }
  echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
}
L=$PWD/siril-0.9_amd
for rep in 1 2; do
  run base_$rep
  run valu800_$rep SG_LIB_PATH=$L/lib_ab1/libsirilgpu.so
  run sleep30_$rep SG_LIB_PATH=$L/lib_ab2/libsirilgpu.so
  run sleep90_$rep SG_LIB_PATH=$L/lib_ab3/libsirilgpu.so
done
