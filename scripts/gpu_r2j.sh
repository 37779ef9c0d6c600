#!/bin/bash
# A/B: lane-pair vs single-lane SIGMA finish (lib_ab1: NB=1 pair, lib_ab2: NB=1 single),
# 256-px (NI=2) and 128-px (NI=1) tiles; timeline of the single-lane finish
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r2j}
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 3; }
  echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
}
L1=$PWD/siril-0.9_amd/lib_ab1/libsirilgpu.so
L2=$PWD/siril-0.9_amd/lib_ab2/libsirilgpu.so
for rep in 1 2; do
  run pair_ni2_$rep SG_HIST_NI=2 SG_LIB_PATH=$L1
  run single_ni2_$rep SG_HIST_NI=2 SG_LIB_PATH=$L2
  run pair_ni1_$rep SG_HIST_NI=1 SG_LIB_PATH=$L1
  run single_ni1_$rep SG_HIST_NI=1 SG_LIB_PATH=$L2
done
SG_LIB_PATH=$L2 timeout -k 10 200 python scripts/timeline2.py > $O/timeline_single.log 2>&1 && grep -v amdgpu.ids $O/timeline_single.log | head -8
SG_LIB_PATH=$L1 timeout -k 10 200 python scripts/timeline2.py > $O/timeline_pair.log 2>&1 && grep -v amdgpu.ids $O/timeline_pair.log | head -8
