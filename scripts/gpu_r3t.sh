#!/bin/bash
# re-tune after the tile-start changes: build-phase priority (SG_HIST_PRIO 0 / 1 / 2 / 3) and
# two half blocks in flight (lib_ab2, -DSGH_NB=2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r3t}
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 3; }
  echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
}
L=$PWD/siril-0.9_amd
for rep in 1 2; do
  run prio1_$rep
  run prio0_$rep SG_HIST_PRIO=0
  run prio2_$rep SG_HIST_PRIO=2
  run prio3_$rep SG_HIST_PRIO=3
  run nb2_$rep SG_LIB_PATH=$L/lib_ab2/libsirilgpu.so
done
