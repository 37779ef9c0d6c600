#!/bin/bash
# re-tune after the binning change: two 16-frame blocks in flight (lib_nb2, -DSGH_NB=2) vs one
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4x}
mkdir -p $O
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 3; }
  echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
}
L=$PWD/siril-0.9_amd
for rep in 1 2 3; do
  run nb1_$rep
  run nb2_$rep SG_LIB_PATH=$L/lib_nb2/libsirilgpu.so
done
