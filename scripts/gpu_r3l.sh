#!/bin/bash
# 256-pixel tiles (SG_HIST_NI=2, 8-wave workgroups, 2 per CU) against the default 128-pixel tiles
# after the round-2 VALU reductions
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r3l}
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 3; }
  echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
}
for rep in 1 2 3; do
  run ni1_$rep
  run ni2_$rep SG_HIST_NI=2
done
