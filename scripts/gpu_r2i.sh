#!/bin/bash
# A/B: histogram build with 2 (default lib) vs 1 (lib_ab1) 16-frame blocks in flight per wave
# (256-px tiles), the 128-px tiles (SG_HIST_NI=1), and the NB=2 phase breakdown
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r2i}
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 3; }
  echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
}
for rep in 1 2; do
  run nb2_$rep SG_HIST_NI=2
  run nb1_$rep SG_HIST_NI=2 SG_LIB_PATH=$PWD/siril-0.9_amd/lib_ab1/libsirilgpu.so
  run ni1_$rep SG_HIST_NI=1
done
run nb2_d3 SG_HIST_NI=2 SG_HIST_DBG=3
run nb2_d2 SG_HIST_NI=2 SG_HIST_DBG=2
run nb2_d1 SG_HIST_NI=2 SG_HIST_DBG=1
