#!/bin/bash
# build-phase load depth A/B (scalar table loads since d71c006): base (NBUF 2 x 16 frames),
# lib_ab1 NBUF=3, lib_ab2 half blocks NB=2 (NI=1), lib_ab3 half blocks NB=1 (NI=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r2u}
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 3; }
  echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
}
L=$PWD/siril-0.9_amd
for rep in 1 2; do
  run base_$rep
  run nbuf3_$rep SG_LIB_PATH=$L/lib_ab1/libsirilgpu.so
  run half_nb2_$rep SG_LIB_PATH=$L/lib_ab2/libsirilgpu.so
  run half_nb1_$rep SG_LIB_PATH=$L/lib_ab3/libsirilgpu.so
done
