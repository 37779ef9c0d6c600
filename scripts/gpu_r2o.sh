#!/bin/bash
# SIGMA finish with lanes pulling columns: GPU tests, then A/B default (NB=2 pull) / lib_ab1 (NB=1
# pull) / lib_ab2 (NB=1 lane pairs), both tile widths
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r2m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest_gpu.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 3; }
  echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
}
L1=$PWD/siril-0.9_amd/lib_ab1/libsirilgpu.so
L2=$PWD/siril-0.9_amd/lib_ab2/libsirilgpu.so
for rep in 1 2; do
  run nb2pull_ni2_$rep SG_HIST_NI=2
  run nb1pull_ni2_$rep SG_HIST_NI=2 SG_LIB_PATH=$L1
  run nb1pair_ni2_$rep SG_HIST_NI=2 SG_LIB_PATH=$L2
  run pull_ni1_$rep SG_HIST_NI=1 SG_LIB_PATH=$L1
  run pair_ni1_$rep SG_HIST_NI=1 SG_LIB_PATH=$L2
done
