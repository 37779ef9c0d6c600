#!/bin/bash
# tiles per workgroup (lib_ab2 built with the tile loop, -DSGH_TPW_MAX=4; SG_HIST_TPW = 1, 2, 4)
# against HEAD (no loop); GPU tests of HEAD first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r3p}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 3; }
  echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
}
L=$PWD/siril-0.9_amd/lib_ab2/libsirilgpu.so
for rep in 1 2; do
  run head_$rep
  run loop_t1_$rep SG_LIB_PATH=$L SG_HIST_TPW=1
  run loop_t2_$rep SG_LIB_PATH=$L SG_HIST_TPW=2
  run loop_t4_$rep SG_LIB_PATH=$L SG_HIST_TPW=4
done
SG_LIB_PATH=$L SG_HIST_TPW=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_stack.py tests/test_gpu_bands.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_tpw2.log 2>&1; echo "tpw2 tests rc=$?"; tail -1 $O/pytest_tpw2.log
