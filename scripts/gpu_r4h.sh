#!/bin/bash
# 256-pixel tiles on 4 waves (SG_HIST_NI=2: two dwords per lane and frame = 512-byte row
# segments, two workgroups per CU, up to 256 VGPRs): parity under SG_HIST_NI=2, then A/B
# against the 128-pixel default, NB2=1 (lib_nb1) and the round-2 8-wave variant (lib_w8)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4h}
mkdir -p $O
SG_HIST_NI=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_stack.py tests/test_gpu_fullsize.py tests/test_gpu_edges.py tests/test_gpu_bands.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_ni2.log 2>&1 || { echo "pytest ni2 failed"; tail -30 $O/pytest_ni2.log; exit 3; }
tail -1 $O/pytest_ni2.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 3; }
  echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
}
L=$PWD/siril-0.9_amd
for rep in 1 2; do
  run ni1_$rep
  run ni2w4_$rep SG_HIST_NI=2
  run ni2nb1_$rep SG_HIST_NI=2 SG_LIB_PATH=$L/lib_nb1/libsirilgpu.so
  run ni2w8_$rep SG_HIST_NI=2 SG_LIB_PATH=$L/lib_w8/libsirilgpu.so
done
run ni2w4_lo SG_HIST_NI=2 SG_HIST_DBG=3
run ni1_lo SG_HIST_DBG=3
