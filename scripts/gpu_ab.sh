#!/bin/bash
# A/B timing of the histogram kernel (SG_HIST_DBG: 0 full, 1 no sigma loop, 2 build only,
# 3 loads only) and of the frame stride (power of two vs padded)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_stack.py -m gpu -x -q -p no:cacheprovider -k hist > gpurun_out/pytest_hist.log 2>&1 || { echo "hist tests failed"; tail -30 gpurun_out/pytest_hist.log | cut -c1-400; exit 3; }
tail -1 gpurun_out/pytest_hist.log
for cfg in "0 0" "2 0" "3 0"; do
  set -- $cfg
  SG_HIST_DBG=$1 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --frame-pad $2 > gpurun_out/ab_$1_$2.log 2>&1 || { echo "ab $cfg failed"; tail -5 gpurun_out/ab_$1_$2.log; exit 3; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_$1_$2.log').read().splitlines()[-1]);print('dbg=$1 pad=$2', d['kernel_ms'], d['ms_per_step'], d['roofline']['achieved'], d['redo_pixels'])"
done
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log | cut -c1-300
