#!/bin/bash
# A/B of the histogram kernel vs registration shifts (alignment of the pixel-pair loads)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_stack.py -m gpu -x -q -p no:cacheprovider -k hist > gpurun_out/pytest_hist.log 2>&1 || { echo "hist tests failed"; tail -30 gpurun_out/pytest_hist.log | cut -c1-400; exit 3; }
tail -1 gpurun_out/pytest_hist.log
for cfg in "0 16 x" "3 16 x" "5 16 x" "0 0 x"; do
  set -- $cfg
  ex=""; [ "$3" != "x" ] && ex=$3
  SG_HIST_DBG=$1 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --maxshift $2 $ex > gpurun_out/ab3.log 2>&1 || { echo "ab $cfg failed"; tail -5 gpurun_out/ab3.log; exit 3; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab3.log').read().splitlines()[-1]);print('$cfg', d['kernel_ms'], d['ms_per_step'], d['redo_pixels'])"
done
