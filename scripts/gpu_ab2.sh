#!/bin/bash
# A/B: aligned (no shifts) vs shifted loads
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "3 0" "3 16" "0 0" "0 16"; do
  set -- $cfg
  SG_HIST_DBG=$1 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --maxshift $2 > gpurun_out/ab2_$1_$2.log 2>&1 || { echo "ab $cfg failed"; tail -5 gpurun_out/ab2_$1_$2.log; exit 3; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab2_$1_$2.log').read().splitlines()[-1]);print('dbg=$1 maxshift=$2', d['kernel_ms'], d['ms_per_step'], d['roofline']['achieved'], d['redo_pixels'])"
done
