#!/bin/bash
# k_stack_hist sensitivity: finish chain length (sigma twice), occupancy (LDS pad -> 3 blocks/CU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
run() { # name dbg pad extra-args
  local n=$1 d=$2 pad=$3; shift 3
  SG_HIST_LDSPAD=$pad SG_HIST_DBG=$d timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/diag/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/diag/$n.log; exit 3; }
  python3 -c "import json;d=json.loads(open('gpurun_out/diag/$n.log').read().splitlines()[-1]);print('$n', d['kernel_ms'], d['ms_per_step'], d['redo_pixels'])"
}
run full 0 0
run sigma_twice 9 0
run full_3blk 0 6144
run noload_3blk 3 6144
run nofin_3blk 2 6144
