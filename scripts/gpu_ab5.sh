#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab5
run() { local n=$1 d=$2 g=$3; shift 3
  SG_HIST_GRID=$g SG_HIST_DBG=$d timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/ab5/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab5/$n.log; exit 3; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab5/$n.log').read().splitlines()[-1]);print('$n', d['kernel_ms'], d['ms_per_step'], d['redo_pixels'])"
}
python3 -c "
import ctypes; h=ctypes.CDLL('libamdhip64.so')
" 
for g in 512 1024 1536 2048 4096 131072; do run full_g$g 0 $g; done
for g in 1024 2048 131072; do run lo_g$g 3 $g; done
