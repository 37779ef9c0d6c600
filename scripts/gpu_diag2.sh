#!/bin/bash
# k_stack_hist ablations: prefix-only finish, loads-only vs shift alignment
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
run() { # name dbg extra-args
  local n=$1 d=$2; shift 2
  SG_HIST_DBG=$d timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/diag/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/diag/$n.log; exit 3; }
  python3 -c "import json;d=json.loads(open('gpurun_out/diag/$n.log').read().splitlines()[-1]);print('$n', d['kernel_ms'], d['ms_per_step'], d['redo_pixels'])"
}
run full 0
run prefix_only 1
run no_finish 2
run loads_only 3
run loads_only_noshift 3 --maxshift 0
run loads_only_even 3 --even-shifts
run loads_only_noy 3 --zero-shift y
run full_noshift 0 --maxshift 0
run full_pad 0 --frame-pad 4096
