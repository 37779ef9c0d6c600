#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab4
run() { local n=$1 d=$2; shift 2
  SG_HIST_DBG=$d timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/ab4/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab4/$n.log; exit 3; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab4/$n.log').read().splitlines()[-1]);print('$n', d['kernel_ms'], d['ms_per_step'], d['redo_pixels'])"
}
run full 0
run full_voff 10
run loads_only 3
run no_finish 2
