#!/bin/bash
# occupancy sensitivity of k_stack_hist: LDS pad -> 3 / 2 workgroups per CU, per debug mode
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab6
run() { local n=$1 d=$2 pad=$3; shift 3
  SG_HIST_LDSPAD=$pad SG_HIST_DBG=$d timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ab6/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab6/$n.log; exit 3; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab6/$n.log').read().splitlines()[-1]);print('$n', d['kernel_ms'], d['ms_per_step'])"
}
for pad in 0 6144 45000; do
  run full_p$pad 0 $pad
  run nofin_p$pad 2 $pad
  run lo_p$pad 3 $pad
done
