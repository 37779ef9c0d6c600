#!/bin/bash
# k_stack_hist time breakdown with the raised build priority: loads only (dbg 3), loads +
# binning (dbg 2), + prefix without the pass loop (dbg 1), full (0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/hbd
for r in 1 2; do
  for d in 3 2 1 0; do
    SG_HIST_DBG=$d timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/hbd/d${d}_$r.log 2>&1 || { echo "dbg $d failed"; tail -5 gpurun_out/hbd/d${d}_$r.log; exit 3; }
    python3 -c "import json;d=json.loads(open('gpurun_out/hbd/d${d}_$r.log').read().splitlines()[-1]);print('dbg $d', d['kernel_ms'])"
  done
done
