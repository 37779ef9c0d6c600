#!/bin/bash
# k_stack_hist phase breakdown for both tile widths: loads only (dbg 3), build without the
# finish (dbg 2), build + prefix (dbg 1), full (dbg 0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r2g}
mkdir -p $O
for ni in 2 1; do
  for dbg in 3 2 1 0; do
    SG_HIST_NI=$ni SG_HIST_DBG=$dbg timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/b_ni${ni}_d$dbg.log 2>&1 || { echo bench failed; tail -20 $O/b_ni${ni}_d$dbg.log; exit 3; }
    echo "NI=$ni dbg=$dbg $(grep '^{' $O/b_ni${ni}_d$dbg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel_ms"])')"
  done
done
