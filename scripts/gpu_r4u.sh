#!/bin/bash
# default bench x3 (regression check of configs[2])
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4u}
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_$rep.log 2>&1 || { echo "bench failed"; tail -20 $O/b_$rep.log; exit 3; }
  echo "b_$rep $(grep '^{' $O/b_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
done
