#!/bin/bash
# WINSORIZED histogram finish: 2 waves x 64 lanes (default) vs 4 waves x 32 lanes (dbg 20),
# configs[4] at one GPU; parity of the dbg 20 variant via the hist-path GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/wab
mkdir -p $O
SG_HIST_DBG=20 timeout -k 10 300 python -u -m pytest tests/test_gpu_stack.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "hist and 4" > $O/pytest.log 2>&1
rc=$?; echo "pytest(dbg20) rc=$rc"; tail -2 $O/pytest.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for d in 0 20; do
    SG_HIST_DBG=$d timeout -k 10 300 python bench.py --workload winsorized-rgb --steps 3 --warmup 1 --no-cpu-baseline > $O/d$d.log 2>&1 || { echo "d$d failed"; tail -5 $O/d$d.log; exit 3; }
    echo "dbg=$d: $(grep '^{' $O/d$d.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms"])')"
  done
done
