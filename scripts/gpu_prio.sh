#!/bin/bash
# histogram path: wave priority of the build phase A/B (configs[2] bench, kernel time)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/prio
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stack.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k hist > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
for P in 1 4 1 4 1 4; do
  SG_HIST_PRIO=$P timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/p$P.log 2>&1 || { echo "p$P failed"; tail -5 $O/p$P.log; exit 3; }
  echo "prio=$P: $(grep '^{' $O/p$P.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"])')"
done
