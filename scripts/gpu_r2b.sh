#!/bin/bash
# round 2: GPU tests (incl. row bands), then the default bench once
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r2b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest_gpu.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 3; }
grep '^{' $O/bench.log
