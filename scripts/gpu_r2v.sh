#!/bin/bash
# GPU tests + bench at HEAD (half-block build for NI = 1, fast sigma)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r2v}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 && grep '^{' $O/bench.log | cut -c1-400
