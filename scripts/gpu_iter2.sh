#!/bin/bash
# iteration pass: GPU parity tests, then bench + finish ablation
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/it
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/it/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/it/pytest_gpu.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
run() { # name dbg extra-args
  local n=$1 d=$2; shift 2
  SG_HIST_DBG=$d timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/it/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/it/$n.log; exit 3; }
  python3 -c "import json;d=json.loads(open('gpurun_out/it/$n.log').read().splitlines()[-1]);print('$n', d['kernel_ms'], d['ms_per_step'], d['redo_pixels'], d['roofline']['frac'])"
}
run full 0
run prefix_only 1
run no_finish 2
run loads_only 3

