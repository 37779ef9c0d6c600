#!/bin/bash
# border-row normalised zeros on the histogram path (SIGMA, additive normalisation): GPU tests,
# then the additive-scaling bench x2 and the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4i}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --normalize additive-scaling --steps 10 --warmup 5 --no-cpu-baseline > $O/norm_$rep.log 2>&1 || { echo "norm bench failed"; tail -20 $O/norm_$rep.log; exit 3; }
  echo "norm_$rep $(grep '^{' $O/norm_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
done
timeout -k 10 300 python bench.py --steps 10 --warmup 5 --no-cpu-baseline > $O/sigma.log 2>&1 || { echo "bench failed"; tail -20 $O/sigma.log; exit 3; }
echo "sigma $(grep '^{' $O/sigma.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
