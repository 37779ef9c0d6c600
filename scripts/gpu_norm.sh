#!/bin/bash
# normalised stacks on the histogram path: GPU parity tests, then the sigma workload timed
# without / with normalisation
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/norm
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
for nm in none additive-scaling multiplicative-scaling; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --normalize $nm > $O/b_$nm.log 2>&1 || { tail -5 $O/b_$nm.log; exit 3; }
  echo "$nm $(grep -o '"ms_per_step": [0-9.]*' $O/b_$nm.log) $(grep -o '"kernel_ms": [0-9.]*' $O/b_$nm.log) $(grep -o '"redo_pixels": [0-9]*' $O/b_$nm.log) $(grep -o '"slow_pixels": [0-9]*' $O/b_$nm.log)"
done
