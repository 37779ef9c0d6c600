#!/bin/bash
# fused column pass: pair blocks per strip (SG_REG_PB) so the reference-spectrum columns are
# re-read from L2; register tests under PB=4, then configs[1] A/B PB 1 / 2 / 4 / 8
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4n}
mkdir -p $O
SG_REG_PB=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_register.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_reg.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_reg.log; exit 3; }
tail -1 $O/pytest_reg.log
for rep in 1 2; do
  for pb in 1 2 4 8; do
    SG_REG_PB=$pb timeout -k 10 300 python bench.py --workload register-mean --steps 10 --warmup 3 --no-cpu-baseline > $O/pb${pb}_$rep.log 2>&1 || { echo "bench failed"; tail -20 $O/pb${pb}_$rep.log; exit 3; }
    echo "pb$pb $rep $(grep '^{' $O/pb${pb}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms"], d["register_shifts_exact"])')"
  done
done
