#!/bin/bash
# half-spectrum registration: pairs per launch A/B (configs[1] bench)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/rb
mkdir -p $O
for r in 1 2; do
  for B in 1 2 4 16 32 64; do
    SG_REG_BATCH=$B timeout -k 10 300 python bench.py --workload register-mean --steps 5 --warmup 2 --no-cpu-baseline > $O/b$B.log 2>&1 || { echo bench failed; tail -20 $O/b$B.log; exit 3; }
    echo "B=$B: $(grep '^{' $O/b$B.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms"]["register"], d["register_shifts_exact"])')"
  done
done
