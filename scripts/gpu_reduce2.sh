#!/bin/bash
# pixel-pair reduce kernel: GPU stacking tests, configs[1] bench A/B (old kernel vs pairs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/red2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log | cut -c1-300
[ $rc -eq 0 ] || { grep -E 'Error|assert|FAIL' $O/pytest.log | head -20; exit $rc; }
for R in 1 0 1 0; do
  SG_REDUCE1=$R timeout -k 10 300 python bench.py --workload register-mean --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_r$R.log 2>&1 || { echo bench failed; tail -20 $O/bench_r$R.log; exit 3; }
  echo "reduce1=$R: $(grep '^{' $O/bench_r$R.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms"], d["roofline"]["achieved"], d["register_shifts_exact"])')"
done
