#!/bin/bash
# half-spectrum registration (3 plane passes) vs the 4-pass order: GPU registration tests,
# configs[1] bench A/B, kernel stats of the new order
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/rh
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_register.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_reg.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_reg.log | cut -c1-300
[ $rc -eq 0 ] || { grep -E 'Error|assert|FAIL' $O/pytest_reg.log | head -20; exit $rc; }
for P in 2 2; do
  SG_REG_PATH=$P timeout -k 10 300 python bench.py --workload register-mean --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_p$P.log 2>&1 || { echo bench failed; tail -20 $O/bench_p$P.log; exit 3; }
  echo "path $P: $(grep '^{' $O/bench_p$P.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms"], d["register_shifts_exact"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload register-mean --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 4; }
cut -d, -f1-4 $O/prof/run_kernel_stats.csv
