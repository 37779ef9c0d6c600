#!/bin/bash
# Evidence pass (output dir = $1): GPU parity tests, the three bench workloads (default one with the
# CPU baseline), kernel-trace stats, FETCH_SIZE / WRITE_SIZE traffic of the dominant kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload winsorized-rgb --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_wins.log 2>&1 || { echo wins bench failed; tail -20 $O/bench_wins.log; exit 6; }
grep '^{' $O/bench_wins.log
timeout -k 10 300 python bench.py --workload register-mean --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_regmean.log 2>&1 || { echo regmean bench failed; tail -20 $O/bench_regmean.log; exit 7; }
grep '^{' $O/bench_regmean.log
timeout -k 10 300 python bench.py --normalize additive-scaling --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_norm.log 2>&1 || { echo norm bench failed; tail -20 $O/bench_norm.log; exit 8; }
grep '^{' $O/bench_norm.log | cut -c1-600
bash scripts/gpu_pmc_traffic.sh > $O/traffic.log 2>&1 || { echo traffic failed; cat $O/traffic.log; exit 5; }
cat gpurun_out/traffic/traffic_sigma_512x4096x4096.json
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 3; }
grep '^{' $O/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 4; }
cat $O/prof/run_kernel_stats.csv
