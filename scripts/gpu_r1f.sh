#!/bin/bash
# Round-1 evidence pass: GPU parity tests, bench (with CPU baseline), kernel-trace stats,
# FETCH_SIZE / WRITE_SIZE traffic of the dominant kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r1f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r1f/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r1f/pytest_gpu.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc_traffic.sh > gpurun_out/r1f/traffic.log 2>&1 || { echo traffic failed; cat gpurun_out/r1f/traffic.log; exit 5; }
cp gpurun_out/traffic/traffic_sigma_512x4096x4096.json profiles/ && cat profiles/traffic_sigma_512x4096x4096.json
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/r1f/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/r1f/bench.log; exit 3; }
grep '^{' gpurun_out/r1f/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1f/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r1f/prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/r1f/prof.log; exit 4; }
cat gpurun_out/r1f/prof/run_kernel_stats.csv
