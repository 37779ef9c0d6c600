#!/bin/bash
# Round-1 evidence pass: GPU parity tests, bench (with CPU baseline), kernel-trace stats,
# FETCH_SIZE / WRITE_SIZE passes over one bench step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log | cut -c1-400
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 3; }
cat gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof.log; exit 4; }
cat gpurun_out/prof/run_kernel_stats.csv
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_$grp -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_$grp.log 2>&1 || { echo "pmc $grp failed"; tail -5 gpurun_out/pmc_$grp.log; exit 5; }
  grep k_stack gpurun_out/pmc_$grp/run_counter_collection.csv | awk -F, '{print $(NF-1), $NF}'
done
