#!/bin/bash
# iteration pass: GPU tests, bench, kernel stats, instruction-mix counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log | cut -c1-400
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 3; }
cat gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof.log; exit 4; }
cat gpurun_out/prof/run_kernel_stats.csv
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVES --output-format csv -d gpurun_out/pmc_i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_i.log 2>&1 || { echo pmc failed; exit 5; }
grep k_stack_hist gpurun_out/pmc_i/run_counter_collection.csv | awk -F, '{print $(NF-3), $(NF-2)}'
