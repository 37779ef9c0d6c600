#!/bin/bash
# HBM traffic of the bench's dominant kernel: one FETCH_SIZE and one WRITE_SIZE pass (each its
# own rocprofv3 run, MI355X_MICROARCH.md), parsed into profiles/traffic_<workload>.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/traffic/$grp -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/traffic/$grp.log 2>&1 || { echo "pmc $grp failed"; tail -5 gpurun_out/traffic/$grp.log; exit 5; }
done
python3 scripts/pmc_traffic.py gpurun_out/traffic/FETCH_SIZE gpurun_out/traffic/WRITE_SIZE k_stack_hist gpurun_out/traffic/traffic_sigma_512x4096x4096.json
