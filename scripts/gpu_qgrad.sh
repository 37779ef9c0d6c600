#!/bin/bash
# quality gradient kernel: threads per workgroup A/B (configs[1], kernel stats)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/qgrad
mkdir -p $O
for T in 64 128 256 64 128 256; do
  SG_QGRAD_THREADS=$T timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$T -o run -- python3 bench.py --workload register-mean --steps 3 --warmup 1 --no-cpu-baseline > $O/t$T.log 2>&1 || { echo "t$T failed"; tail -5 $O/t$T.log; exit 3; }
  python3 -c "
import csv
for r in csv.DictReader(open('$O/t$T/run_kernel_stats.csv')):
    if r['Name'].startswith('k_quality_grad'): print('T=$T', r['Calls'], float(r['AverageNs'])/1e3, 'us')
"
done
