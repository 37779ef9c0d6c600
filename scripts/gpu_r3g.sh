#!/bin/bash
# kernel profile of the normalised (additive-scaling) SIGMA stack
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r3g}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --normalize additive-scaling > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 4; }
cut -c1-170 $O/prof/run_kernel_stats.csv
