#!/bin/bash
# normalised SIGMA stack (GUI default additive + scaling) at HEAD, with its kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r2x}
mkdir -p $O
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --normalize additive-scaling > $O/bench_norm.log 2>&1 && grep '^{' $O/bench_norm.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])' || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --normalize additive-scaling > $O/prof.log 2>&1 || exit 4
cut -c1-160 $O/prof/run_kernel_stats.csv
