#!/bin/bash
# half-spectrum registration: column strip width A/B (configs[1] bench + kernel stats)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/rhcw
mkdir -p $O
for CW in 4 2 1 8; do
  SG_REG_CW=$CW timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cw$CW -o run -- python3 bench.py --workload register-mean --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_cw$CW.log 2>&1 || { echo bench failed; tail -20 $O/bench_cw$CW.log; exit 3; }
  echo "CW $CW: $(grep '^{' $O/bench_cw$CW.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms"]["register"], d["register_shifts_exact"])')"
  python3 -c "
import csv
for r in csv.DictReader(open('$O/cw$CW/run_kernel_stats.csv')):
    n=r['Name'].split('(')[0]
    if n.startswith('k_reg'): print('   %-30s %5s %8.1f us' % (n, r['Calls'], float(r['AverageNs'])/1e3))
"
done
