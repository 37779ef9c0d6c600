#!/bin/bash
# general replay loop with register chunks for N <= 512 (replay_pixel<8>): GPU tests, configs[4]
# A/B against HEAD before (lib_ab3), replay kernel time from rocprofv3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4r}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
L=$PWD/siril-0.9_amd
for v in new old; do
  E=""; [ $v = old ] && E="SG_LIB_PATH=$L/lib_ab3/libsirilgpu.so"
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 bench.py --workload winsorized-rgb --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_$v.log 2>&1 || { echo "prof $v failed"; tail -20 $O/prof_$v.log; exit 3; }
  echo "$v $(grep '^{' $O/prof_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms"])')"
  grep -h "replay" $O/prof_$v/run_kernel_stats.csv | cut -c1-120
done
