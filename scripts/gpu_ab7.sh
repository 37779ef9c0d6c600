#!/bin/bash
# A/B of k_stack_hist builds (register buffers per wave), same box, 10 steps each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab7
run() { local n=$1 lib=$2 d=$3
  SG_LIB_PATH=$lib SG_HIST_DBG=$d timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab7/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab7/$n.log; exit 3; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab7/$n.log').read().splitlines()[-1]);print('$n', d['kernel_ms'], d['ms_per_step'])"
}
for v in lib lib_ab2 lib_ab4; do
  run full_$v siril-0.9_amd/$v/libsirilgpu.so 0
  run lo_$v siril-0.9_amd/$v/libsirilgpu.so 3
done
run full_lib_again siril-0.9_amd/lib/libsirilgpu.so 0
