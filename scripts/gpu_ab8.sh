#!/bin/bash
# A/B of k_stack_hist builds with the build phase at raised priority: 2 vs 3 register
# buffers per wave (configs[2] bench, same box, 10 steps each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab8
run() { local n=$1 lib=$2
  SG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab8/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab8/$n.log; exit 3; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab8/$n.log').read().splitlines()[-1]);print('$n', d['kernel_ms'], d['ms_per_step'])"
}
for r in 1 2 3; do
  for v in lib lib_ab3; do
    run ${v}_$r siril-0.9_amd/$v/libsirilgpu.so || exit 3
  done
done
