#!/bin/bash
# registration FFT: raised wave priority for the memory-reading first pass (lib_abp, built
# with -DSG_FFT_PRIO) vs the default build; configs[1] bench, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/fprio
mkdir -p $O
for r in 1 2 3; do
  for v in lib lib_abp; do
    SG_LIB_PATH=siril-0.9_amd/$v/libsirilgpu.so timeout -k 10 300 python bench.py --workload register-mean --steps 5 --warmup 2 --no-cpu-baseline > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 3; }
    echo "$v: $(grep '^{' $O/$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms"]["register"], d["register_shifts_exact"])')"
  done
done
