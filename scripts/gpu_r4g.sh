#!/bin/bash
# k_stack_replay kernel time: HEAD before (lib_ab3) vs the fast SIGMA passes + batched gather +
# compact sort loops, from rocprofv3 kernel traces; then the replay probe (SG_HIST_DBG=12)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4g}
mkdir -p $O
L=$PWD/siril-0.9_amd
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_new -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/prof_new.log 2>&1 || { echo "prof new failed"; tail -20 $O/prof_new.log; exit 3; }
SG_LIB_PATH=$L/lib_ab3/libsirilgpu.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_old -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/prof_old.log 2>&1 || { echo "prof old failed"; tail -20 $O/prof_old.log; exit 3; }
for v in new old; do echo "$v: $(find $O/prof_$v -name '*kernel_stats.csv' | xargs grep -h 'replay\|k_stack_hist' | cut -c1-160)"; done
SG_HIST_DBG=12 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/replay_prof.log 2>&1 || { echo "replay prof failed"; tail -20 $O/replay_prof.log; exit 3; }
grep -a "replay" $O/replay_prof.log | tail -2
