#!/bin/bash
# column-pass strip mapping A/B: parity for both column kernels, kernel times for
# (persistent, xcd-map) combos, FETCH_SIZE per column kernel with and without the map
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/rx; mkdir -p $O
for p in 1 0; do
SG_REG_PERSIST=$p timeout -k 10 300 python -u -m pytest tests/test_gpu_register.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_p$p.log 2>&1
rc=$?; echo "pytest persist=$p rc=$rc"; tail -1 $O/pytest_p$p.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
done
for p in 1 0; do for x in 1 0; do
SG_REG_PERSIST=$p SG_REG_XCD=$x timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$p$x -o run -- python3 bench.py --workload register-mean --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_k$p$x.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_k$p$x.log; exit 3; }
grep '^{' $O/bench_k$p$x.log | cut -c100-190
done; done
for x in 1 0; do
SG_REG_PERSIST=0 SG_REG_XCD=$x timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$x -o run -- python3 bench.py --workload register-mean --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_f$x.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc_f$x.log; exit 4; }
done
echo done
