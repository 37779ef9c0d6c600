#!/bin/bash
# registration FFT iteration: register parity tests, then register-mean under kernel trace (A/B knob SG_REG_PERSIST)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/rp
timeout -k 10 300 python -u -m pytest tests/test_gpu_register.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/rp/pytest_reg.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/rp/pytest_reg.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
for p in 1 0; do
SG_REG_PERSIST=$p timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp/k$p -o run -- python3 bench.py --workload register-mean --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rp/bench_k$p.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/rp/bench_k$p.log; exit 3; }
SG_REG_PERSIST=$p timeout -k 10 200 python3 bench.py --workload register-mean --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/rp/bench_k${p}_plain.log 2>&1 || { echo "bench failed"; exit 3; }
grep '^{' gpurun_out/rp/bench_k${p}_plain.log | cut -c1-200
done
