#!/bin/bash
# round-1 first GPU pass: parity tests, short bench, kernel-trace profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== host"; (nproc; lscpu | grep -E 'Model name|^CPU\(s\)|Thread|Socket') > gpurun_out/host.txt 2>&1
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
echo "== pytest gpu"
timeout -k 10 420 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== bench"
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 3; }
cat gpurun_out/bench.log
echo "== rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof.log; exit 4; }
find gpurun_out/prof -name '*stats*' | head
