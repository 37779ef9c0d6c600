#!/bin/bash
# round 2: GPU tests, then the default bench with both histogram tile widths (SG_HIST_NI 2 / 1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r2c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest_gpu.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
for ni in 2 1 2 1; do
  SG_HIST_NI=$ni timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_ni$ni.log 2>&1 || { echo bench failed; tail -20 $O/bench_ni$ni.log; exit 3; }
  echo "NI=$ni $(grep '^{' $O/bench_ni$ni.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["redo_pixels"])')"
done
for ni in 2 1; do
  SG_HIST_NI=$ni SG_HIST_DBG=3 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_lo_ni$ni.log 2>&1 || { echo bench failed; tail -20 $O/bench_lo_ni$ni.log; exit 3; }
  echo "loads-only NI=$ni $(grep '^{' $O/bench_lo_ni$ni.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel_ms"])')"
done
