#!/bin/bash
# Evidence pass (output dir = $1): GPU parity tests, smoke, the three bench workloads (default
# one with the CPU baseline, as the driver runs it), kernel-trace stats, FETCH_SIZE / WRITE_SIZE
# traffic of the dominant kernel, and a 2-rank rehearsal of the multi-GPU flow on one GPU (gloo)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_gpu.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 9; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 3; }
grep '^{' $O/bench.log | cut -c1-700
timeout -k 10 300 python bench.py --workload winsorized-rgb --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_wins.log 2>&1 || { echo wins bench failed; tail -20 $O/bench_wins.log; exit 6; }
timeout -k 10 300 python bench.py --workload register-mean --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_regmean.log 2>&1 || { echo regmean bench failed; tail -20 $O/bench_regmean.log; exit 7; }
timeout -k 10 300 python bench.py --normalize additive-scaling --steps 10 --warmup 5 --no-cpu-baseline > $O/bench_norm.log 2>&1 || { echo norm bench failed; tail -20 $O/bench_norm.log; exit 8; }
for f in bench_wins bench_regmean bench_norm; do echo "$f $(grep '^{' $O/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("kernel_ms"), d.get("stage_ms"))')"; done
bash scripts/gpu_pmc_traffic.sh > $O/traffic.log 2>&1 || { echo traffic failed; cat $O/traffic.log; exit 5; }
cat gpurun_out/traffic/traffic_sigma_512x4096x4096.json | tr -d '\n'; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 4; }
grep -h "k_stack_hist\|replay" $O/prof/run_kernel_stats.csv | cut -c1-200
SG_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/rehearse2.log 2>&1 || { echo rehearsal failed; tail -20 $O/rehearse2.log; exit 10; }
grep '^{' $O/rehearse2.log | cut -c1-300
