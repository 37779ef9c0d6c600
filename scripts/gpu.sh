#!/bin/bash
# The one GPU runner (replaces round 1/2's per-experiment launchers; they live in git history
# before round 3).  Run on the box through gpurun:
#   gpurun --timeout 900 -- 'bash scripts/gpu.sh OUT STEP [STEP ...]'
# Results go to gpurun_out/OUT/.  Steps run in order; the first failing step ends the run
# (no GPU step runs after a fault, an abort or a time limit).
#   test[=K]                    pytest -m gpu (optionally -k K), per-test timeout 200 s
#   testall[=K]                 the same, going on past assertion failures (at most 8)
#   smoke                       __graft_entry__.smoke()
#   bench=NAME[:ARGS]           python bench.py ARGS -> NAME.log + one summary line
#   env=NAME:VAR=V[;VAR=V]:ARGS the same with an environment (A/B: SG_* knobs, SG_LIB_PATH)
#   prof=NAME[:ARGS]            rocprofv3 --kernel-trace --stats of bench.py ARGS -> NAME/
#   pmc=NAME[@K1,K2][:ARGS]     FETCH_SIZE and WRITE_SIZE passes (own runs) -> NAME_traffic.json
#                               (kernels K: default $PMC_KERNEL or k_stack_hist; several = per-step totals)
#   sq=NAME:CTRS[:ARGS]         one rocprofv3 --pmc pass with counters CTRS ('+' between them,
#                               within the per-block slot limits) -> NAME.txt (pmc_sum.py)
#   py=NAME:SCRIPT[:ARGS]       python SCRIPT ARGS -> NAME.log
#   bin=NAME:EXE[:ARGS]         a built probe (tools/), 300 s limit -> NAME.log
#   dist=NAME:NPROC[:ARGS]      bench.py under torchrun with NPROC ranks on this one GPU
#                               (SG_BENCH_REHEARSE=1: gloo collectives; a rehearsal of the multi-GPU flow)
# ARGS use ',' between words (bench=cfg1:--workload,register-mean).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:?output directory}
shift
mkdir -p "$O"

fail() { echo "FAILED: $1"; [ -f "$2" ] && tail -30 "$2"; exit 3; }
summary() {
  grep '^{' "$1" | tail -1 | python3 -c 'import json,sys
d=json.loads(sys.stdin.read())
r=d.get("roofline",{})
print(d.get("value"), d.get("unit"), "ms/step", d.get("ms_per_step"), "kernel", d.get("kernel_ms", d.get("stage_ms")), "frac", r.get("frac"))'
}

for step in "$@"; do
  kind=${step%%=*}
  spec=${step#*=}
  [ "$kind" = "$step" ] && spec=""
  case $kind in
    test|testall)
      k=(); [ -n "$spec" ] && k=(-k "${spec//,/ }")   # commas between the words of a -k expression
      x=-x; [ "$kind" = testall ] && x=--maxfail=8
      lim=900; [ -n "$spec" ] && lim=600     # a selection runs under a shorter limit
      timeout -k 10 $lim python -u -m pytest tests -m gpu $x -v --durations=15 --timeout 200 --timeout-method thread "${k[@]}" \
        > "$O/pytest_gpu.log" 2>&1; rc=$?
      # testall goes on after plain test failures (pytest exit 1), never after a crash or a timeout
      if [ $rc -ne 0 ] && { [ "$kind" = test ] || [ $rc -ne 1 ]; }; then fail test "$O/pytest_gpu.log"; fi
      grep -E "^(FAILED|ERROR)" "$O/pytest_gpu.log"; tail -1 "$O/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || fail smoke "$O/smoke.log"
      tail -1 "$O/smoke.log" ;;
    bench)
      name=${spec%%:*}; args=""; [ "$name" != "$spec" ] && args=${spec#*:}
      timeout -k 10 600 python bench.py ${args//,/ } > "$O/$name.log" 2>&1 || fail "bench $name" "$O/$name.log"
      echo "$name: $(summary "$O/$name.log")" ;;
    env)
      name=${spec%%:*}; rest=${spec#*:}; vars=${rest%%:*}; args=""; [ "$vars" != "$rest" ] && args=${rest#*:}
      timeout -k 10 600 env ${vars//;/ } python bench.py ${args//,/ } > "$O/$name.log" 2>&1 || fail "env $name" "$O/$name.log"
      echo "$name: $(summary "$O/$name.log")" ;;
    prof)
      name=${spec%%:*}; args=""; [ "$name" != "$spec" ] && args=${spec#*:}
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$name" -o run -- \
        python3 bench.py ${args//,/ } > "$O/$name.log" 2>&1 || fail "prof $name" "$O/$name.log"
      echo "$name: $(summary "$O/$name.log")" ;;
    pmc)
      name=${spec%%:*}; args=""; [ "$name" != "$spec" ] && args=${spec#*:}
      kern=${PMC_KERNEL:-k_stack_hist}; [ "${name#*@}" != "$name" ] && { kern=${name#*@}; name=${name%%@*}; }
      for grp in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$O/${name}_$grp" -o run -- \
          python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${args//,/ } > "$O/${name}_$grp.log" 2>&1 \
          || fail "pmc $grp" "$O/${name}_$grp.log"
      done
      python3 scripts/pmc_traffic.py "$O/${name}_FETCH_SIZE" "$O/${name}_WRITE_SIZE" "$kern" \
        "$O/${name}_traffic.json" ${PMC_STEPS:-1} || fail "pmc parse" ;;
    sq)
      name=${spec%%:*}; rest=${spec#*:}; ctrs=${rest%%:*}; args=""; [ "$ctrs" != "$rest" ] && args=${rest#*:}
      timeout -s KILL 180 rocprofv3 --pmc ${ctrs//+/ } --output-format csv -d "$O/$name" -o run -- \
        python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline ${args//,/ } > "$O/$name.log" 2>&1 \
        || fail "sq $name" "$O/$name.log"
      python3 scripts/pmc_sum.py "$O/$name" "${PMC_KERNEL:-k_stack}" > "$O/$name.txt" || fail "sq parse"
      cat "$O/$name.txt" ;;
    dist)
      name=${spec%%:*}; rest=${spec#*:}; np=${rest%%:*}; args=""; [ "$np" != "$rest" ] && args=${rest#*:}
      SG_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$np" \
        --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus "$np" ${args//,/ } > "$O/$name.log" 2>&1 \
        || fail "dist $name" "$O/$name.log"
      echo "$name: $(summary "$O/$name.log")" ;;
    py)
      name=${spec%%:*}; rest=${spec#*:}; script=${rest%%:*}; args=""; [ "$script" != "$rest" ] && args=${rest#*:}
      timeout -k 10 900 python -u "$script" ${args//,/ } > "$O/$name.log" 2>&1 || fail "py $name" "$O/$name.log"
      tail -3 "$O/$name.log" ;;
    bin)
      name=${spec%%:*}; rest=${spec#*:}; exe=${rest%%:*}; args=""; [ "$exe" != "$rest" ] && args=${rest#*:}
      timeout -k 10 300 "$exe" ${args//,/ } > "$O/$name.log" 2>&1 || fail "bin $name" "$O/$name.log"
      tail -40 "$O/$name.log" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps ok"
