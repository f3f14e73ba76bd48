#!/bin/bash
# GPU sweep of engine environment knobs: quick kernel-5 parity tests on the
# working tree, then bench.py once per configuration in $CONFIGS (";"-separated
# lists of VAR=value pairs; "base" = ab/$BASE/lib, "-" = defaults), twice over.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
BASE=${BASE:-base}
CONFIGS=${CONFIGS:-"-;base"}
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_fullsize.py tests/test_gpu_edge.py -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/sw_tests.log 2>&1 || { tail -40 gpurun_out/sw_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/sw_tests.log
IFS=';' read -ra CFG <<< "$CONFIGS"
for i in 1 2; do
  n=0
  for cfg in "${CFG[@]}"; do
    n=$((n + 1))
    envs=()
    if [ "$cfg" = base ]; then envs=("DYMU_LIBDIR=$GRAFT_REPO_ROOT/ab/$BASE/lib");
    elif [ "$cfg" != - ]; then read -ra envs <<< "$cfg"; fi
    log=gpurun_out/sw_${n}_$i.log
    timeout -k 10 300 env "${envs[@]}" python -u bench.py --no-planner --cpu-sample 0 --steps 10 --warmup 2 ${BENCH_ARGS} > $log 2>&1 || { tail -20 $log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('[$cfg] run $i', d['ms_per_step'], d['config']['passes_per_solve'], d['roofline']['launches_per_solve'] if d['roofline'] else None, d['roofline']['avg_launch_us'] if d['roofline'] else None)"
  done
done
