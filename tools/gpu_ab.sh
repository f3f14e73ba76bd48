#!/bin/bash
# A/B on the GPU: quick kernel-5 parity tests on the working tree, then bench.py
# alternating the working tree (new) and ab/$BASE/lib (base), twice each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
BASE=${BASE:-base}
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_fullsize.py tests/test_gpu_edge.py -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/ab_tests.log
for i in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export DYMU_LIBDIR=$GRAFT_REPO_ROOT/ab/$BASE/lib; else unset DYMU_LIBDIR; fi
    timeout -k 10 300 python -u bench.py --no-planner --cpu-sample 0 --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/ab_$v$i.log 2>&1 || { tail -20 gpurun_out/ab_$v$i.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v$i.log').read().strip().splitlines()[-1]); print('$v$i', d['ms_per_step'], d['config']['passes_per_solve'], d['config']['tile_visits_per_solve'], d['roofline']['avg_launch_us'] if d['roofline'] else None)"
  done
done
