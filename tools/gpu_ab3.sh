#!/bin/bash
# A/B on the GPU: kernel-5 parity tests on the working tree, then bench.py alternating
# the working tree (new) and ab/$BASE/lib (base), three times each, 20 steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-ab3}; mkdir -p $O; export TMPDIR=/tmp
BASE=${BASE:-head}
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_maze.py tests/test_gpu_edge.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 $O/tests.log
for i in $(seq 1 ${PAIRS:-3}); do
  for v in new base; do
    if [ $v = base ]; then export DYMU_LIBDIR=$GRAFT_REPO_ROOT/ab/$BASE/lib; else unset DYMU_LIBDIR; fi
    if [ $v = new ]; then ENVV="${NEW_ENV:-X_=0}"; else ENVV="X_=0"; fi
    env $ENVV timeout -k 10 300 python -u bench.py --no-planner --no-variants --cpu-sample 0 --sustain-s 0 --steps 20 --warmup 3 > $O/bench_$v$i.log 2>&1 || { tail -20 $O/bench_$v$i.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_$v$i.log').read().strip().splitlines()[-1]); print('$v$i', d['ms_per_step'], d['config']['passes_per_solve'], d['config']['tile_visits_per_solve'], d['config']['inner_sweeps_per_solve'], d['roofline']['avg_launch_us'])"
  done
done
