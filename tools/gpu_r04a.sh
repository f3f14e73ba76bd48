#!/bin/bash
# Round 4, monotone combine (v32): the arithmetic and maze parity tests, then the
# headline bench and the 16384^2 maze against the v31 build (ab/v31/lib), twice each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_maze.py -x -v -s \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|maze16384" $O/tests.log | tail -5
for i in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export DYMU_LIBDIR=$GRAFT_REPO_ROOT/ab/v31/lib; else unset DYMU_LIBDIR; fi
    timeout -k 10 300 python -u bench.py --no-planner --cpu-sample 0 --no-variants --steps 10 --warmup 2 > $O/bench_$v$i.log 2>&1 || { tail -20 $O/bench_$v$i.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_$v$i.log').read().strip().splitlines()[-1]); print('$v$i', d['ms_per_step'], d['config']['passes_per_solve'], d['config']['tile_visits_per_solve'], d.get('parity'))"
  done
done
for v in new base; do
  if [ $v = base ]; then export DYMU_LIBDIR=$GRAFT_REPO_ROOT/ab/v31/lib; else unset DYMU_LIBDIR; fi
  timeout -k 10 600 python tools/maze_bench.py 16384 64 2 > $O/maze16384_$v.json 2> $O/maze16384_$v.err || { tail $O/maze16384_$v.err; exit 1; }
  echo "$v $(cat $O/maze16384_$v.json)"
done
