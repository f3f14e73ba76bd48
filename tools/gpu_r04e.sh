#!/bin/bash
# Round 4: sparse passes (k_fim_sparse) -- the barrier probe, parity
# with every pass forced sparse, the maze and the headline with and without them, the
# dense kernel after the pass-body refactor against HEAD's build (ab/head), the
# exact-tie early-exit tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04e; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 ./tools/barrier_probe3 4000 > $O/barrier_probe3.log 2>&1 || { cat $O/barrier_probe3.log; exit 1; }
cat $O/barrier_probe3.log
DYMU_SPARSE_MAX=1000000000 timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py -x -q --timeout 120 --timeout-method thread > $O/sparse_forced_tests.log 2>&1 || { tail -40 $O/sparse_forced_tests.log; exit 1; }
tail -2 $O/sparse_forced_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py -x -v --timeout 120 --timeout-method thread > $O/sparse_tests.log 2>&1 || { tail -40 $O/sparse_tests.log; exit 1; }
tail -3 $O/sparse_tests.log
DYMU_SPARSE_MAX=1000000000 timeout -k 10 600 python -u -m pytest tests/test_gpu_update.py tests/test_planner.py -x -q --timeout 120 --timeout-method thread > $O/sparse_forced_update_planner.log 2>&1 || { tail -40 $O/sparse_forced_update_planner.log; exit 1; }
tail -2 $O/sparse_forced_update_planner.log
# XCC-register selection + L1-only barrier, only if the probe saw no stale read with it
if [ "$(grep -c 'xcc0-reg.*flags 0' $O/barrier_probe3.log)" = "8" ]; then
  DYMU_SPARSE_XCC=1 DYMU_SPARSE_FENCE=0 DYMU_SPARSE_MAX=1000000000 timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_sparse.py -x -q --timeout 120 --timeout-method thread > $O/sparse_xcc_tests.log 2>&1 || { tail -40 $O/sparse_xcc_tests.log; exit 1; }
  tail -2 $O/sparse_xcc_tests.log
  for v in 256 1024; do
    DYMU_SPARSE_XCC=1 DYMU_SPARSE_FENCE=0 DYMU_SPARSE_MAX=$v timeout -k 10 300 python tools/maze_bench.py 4096 64 3 > $O/maze4096_xcc$v.json 2>&1 || { tail $O/maze4096_xcc$v.json; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/maze4096_xcc$v.json').read().strip().splitlines()[-1]); print('maze4096 xcc sparse_max=$v', d['ms_per_solve'], d['passes'], d['launches'], d['tile_visits'], d['parity'])"
  done
fi
for v in 0 256 1024; do
  DYMU_SPARSE_MAX=$v timeout -k 10 300 python tools/maze_bench.py 4096 64 3 > $O/maze4096_s$v.json 2>&1 || { tail $O/maze4096_s$v.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/maze4096_s$v.json').read().strip().splitlines()[-1]); print('maze4096 sparse_max=$v', d['ms_per_solve'], d['passes'], d['launches'], d['tile_visits'], d['parity'])"
done
DYMU_SPARSE_MAX=1024 timeout -k 10 300 python tools/maze_bench.py 16384 64 1 > $O/maze16384_s1024.json 2>&1 || { tail $O/maze16384_s1024.json; exit 1; }
python3 -c "import json; d=json.loads(open('$O/maze16384_s1024.json').read().strip().splitlines()[-1]); print('maze16384 sparse_max=1024', d['ms_per_solve'], d['passes'], d['launches'], d['tile_visits'], d['parity'])"
for i in 1 2; do
  for v in head:0 new:0 new:256 new:1024; do
    lib=${v%%:*}; sm=${v##*:}
    if [ $lib = head ]; then export DYMU_LIBDIR=$GRAFT_REPO_ROOT/ab/head/lib; else unset DYMU_LIBDIR; fi
    DYMU_SPARSE_MAX=$sm timeout -k 10 300 python -u bench.py --no-planner --no-variants --cpu-sample 0 --steps 10 --warmup 2 > $O/bench_${lib}_$sm.$i.log 2>&1 || { tail -20 $O/bench_${lib}_$sm.$i.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${lib}_$sm.$i.log').read().strip().splitlines()[-1]); print('bench $v.$i', d['ms_per_step'], d['config']['passes_per_solve'], d['config'].get('launches_per_solve'), d['roofline']['avg_launch_us'] if d['roofline'] else None)"
  done
done
unset DYMU_LIBDIR
timeout -k 10 300 python -u -m pytest tests/test_planner.py -k "early_exit" -x -v --timeout 120 --timeout-method thread > $O/early_exit_tests.txt 2>&1 || { tail -30 $O/early_exit_tests.txt; exit 1; }
tail -3 $O/early_exit_tests.txt
