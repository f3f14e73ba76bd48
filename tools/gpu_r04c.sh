#!/bin/bash
# Round 4: what a sparse pass costs -- grid barriers among few workgroups (one XCD vs
# spread) against the launch, and the phase trace of one serpentine-maze pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 ./tools/barrier_probe3 4000 > $O/barrier_probe3.log 2>&1 || { cat $O/barrier_probe3.log; exit 1; }
cat $O/barrier_probe3.log
DYMU_PRIO_TRACE=3000 timeout -k 10 300 python tools/maze_bench.py 4096 64 1 > $O/maze4096.json 2> $O/maze_trace.log || { tail $O/maze_trace.log; exit 1; }
python tools/trace_show.py $O/maze_trace.log
DYMU_PRIO_TRACE=1000 timeout -k 10 300 python tools/maze_bench.py 4096 64 1 > $O/maze4096b.json 2> $O/maze_trace_b.log || { tail $O/maze_trace_b.log; exit 1; }
python tools/trace_show.py $O/maze_trace_b.log
# per-pass list statistics and the launch gaps of the maze solve
MAZE_PASS_STATS=1 timeout -k 10 300 python tools/maze_bench.py 4096 64 1 > $O/maze4096_stats.json 2>&1 || { tail $O/maze4096_stats.json; exit 1; }
head -1 $O/maze4096_stats.json
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o maze -- python3 $R/tools/maze_bench.py 4096 64 1 > $R/$O/maze_rocprof.json 2> $R/$O/maze_rocprof.err) || { tail -20 $O/maze_rocprof.err; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/maze_kernel_stats.csv \;
find $O/kt -name "*kernel_trace.csv" -exec cp {} $O/maze_kernel_trace.csv \;
python tools/gap_stats.py $O/maze_kernel_trace.csv
rm -rf $O/kt
# the exact-tie early exit and the equal-count kernel (new this round)
timeout -k 10 300 python -u -m pytest tests/test_planner.py -k "early_exit" -x -v --timeout 120 --timeout-method thread > $O/early_exit_tests.txt 2>&1 || { tail -30 $O/early_exit_tests.txt; exit 1; }
tail -5 $O/early_exit_tests.txt
