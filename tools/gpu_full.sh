#!/bin/bash
# One GPU call: gpu tests, smoke, bench, then rocprofv3 kernel stats of a short bench (no CPU leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
bash tools/gpu_check.sh || exit 1
cp gpurun_out/bench.log gpurun_out/bench_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-planner --cpu-sample 0 --steps 5 --warmup 2 > gpurun_out/prof_$TAG.log 2>&1 || { echo rocprof failed; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
tail -1 gpurun_out/prof_$TAG.log
find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -3
