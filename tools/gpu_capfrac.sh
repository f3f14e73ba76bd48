#!/bin/bash
# The per-pass target capped at a fraction of the active list (default 0.9,
# DYMU_PRIO_CAPFRAC): the whole GPU suite at the default, then config 3 and the
# 4096^2 maze at neighbouring fractions.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/cf3
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/cf3/tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/cf3/tests.log | head; tail -30 gpurun_out/cf3/tests.log; exit 1; }
tail -1 gpurun_out/cf3/tests.log
TAG=cf3 REPS=2 CONFIGS="cf09;cf085:DYMU_PRIO_CAPFRAC=0.85;cf095:DYMU_PRIO_CAPFRAC=0.95" bash tools/gpu_knobs.sh || exit 1
for v in 0.85 0.95; do
  DYMU_PRIO_CAPFRAC=$v timeout -k 10 200 python -u tools/maze_bench.py 4096 64 2 > gpurun_out/cf3/m4096_$v.json 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d['parity']; print('maze4096', sys.argv[2], d['ms_per_solve'], d['passes'], d['tile_visits'], p['max_rel'])" gpurun_out/cf3/m4096_$v.json $v
done
