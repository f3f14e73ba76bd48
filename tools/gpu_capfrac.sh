#!/bin/bash
# The per-pass target capped at a fraction of the active list (DYMU_PRIO_CAPFRAC):
# kernel-5 parity with the cap, config 3 A/B, configs 2/5, the maze at 16384^2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/cf2
export TMPDIR=/tmp
DYMU_PRIO_CAPFRAC=0.9 timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_update.py tests/test_planner.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cf2/tests.log 2>&1 || { tail -30 gpurun_out/cf2/tests.log; exit 1; }
tail -1 gpurun_out/cf2/tests.log
TAG=cf2 REPS=3 CONFIGS="new;cf09:DYMU_PRIO_CAPFRAC=0.9" bash tools/gpu_knobs.sh || exit 1
for v in 0 0.9; do
  DYMU_PRIO_CAPFRAC=$v timeout -k 10 300 python -u tools/configs.py > gpurun_out/cf2/configs_$v.json 2> gpurun_out/cf2/configs_$v.err || { tail gpurun_out/cf2/configs_$v.err; exit 1; }
  echo "configs $v: $(cat gpurun_out/cf2/configs_$v.json | head -c 900)"
done
DYMU_PRIO_CAPFRAC=0.9 timeout -k 10 300 python -u tools/maze_bench.py 16384 64 2 > gpurun_out/cf2/m16k_0.9.json 2>&1 || exit 1
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d['parity']; print('maze16k 0.9', d['ms_per_solve'], d['passes'], d['tile_visits'], p['max_rel'])" gpurun_out/cf2/m16k_0.9.json
