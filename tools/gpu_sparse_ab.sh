#!/bin/bash
# A/B of sparse kernel-5 grids (DYMU_SPARSE_TPW): parity tests with the knob on,
# then config 2/5 timings and the bench at 4096^2 / 16384^2 for TPW = 0 / 4 / 8.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
DYMU_SPARSE_TPW=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_update.py tests/test_gpu_edge.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sp_tests.log 2>&1 || { tail -40 gpurun_out/sp_tests.log; exit 1; }
tail -1 gpurun_out/sp_tests.log
for t in 0 4 8; do
  DYMU_SPARSE_TPW=$t timeout -k 10 300 python -u tools/configs.py > gpurun_out/sp_cfg_$t.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/sp_cfg_$t.json')); print('TPW $t', 'cfg2', round(d['config2']['solve_ms'],3), 'cfg5', round(d['config5']['windowed_ms'],3), 'clear', round(d['config5_clear']['decrease_only_ms'],3))"
done
for sz in 4096 16384; do
 for t in 0 4 8; do
  DYMU_SPARSE_TPW=$t timeout -k 10 300 python -u bench.py --no-planner --cpu-sample 0 --steps 10 --warmup 2 --size $sz > gpurun_out/sp_b_${sz}_$t.log 2>&1 || { tail -5 gpurun_out/sp_b_${sz}_$t.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sp_b_${sz}_$t.log').read().strip().splitlines()[-1]); print('$sz TPW $t', d['ms_per_step'], d['config']['passes_per_solve'], d['roofline']['avg_launch_us'])"
 done
done
