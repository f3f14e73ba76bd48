#!/bin/bash
# Edge-column experiment: kernel-5 parity tests, then the A/B knob runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ec
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_edge.py tests/test_gpu_slabs.py tests/test_gpu_update.py tests/test_gpu_properties.py tests/test_gpu_dist_ipc.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ec/tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/ec/tests.log | head; tail -30 gpurun_out/ec/tests.log; exit 1; }
tail -1 gpurun_out/ec/tests.log
TAG=ec REPS=2 CONFIGS="base_r2;new;noec:DYMU_EC=0" bash tools/gpu_knobs.sh
