#!/bin/bash
# Lazy initialisation: the GPU suite on the working tree (all tests, durations),
# then the A/B knob runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/lazy
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --durations=15 --timeout 300 --timeout-method thread > gpurun_out/lazy/tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" gpurun_out/lazy/tests.log | tail -12
case $rc in 0|1) ;; *) exit $rc ;; esac
TAG=lazy REPS=2 CONFIGS="base_ec;new;nolazy:DYMU_LAZY=0" bash tools/gpu_knobs.sh
