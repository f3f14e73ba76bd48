#!/bin/bash
# One GPU call: the -m gpu suite, smoke, then bench.py (stops at the first failure).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
