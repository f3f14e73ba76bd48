#!/bin/bash
# One GPU call: gpu tests, smoke, bench, rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
