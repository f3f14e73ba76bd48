#!/bin/bash
# GPU test suite (+ smoke) in one call; output under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gputest.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/gputest.log | tail -3
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/gputest.log | head -30; tail -60 gpurun_out/gputest.log; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
