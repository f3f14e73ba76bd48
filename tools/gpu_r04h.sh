#!/bin/bash
# Round 4 final measurement: rocprofv3 kernel trace + stats of the bench and the PMC
# passes for the current kernel (tools/prof_r03.sh, VTAG r04_v32), then the default
# bench.py line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04h; mkdir -p $O; export TMPDIR=/tmp
VTAG=r04_v32 bash tools/prof_r03.sh > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
tail -8 $O/prof.log
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 1500 $O/bench.json
