#!/bin/bash
# Round 4 final validation: pytest -m gpu (one process) and smoke().
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04g}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.txt 2>&1 || { tail -50 $O/gputest.txt; exit 1; }
tail -3 $O/gputest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -30 $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
