#!/bin/bash
# Round 4, v33: rocprofv3 kernel trace + stats of the bench and the PMC passes
# (tools/prof_r03.sh, VTAG r04_v33), then the default bench.py line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04k; mkdir -p $O; export TMPDIR=/tmp
VTAG=r04_v33 bash tools/prof_r03.sh > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
tail -6 $O/prof.log
cp gpurun_out/prof_r04_v33/profiles/pmc_r04_v33.json profiles/ || exit 1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['avg_launch_us'], d['parity']['max_rel'], d['parity']['ok'])"
