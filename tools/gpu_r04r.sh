#!/bin/bash
# Round 4, v35: rocprofv3 kernel trace + stats of the bench and the PMC passes
# (tools/prof_r03.sh, VTAG r04_v35), the default bench.py line, the 16384^2 maze, the
# side configurations at 4096^2 and the early exit at 16384^2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04r; mkdir -p $O; export TMPDIR=/tmp
VTAG=r04_v35 bash tools/prof_r03.sh > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
tail -6 $O/prof.log
cp gpurun_out/prof_r04_v35/profiles/pmc_r04_v35.json profiles/ || exit 1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['avg_launch_us'], d['parity']['max_rel'], d['parity']['ok'], d['variants'])"
timeout -k 10 300 python tools/maze_bench.py 16384 64 1 > $O/maze16384_v35.json 2>&1 || { tail $O/maze16384_v35.json; exit 1; }
python3 -c "import json; d=json.loads(open('$O/maze16384_v35.json').read().strip().splitlines()[-1]); print('maze16384', d['ms_per_solve'], d['passes'], d['parity']['max_rel'], d['parity']['ok'])"
timeout -k 10 300 python tools/configs.py > $O/configs_4096_v35.json 2>&1 || { tail $O/configs_4096_v35.json; exit 1; }
tail -c 1200 $O/configs_4096_v35.json
timeout -k 10 300 python tools/early_exit_bench.py 16384 > $O/early_exit_v35.json 2>&1 || { tail $O/early_exit_v35.json; exit 1; }
tail -c 800 $O/early_exit_v35.json
