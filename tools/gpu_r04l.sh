#!/bin/bash
# Round 4, v33: phase traces of three headline passes (early / middle / late) and the
# 16384^2 serpentine maze against the oracle FMM.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04l; mkdir -p $O; export TMPDIR=/tmp
for p in 200 800 1400; do
  DYMU_PRIO_TRACE=$p timeout -k 10 300 python tools/probe1.py 16384 1 > $O/trace$p.out 2> $O/trace$p.log || { tail $O/trace$p.log; exit 1; }
  echo "pass $p"; python tools/trace_show.py $O/trace$p.log
done
timeout -k 10 300 python tools/maze_bench.py 16384 64 1 > $O/maze16384_v33.json 2>&1 || { tail $O/maze16384_v33.json; exit 1; }
python3 -c "import json; d=json.loads(open('$O/maze16384_v33.json').read().strip().splitlines()[-1]); print('maze16384', d['ms_per_solve'], d['passes'], d['parity'])"
