#!/bin/bash
# Round 4, v34: sweep cap 16 vs 18 on grids below 2^18 tiles (4096^2 configs 2/5, the
# 4096^2 maze, 2048^2 config 3).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04q; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
for c in 16 18; do
  DYMU_MAX_INNER=$c timeout -k 10 300 python tools/configs.py > $O/configs_c$c.$i.json 2>&1 || { tail $O/configs_c$c.$i.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/configs_c$c.$i.json').read().strip().splitlines()[-1]); print('cap $c configs: c2 solve', round(d['config2']['solve_ms'],3), 'c5 window', round(d['config5']['windowed_ms'],3), 'c5 clear', round(d['config5_clear']['decrease_only_ms'],3))"
  DYMU_MAX_INNER=$c timeout -k 10 300 python tools/maze_bench.py 4096 64 3 > $O/maze_c$c.$i.json 2>&1 || { tail $O/maze_c$c.$i.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/maze_c$c.$i.json').read().strip().splitlines()[-1]); print('cap $c maze4096', d['ms_per_solve'], d['passes'], d['parity']['ok'])"
  DYMU_MAX_INNER=$c timeout -k 10 300 python -u bench.py --size 2048 --steps 20 --warmup 3 --cpu-sample 0 --no-planner --no-variants --no-parity > $O/b2048_c$c.$i.json 2>&1 || { tail $O/b2048_c$c.$i.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b2048_c$c.$i.json').read().strip().splitlines()[-1]); print('cap $c 2048^2', d['ms_per_step'], d['config']['passes_per_solve'])"
done
done
