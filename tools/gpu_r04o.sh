#!/bin/bash
# Round 4, v34: 32768^2 on one GPU, and bench.py --gpus 2 with both ranks on one GPU
# (transport and K chosen on the node).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04o; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --size 32768 --steps 3 --warmup 1 --cpu-sample 0 --no-planner --no-variants --no-parity > $O/bench_32k_v34.json 2> $O/bench_32k.err || { tail -20 $O/bench_32k.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_32k_v34.json').read().strip().splitlines()[-1]); print('32k', d['value'], d['ms_per_step'], d['config']['passes_per_solve'])"
timeout -k 10 600 python -u bench.py --gpus 2 --steps 3 --warmup 1 --cpu-sample 0 > $O/bench_g2_v34.json 2> $O/bench_g2.err || { tail -20 $O/bench_g2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_g2_v34.json').read().strip().splitlines()[-1]); print('g2', d['ms_per_step'], d['config']['transport'], d['config']['passes_per_exchange'], d['config'].get('k_autotune_ms'), d['parity']['ok'])"
