#!/bin/bash
# v31 side measurements in one gpurun call: the packed-key-bin parity test, 32768^2 on one
# GPU, and the multi-rank rehearsal at 16384^2 (1/2/4/8 ranks) and 32768^2 (1/8).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03k; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py -m gpu -x -q -k "packed_key_bins" --timeout 120 --timeout-method thread > $O/test_pack.log 2>&1 || { tail -30 $O/test_pack.log; exit 1; }
tail -1 $O/test_pack.log
timeout -k 10 300 python bench.py --size 32768 --steps 3 --warmup 1 --cpu-sample 0 --no-planner --no-variants > $O/bench_32k.json 2> $O/bench_32k.err || { tail $O/bench_32k.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_32k.json').read().strip().splitlines()[-1]); print('32k', d['value'], d['ms_per_step'], d['config']['passes_per_solve'])"
timeout -k 10 300 python tools/vdist_rehearsal.py 16384 4 1 2 4 8 > $O/vdist16k.txt 2>&1 || { tail $O/vdist16k.txt; exit 1; }
cat $O/vdist16k.txt
timeout -k 10 400 python tools/vdist_rehearsal.py 32768 4 1 8 > $O/vdist32k.txt 2>&1 || { tail $O/vdist32k.txt; exit 1; }
cat $O/vdist32k.txt
