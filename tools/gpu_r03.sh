#!/bin/bash
# Round-3 validation in one gpurun call: GPU tests + smoke, the default bench
# line, the sharded loop at N=1 (RCCL) and N=2 on one GPU (IPC transport), each
# with its stitched-map self-check.  Output under gpurun_out/$TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r03}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/gputest.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/gputest.log | tail -3
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $O/gputest.log | head -30; tail -40 $O/gputest.log; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
[ -n "$NO_DECOMP" ] || timeout -k 10 200 python tools/pass_decomp.py --out $O --tag decomp16k > $O/decomp16k.json 2> $O/decomp16k.err || { echo decomp failed; tail -20 $O/decomp16k.err; exit 1; }
[ -n "$NO_DECOMP" ] || cat $O/decomp16k.json
[ -n "$CONFIGS" ] && { timeout -k 10 300 python tools/configs.py > $O/configs_4096.json 2> $O/configs.err || { echo configs failed; tail $O/configs.err; exit 1; }; cat $O/configs_4096.json; }
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python bench.py --sharded --steps 5 --cpu-sample 0 > $O/bench_sharded_n1.json 2> $O/bench_sharded_n1.err || { echo sharded n1 failed; tail -20 $O/bench_sharded_n1.err; exit 1; }
timeout -k 10 400 python bench.py --gpus 2 --exchange ipc --steps 3 --warmup 1 --cpu-sample 0 > $O/bench_ipc_n2.json 2> $O/bench_ipc_n2.err || { echo ipc n2 failed; tail -20 $O/bench_ipc_n2.err; exit 1; }
[ -n "$LINEAR2048" ] && { timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-planner --no-variants --cpu-linear-size 2048 > $O/bench_linear2048.json 2> $O/bench_linear2048.err || { echo linear2048 failed; tail $O/bench_linear2048.err; exit 1; }; }
for f in bench bench_sharded_n1 bench_ipc_n2; do python -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('parity'), d.get('variants'))"; done
