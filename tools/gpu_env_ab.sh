#!/bin/bash
# A/B of one environment knob in one gpurun call: kernel-5 parity tests with the
# knob's new setting, then bench.py alternating  $AB_VAR=$AB_NEW  and  $AB_VAR=$AB_OLD.
# Output under gpurun_out/$TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-envab}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
: "${AB_VAR:?}" "${AB_NEW:?}" "${AB_OLD:?}"
if [ -z "$SKIP_TESTS" ]; then
  env $AB_VAR=$AB_NEW timeout -k 10 600 python -u -m pytest ${AB_TESTS:-tests/test_gpu_solver.py tests/test_gpu_fullsize.py tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_update.py} -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for i in $(seq 1 ${REPS:-3}); do
  for v in new old; do
    if [ $v = new ]; then val=$AB_NEW; else val=$AB_OLD; fi
    env $AB_VAR=$val timeout -k 10 300 python -u bench.py --no-planner --no-variants --cpu-sample 0 --steps 10 --warmup 2 ${BENCH_ARGS} > $O/bench_$v$i.json 2> $O/bench_$v$i.err || { tail -20 $O/bench_$v$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_$v$i.json').read().strip().splitlines()[-1]); c=d['config']; print('$v$i', d['ms_per_step'], c['passes_per_solve'], c['tile_visits_per_solve'], d['roofline']['avg_launch_us'] if d['roofline'] else None)"
  done
done
