set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_slabs.py tests/test_gpu_sharded.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fused_tests.log 2>&1 || { tail -40 gpurun_out/fused_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/fused_tests.log
for i in 1 2; do
 for v in new base; do
  if [ $v = base ]; then export DYMU_LIBDIR=$GRAFT_REPO_ROOT/ab/base/lib; else unset DYMU_LIBDIR; fi
  timeout -k 10 300 python -u bench.py --sharded --no-planner --cpu-sample 0 --steps 5 --warmup 2 > gpurun_out/fsh_$v$i.log 2>&1 || { tail -20 gpurun_out/fsh_$v$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/fsh_$v$i.log').read().strip().splitlines()[-1]); print('sharded N=1 $v$i', d['ms_per_step'], d['config'].get('exchange_rounds_per_solve'), d['config']['passes_per_solve'])"
 done
done
for v in new base; do
  if [ $v = base ]; then export DYMU_LIBDIR=$GRAFT_REPO_ROOT/ab/base/lib; else unset DYMU_LIBDIR; fi
  echo "vdist $v"; timeout -k 10 300 python -u tools/vdist_rehearsal.py 16384 4 2 8 2>&1 | tee gpurun_out/fvd_$v.log | cut -c1-200 || exit 1
done
