#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT="$R/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "[$(date +%T)] $name" >> "$OUT/steps.log"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> "$OUT/steps.log"
  return $rc
}
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
: > "$OUT/steps.log"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step gpu_tests 900 python -m pytest tests -m gpu -q; rc=$?; ok_or_testfail $rc || exit $rc
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
step bench 900 python bench.py ${BENCH_ARGS:-} || exit $?
if [ "${SKIP_PROF:-0}" != 1 ]; then
  cd /tmp
  step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-sample 0 || exit $?
fi
