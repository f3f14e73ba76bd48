#!/bin/bash
# One parameterised GPU-box launcher (replaces the per-call gpu_r0*.sh scripts).
# usage (on the box, via gpurun): bash tools/gpu_run.sh TAG STEP [STEP ...]
# Output under gpurun_out/TAG/.  Each step runs under its own time limit; the first
# failing step ends the call (no GPU step after a failure).
# Steps:
#   tests[=PYTEST_ARGS]   pytest -m gpu (default: all of tests/), one process
#   smoke                 __graft_entry__.smoke()
#   bench[=ARGS]          python bench.py ARGS (default line)
#   quick                 bench.py --no-planner --cpu-sample 0 --no-variants --steps 10 --warmup 2
#   maze=N                tools/maze_bench.py N 64 1
#   configs               tools/configs.py (config 2 / 5 at 4096^2)
#   early=N               tools/early_exit_bench.py N
#   plearly=N             tools/planner_early_exit_bench.py N
#   vdist=N[:K[:S...]]    tools/vdist_rehearsal.py N K S... (1-8 virtual ranks)
#   prof=VTAG             tools/prof_r03.sh (rocprofv3 --stats + PMC passes)
#   py=SCRIPT[:ARGS]      python SCRIPT ARGS (any other tool), output SCRIPT.out
# Other steps take ':'-separated arguments (tests=tests/test_planner.py:-k:ties~or~exit).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p "$O"; export TMPDIR=/tmp
run() {  # run NAME SECONDS CMD... ; stdout -> $O/NAME.out, stderr -> $O/NAME.err
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "!! $name failed rc=$rc"; tail -30 "$O/$name.out"; tail -30 "$O/$name.err"; exit 1
  fi
  tail -c 1500 "$O/$name.out"; echo
}
for step in "$@"; do
  key=${step%%=*}; val=; [ "$key" != "$step" ] && val=${step#*=}
  [ "$key" != py ] && val=${val//:/ }  # ':' separates arguments (vdist=16384:4)
  case $key in
    tests) # '~' inside an argument stands for a space (tests=tests/x.py:-k:a~or~b)
           args=(); for w in ${val:-tests}; do args+=("${w//\~/ }"); done
           run tests 1100 python -u -m pytest "${args[@]}" -m gpu -x -v --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python -u bench.py $val ;;
    quick) run quick 300 python -u bench.py --no-planner --cpu-sample 0 --no-variants --steps 10 --warmup 2 ;;
    maze) run "maze${val// /_}" 600 python -u tools/maze_bench.py $val 64 1 ;;
    configs) run configs 300 python -u tools/configs.py ;;
    early) run "early${val// /_}" 300 python -u tools/early_exit_bench.py $val ;;
    plearly) run "plearly${val// /_}" 900 python -u tools/planner_early_exit_bench.py $val ;;
    vdist) run "vdist${val// /_}" 600 python -u tools/vdist_rehearsal.py $val ;;
    prof) VTAG=$val run prof 900 bash tools/prof_r03.sh ;;
    py) s=${val%%:*}; a=; [ "$s" != "$val" ] && a=${val#*:}
        run "$(basename "$s" .py)" 600 python -u "$s" ${a//:/ } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
