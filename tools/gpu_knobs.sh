#!/bin/bash
# Knob sweep in one gpurun call: bench.py (headline grid, short) once per
# configuration in $CONFIGS ("name:VAR=v,VAR=v;name2:..."; a configuration named
# base* runs ab/<name>/lib through DYMU_LIBDIR), $REPS rounds interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-knobs}
mkdir -p $O
export TMPDIR=/tmp
IFS=';' read -ra CFG <<< "$CONFIGS"
for i in $(seq 1 ${REPS:-2}); do
  for c in "${CFG[@]}"; do
    name=${c%%:*}; vars=${c#*:}
    [ "$vars" = "$c" ] && vars=""
    envs=()
    IFS=',' read -ra KV <<< "$vars"
    for kv in "${KV[@]}"; do [ -n "$kv" ] && envs+=("$kv"); done
    case $name in base*) envs+=("DYMU_LIBDIR=$GRAFT_REPO_ROOT/ab/$name/lib");; esac
    env "${envs[@]}" timeout -k 10 300 python -u bench.py --no-planner --no-variants --cpu-sample 0 --steps ${STEPS:-10} --warmup 2 --size ${SIZE:-16384} > $O/$name.$i.json 2> $O/$name.$i.err || { echo "$name failed"; tail -20 $O/$name.$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$name.$i.json').read().strip().splitlines()[-1]); c=d['config']; print('$name.$i', d['ms_per_step'], c['passes_per_solve'], c['tile_visits_per_solve'], c['inner_sweeps_per_solve'], round(d['roofline']['avg_launch_us'],2))"
  done
done
