#!/bin/bash
# Parameter sweep of the solver (development tool).  RUNS: ';'-separated env
# settings, e.g. RUNS="DYMU_KERNEL=3 DYMU_MAX_INNER=8;DYMU_KERNEL=4"; SIZES.
set -o pipefail
mkdir -p gpurun_out
cd "$(dirname "$0")/.."
log=${LOG:-gpurun_out/sweep.log}
: > $log
IFS=';' read -ra R <<< "$RUNS"
for N in ${SIZES:-16384}; do
  for run in "${R[@]}"; do
    echo "v $run" >> $log
    env $run timeout -k 10 120 python tools/probe.py $N >> $log 2>&1 || exit 1
  done
done
