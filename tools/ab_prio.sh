#!/bin/bash
# A/B of the v3 (plain FIM) and v4 (priority passes) pass kernels on one GPU.
# CONFIGS: space-separated "target:frac" pairs; SIZES: grid sizes.
set -o pipefail
mkdir -p gpurun_out
cd "$(dirname "$0")/.."
log=gpurun_out/ab.log
: > $log
if [ -z "$NOTEST" ]; then
DYMU_KERNEL=4 timeout -k 10 300 python -m pytest tests/test_gpu_solver.py tests/test_gpu_slabs.py tests/test_gpu_sharded.py -x -q >> $log 2>&1 || { echo "tests rc=$?" >> $log; exit 1; }
fi
for N in ${SIZES:-4096 16384}; do
  echo "v3" >> $log
  DYMU_KERNEL=3 timeout -k 10 120 python tools/probe.py $N >> $log 2>&1 || exit 1
  for C in ${CONFIGS:-8192:0}; do
    echo "v4 $C" >> $log
    DYMU_KERNEL=4 DYMU_PRIO_TARGET=${C%%:*} DYMU_PRIO_FRAC=${C##*:} timeout -k 10 120 python tools/probe.py $N >> $log 2>&1 || exit 1
  done
done
