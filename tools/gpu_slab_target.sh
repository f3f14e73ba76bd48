#!/bin/bash
# Slab per-pass target sweep: the row-slab loop with S virtual ranks on one GPU
# (tools/vdist_rehearsal.py) under DYMU_PRIO_TARGET (tiles per pass, absolute) and
# DYMU_PRIO_CAPFRAC.  Output under gpurun_out/$TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-slabt}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
N=${N:-16384}
for cfg in ${CFGS:-"0:0.9" "1536:0.9" "1024:0.9" "512:0.9" "0:0.6" "1024:0.6"}; do
  t=${cfg%%:*}; cf=${cfg##*:}
  echo "== target $t capfrac $cf" | tee -a $O/sweep_$N.txt
  if [ "$t" = 0 ]; then
    DYMU_PRIO_CAPFRAC=$cf timeout -k 10 240 python tools/vdist_rehearsal.py $N 4 ${SS:-2 4 8} >> $O/sweep_$N.txt 2>&1 || { echo failed; tail $O/sweep_$N.txt; exit 1; }
  else
    DYMU_PRIO_TARGET=$t DYMU_PRIO_CAPFRAC=$cf timeout -k 10 240 python tools/vdist_rehearsal.py $N 4 ${SS:-2 4 8} >> $O/sweep_$N.txt 2>&1 || { echo failed; tail $O/sweep_$N.txt; exit 1; }
  fi
done
cat $O/sweep_$N.txt
