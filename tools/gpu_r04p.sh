#!/bin/bash
# Round 4, v34: slab knobs in the 8-rank rehearsal (16384^2, K = 4): sweep cap and
# deadline for slabs below 2^20 tiles (defaults: cap 16, no deadline).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04p; mkdir -p $O; export TMPDIR=/tmp
for cfg in "16:0" "18:0" "20:0" "18:1500" "16:1500" "24:0"; do
  c=${cfg%%:*}; d=${cfg##*:}
  echo "== cap $c deadline $d" | tee -a $O/slab_knobs.txt
  DYMU_MAX_INNER=$c DYMU_SWEEP_DEADLINE=$d timeout -k 10 300 python tools/vdist_rehearsal.py 16384 4 8 >> $O/slab_knobs.txt 2>&1 || { tail $O/slab_knobs.txt; exit 1; }
  tail -1 $O/slab_knobs.txt
done
