#!/bin/bash
# Round 4, v34: the N-GPU rehearsal -- S virtual ranks on one GPU (dymu_vdist_solve), per-rank
# passes, visits and max pass time -- at 16384^2 and 32768^2, K = 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04n; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python tools/vdist_rehearsal.py 16384 4 1 2 4 8 > $O/vdist16k_v34.txt 2>&1 || { tail -20 $O/vdist16k_v34.txt; exit 1; }
cat $O/vdist16k_v34.txt
timeout -k 10 500 python tools/vdist_rehearsal.py 32768 4 1 8 > $O/vdist32k_v34.txt 2>&1 || { tail -20 $O/vdist32k_v34.txt; exit 1; }
cat $O/vdist32k_v34.txt
