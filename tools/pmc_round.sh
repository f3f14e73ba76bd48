#!/bin/bash
# PMC passes on one solve (separate --pmc runs; no trace domains mixed in).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
N=${N:-16384}
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/tools/probe1.py" $N 1 > "$OUT/p$i.log" 2>&1 || exit $?
done
# the writes once more with the maps in cached memory (DYMU_MAP_MEM=0): the same bytes,
# but counted at the calibrated 8-B granularity (uncached 8-B stores count as 32-B requests)
DYMU_MAP_MEM=0 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/w0" -o run -- python3 "$R/tools/probe1.py" $N 1 > "$OUT/w0.log" 2>&1 || exit $?
