#!/bin/bash
# PMC round on the current kernel: the 8-B/lane counter calibration
# (tools/pmc_calib: known bytes, in uncached memory like the maps since round 6;
# PMC_CALIB_MEM=cached for hipMalloc) and the counter passes of tools/pmc_round.sh,
# each pass a separate rocprofv3 --pmc run (no trace domains mixed in).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/pmc"
mkdir -p "$OUT"
# the calibration probe is git-ignored: build it here when this tree has none
[ -x "$R/tools/pmc_calib" ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 "$R/tools/pmc_calib.hip" -o "$R/tools/pmc_calib" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/c1" -o run -- "$R/tools/pmc_calib" 16384 ${PMC_CALIB_MEM:-uc} > "$OUT/c1.log" 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/c2" -o run -- "$R/tools/pmc_calib" 16384 ${PMC_CALIB_MEM:-uc} > "$OUT/c2.log" 2>&1 || exit 1
# the cached-memory write calibration as well: the kernel's writes are counted on a
# cached-map pass too (tools/pmc_round.sh: w0), see tools/pmc_summary.py
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/c3" -o run -- "$R/tools/pmc_calib" 16384 cached > "$OUT/c3.log" 2>&1 || exit 1
bash "$R/tools/pmc_round.sh"
