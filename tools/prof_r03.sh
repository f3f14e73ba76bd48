#!/bin/bash
# Profiles of the current kernel for the bench line: rocprofv3 kernel trace +
# stats of a bench run, then the PMC passes (separate --pmc runs, calibration
# first) condensed into profiles/pmc_$VTAG.json.  Output under gpurun_out/prof_$VTAG.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=${VTAG:-r03_v1}
O=$R/gpurun_out/prof_$V
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 20 --warmup 3 --cpu-sample 0 --no-planner --no-variants --sustain-s 0 > $O/bench_rocprof.json 2> $O/bench_rocprof.err || { tail -20 $O/bench_rocprof.err; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
# the per-dispatch trace is tens of MB: keep the stats only (gpurun copies back <= 64 MiB)
find $O/kt -name "*kernel_trace.csv" -delete
head -5 $O/kernel_stats.csv
cd $R && bash tools/pmc_r02.sh || exit 1
mkdir -p $O/profiles && cd $O && python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc $V "k_fim_pass_dyn<16, true, false>" 16384 || exit 1
