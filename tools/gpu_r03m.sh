#!/bin/bash
# v31 side measurements: the serpentine maze at 4096^2 and 16384^2 (with oracle parity)
# and the early exit at 16384^2.  Output under gpurun_out/r03m.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03m; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python tools/maze_bench.py 4096 > $O/maze4096.json 2> $O/maze4096.err || { tail $O/maze4096.err; exit 1; }
cat $O/maze4096.json
timeout -k 10 300 python tools/early_exit_bench.py 16384 > $O/early_exit.json 2> $O/early_exit.err || { tail $O/early_exit.err; exit 1; }
cat $O/early_exit.json
timeout -k 10 600 python tools/maze_bench.py 16384 64 2 > $O/maze16384.json 2> $O/maze16384.err || { tail $O/maze16384.err; exit 1; }
cat $O/maze16384.json
