#!/bin/bash
# Round 4: the multi-process transports on one GPU -- the GPU-initiated peer
# transport and the IPC transport (ADVICE fixes) against the oracle, then the
# bench's transport choice at --gpus 2 on one GPU.  Output under gpurun_out/r04b.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04b; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist_ipc.py -x -v --timeout 280 \
  --timeout-method thread > $O/dist_tests.log 2>&1 || { tail -60 $O/dist_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/dist_tests.log | tail -20
timeout -k 10 600 python -u -m pytest tests/test_bench_ranks.py -x -v -m gpu --timeout 280 \
  --timeout-method thread > $O/bench_ranks.log 2>&1 || { tail -60 $O/bench_ranks.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/bench_ranks.log | tail -8
timeout -k 10 600 python -u bench.py --gpus 2 --size 16384 --steps 3 --warmup 1 --cpu-sample 0 \
  > $O/bench_g2_16k.log 2>&1 || { tail -30 $O/bench_g2_16k.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_g2_16k.log') if l.startswith('{')][-1]); c=d['config']; print('g2 16k', d['ms_per_step'], c['transport'], c['passes_per_exchange'], c['k_autotune_ms'], d['parity']['ok'])"
