#!/bin/bash
# Round 4: the N-rank bench path rehearsed with 4 ranks sharing one GPU (transport and K
# chosen on the node: IPC vs peer; RCCL refuses ranks that share a device).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04i; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --gpus 4 --steps 3 --warmup 1 --cpu-sample 0 > $O/bench_g4_onegpu.json 2> $O/bench_g4_onegpu.err || { tail -30 $O/bench_g4_onegpu.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_g4_onegpu.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['config'].get('transport'), d['config'].get('passes_per_exchange'), json.dumps(d.get('transport_candidates', d['config'].get('transport_candidates')))[:600], d.get('parity'))"
