"""Rehearse the N-GPU row-slab solve on ONE GPU: dymu_vdist_solve runs the
native exchange loop with S virtual ranks, serialised on one stream.  Per-rank
passes/visits are what N real GPUs would run; wall/S approximates one GPU's
share of the time (no xGMI latency, no concurrency).
usage: python tools/vdist_rehearsal.py [N] [K] [S ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "planning-path_planning_amd"))
import dymu  # noqa: E402
from dymu import dist  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
K = int(sys.argv[2]) if len(sys.argv) > 2 else 16
Ss = [int(x) for x in sys.argv[3:]] or [1, 2, 4, 8]
g = (N // 2, N // 2)
for S in Ss:
    engs, dFs, dTs = [], [], []
    for r in range(S):
        row0, nrows = dymu.slab_rows(N, S, r)
        e = dymu.Engine(device=0)
        dF, dT = e.alloc(8 * nrows * N), e.alloc(8 * (nrows + 2) * N)
        e.synth_speed(dF, N, nrows, N, row0, 1, 0.02, 3, g[0], g[1])
        engs.append(e)
        dFs.append(dF)
        dTs.append(dT)
    dist.vdist_solve(engs, dFs, dTs, N, N, N, g[0], g[1], K)  # warm-up
    t0 = time.perf_counter()
    st = dist.vdist_solve(engs, dFs, dTs, N, N, N, g[0], g[1], K)
    dt = time.perf_counter() - t0
    # busy time of each rank's pass launches (events on every launch, a second
    # solve): the critical path of N real GPUs is about the max over ranks
    for e in engs:
        e.set_profiling(1)
    dist.vdist_solve(engs, dFs, dTs, N, N, N, g[0], g[1], K)
    busy = [e.last_pass_timing()[0] for e in engs]
    for e in engs:
        e.set_profiling(0)
    print(f"S={S} K={K} wall {dt*1e3:.1f} ms  wall/S {dt*1e3/S:.1f} ms  rounds {st[0]['rounds']}  "
          f"passes/rank {[s['passes'] for s in st]}  launches/rank {st[0]['launches']}  "
          f"visits/rank {[s['tile_visits'] for s in st]}  "
          f"pass-busy ms/rank {[round(b, 1) for b in busy]}", flush=True)
    for e, dF, dT in zip(engs, dFs, dTs):
        e.free(dF)
        e.free(dT)
        e.close()
