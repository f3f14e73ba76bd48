"""Planner-level computeTotalCostMap (src/DyMu_GlobalPathPlanning.cpp:364-408)
timings, ties included (VERDICT r4 "do this" 2): the whole class-surface call --
engine early exit, the host's resolution of the reference's pop order at the exit
value (csrc/pop_order.hpp), the band replay -- on three maps per size:
  config3  U(1,5) costs with 2% obstacles (numpy; the config-3 shape),
  const    constant cost (every mirror image ties),
  region   config3 with a constant-cost square of side N/2 around the goal,
  two      costs 1 or 2 (integer sums tie in the reference; round 6),
  int5     integer costs 1..5 with 2% obstacles (round 6).
MAPS=two,int5 picks the maps (default config3,const,region).  Goal at the centre; starts near, mid and far.  Prints one JSON object: per map
and start the median wall ms of 3 calls, the engine passes, the band size and
lastEarlyExit() (tied cells, cells left OPEN at the exit value, exact replay,
host ms).
usage: python tools/planner_early_exit_bench.py [N ...]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "planning-path_planning_amd"))
import dymu  # noqa: E402


def cost_map(kind, N, rng):
    if kind == "const":
        return np.ones((N, N))
    if kind == "two":
        return np.where(rng.random((N, N)) < 0.5, 1.0, 2.0)
    if kind == "int5":
        c = rng.integers(1, 6, size=(N, N)).astype(np.float64)
        c[rng.random((N, N)) < 0.02] = -1.0
        return c
    c = rng.uniform(1.0, 5.0, size=(N, N))
    c[rng.random((N, N)) < 0.02] = -1.0
    if kind == "region":
        c[N // 4:3 * N // 4, N // 4:3 * N // 4] = 1.0
    return c


def safe_start(c, i, j):
    N = c.shape[0]
    for r in range(0, 64):
        for di in range(-r, r + 1):
            ii, jj = i + di, j + r
            if 1 <= ii < N - 1 and 1 <= jj < N - 1 and (c[jj - 1:jj + 2, ii - 1:ii + 2] > 0).all():
                return ii, jj
    raise RuntimeError("no safe start")


def main():
    out = {}
    for N in [int(x) for x in sys.argv[1:]] or [4096]:
        rng = np.random.default_rng(5)
        g = (N // 2, N // 2)
        res = {}
        for kind in os.environ.get("MAPS", "config3,const,region").split(","):
            c = cost_map(kind, N, rng)
            c[g[1] - 1:g[1] + 2, g[0] - 1:g[0] + 2] = np.abs(c[g[1] - 1:g[1] + 2, g[0] - 1:g[0] + 2])
            p = dymu.Planner()
            p.initGlobalLayer(1.0, 0.5, N, N)
            p.setCostMap(c)
            assert p.setGoal(g)
            rows = []
            for (fi, fj) in ((0.52, 0.51), (0.7, 0.6), (0.95, 0.9)):
                s = safe_start(c, int(fi * N), int(fj * N))
                ts = []
                for _ in range(3):
                    t0 = time.perf_counter()
                    rc = p.computeTotalCostMap(s)
                    ts.append(time.perf_counter() - t0)
                rows.append({"start": s, "rc": bool(rc), "ms": round(sorted(ts)[1] * 1e3, 3),
                             "passes": p.lastStats()["passes"], "band": p.lastBandSize(),
                             **p.lastEarlyExit()})
                print(json.dumps({"N": N, "map": kind, **rows[-1]}), file=sys.stderr, flush=True)
            t0 = time.perf_counter()
            p.computeEntireTotalCostMap()
            res[kind] = {"early": rows, "entire_ms": round((time.perf_counter() - t0) * 1e3, 3)}
            p.close()
            del c
        out[str(N)] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
