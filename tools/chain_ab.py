"""A/B of chained visits in one process: for each workload the
solve is timed (median of `reps`) under each DYMU_CHAIN_BELOW / _HOPS / _TICKS
setting (read by the engine at every solve), and each map is compared with the
first setting's (identical +inf mask, max relative difference) and, at <= 4096^2,
with the oracle heap FMM.  Workloads: the serpentine maze (tools/maze_bench.py) at
4096^2 / 16384^2 and the open config-3 grid at 16384^2.  One JSON line per run.
needs the chained-visit build of commit 9b220fe (reverted), e.g. as ab/chain/lib
with DYMU_LIBDIR.  usage: python tools/chain_ab.py [workload ...]   (maze4096 maze16384 open16384 open4096)
settings: CHAIN_AB="below:hops:ticks,below:hops:ticks,..." (default: off, 1024:4:2500)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "planning-path_planning_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tools")]
import dymu  # noqa: E402
import oracle_ffi  # noqa: E402
from maze_bench import serpentine  # noqa: E402


def settings():
    kv = os.environ.get("CHAIN_AB", "0:4:2500,1024:4:2500")
    return [tuple(int(x) for x in s.split(":")) for s in kv.split(",")]


def main():
    o = oracle_ffi.load()
    reps = int(os.environ.get("CHAIN_AB_REPS", "3"))
    for wl in sys.argv[1:] or ["maze4096"]:
        N = int(wl.lstrip("mazeopen"))
        g = (N // 2, N // 2)
        F = o.synth_speed(N, N, seed=1, obst_frac=0.02, obst_seed=3, goal=g)
        if wl.startswith("maze"):
            F = serpentine(F, 64)
        eng = dymu.Engine()
        dF, dT = eng.alloc(8 * N * N), eng.alloc(8 * N * N)
        eng.h2d(dF, F)
        T0 = None
        Tref = o.fmm(F, g)[0] if N <= 4096 else None
        for below, hops, ticks in settings():
            os.environ["DYMU_CHAIN_BELOW"] = str(below)
            os.environ["DYMU_CHAIN_HOPS"] = str(hops)
            os.environ["DYMU_CHAIN_TICKS"] = str(ticks)
            st = eng.solve_device(dF, dT, N, N, N, g[0], g[1])  # warm-up
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                st = eng.solve_device(dF, dT, N, N, N, g[0], g[1])
                ts.append(time.perf_counter() - t0)
            T = np.empty((N, N))
            eng.d2h(T, dT)
            rec = {"workload": wl, "chain_below": below, "hops": hops, "ticks": ticks,
                   "ms": round(sorted(ts)[len(ts) // 2] * 1e3, 3),
                   "ms_all": [round(t * 1e3, 2) for t in ts], "passes": st["passes"],
                   "tile_visits": st["tile_visits"], "sweeps": st["inner_sweeps"]}
            for name, R in (("vs_first", T0), ("vs_fmm", Tref)):
                if R is None:
                    continue
                fin = np.isfinite(R)
                rec[name] = {"mask_equal": bool(np.array_equal(np.isfinite(T), fin)),
                             "max_rel": float((np.abs(T[fin] - R[fin]) / np.maximum(1, R[fin])).max())}
            if T0 is None:
                T0 = T
            print(json.dumps(rec), flush=True)
        eng.free(dF)
        eng.free(dT)
        eng.close()


if __name__ == "__main__":
    main()
