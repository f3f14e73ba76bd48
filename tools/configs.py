"""Timings of the SURVEY s8(d) side configurations on one GPU (development /
documentation tool; the bench line is config 3, bench.py).

  config 2: 4096^2 computeCostMap on the device (dymu_compute_cost_map) + solve
  config 5: config-2 terrain, hazard disc r=20 at 30% of the start->goal line;
            windowed re-propagation (dymu_resolve_window_device) vs cold solve

Inputs are generated on the host (numpy) and uploaded once; every timing is
device time (the engine's own HIP events) of the step, median of `reps`.
Prints one JSON object.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "planning-path_planning_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402

import dymu  # noqa: E402


from gen_golden import config2_inputs  # noqa: E402  (SURVEY s8(d) config 2 inputs)


FIELDS = {"cost": 8, "raw_cost": 8, "slope": 8, "terrain": 4, "is_obstacle": 1, "hazard": 8,
          "traff": 8, "loc_mode": 4}


def main(N=4096, reps=5):
    eng = dymu.Engine()
    out = {"grid": N}
    n = N * N
    elev, terr, lut, slopes = config2_inputs(N)
    dE, dTr = eng.alloc(8 * n), eng.alloc(8 * n)
    eng.h2d(dE, elev)
    eng.h2d(dTr, terr)
    st = {f: eng.alloc(b * n) for f, b in FIELDS.items()}
    dF, dT, dT0 = eng.alloc(8 * n), eng.alloc(8 * n), eng.alloc(8 * n)

    def fresh_state():
        eng.h2d(st["cost"], np.zeros(n))
        eng.h2d(st["is_obstacle"], np.zeros(n, dtype=np.uint8))
        eng.h2d(st["hazard"], np.zeros(n))
        eng.h2d(st["traff"], np.ones(n))
        eng.h2d(st["loc_mode"], np.full(n, -1, dtype=np.int32))

    # config 2: cost map (device) then solve
    tc = []
    for _ in range(reps):
        fresh_state()
        eng.d2h(np.empty(1), dF)  # drain
        t = time.perf_counter()
        eng.compute_cost_map(N, N, N, 1.0, lut, slopes, 1, dE, dTr, st, dF)
        eng.d2h(np.empty(1), dF)
        tc.append((time.perf_counter() - t) * 1e3)
    goal = (3 * N // 4, 3 * N // 4)
    ts, stats = [], None
    for _ in range(reps):
        stats = eng.solve_device(dF, dT, N, N, N, *goal)
        ts.append(stats["ms"])
    out["config2"] = {"cost_map_ms": float(np.median(tc)), "solve_ms": float(np.median(ts)),
                      "Mcells_s_solve": n / np.median(ts) / 1e3, "passes": stats["passes"],
                      "kernel": stats["kernel"],
                      "cost_map_GBs_alg": n * (8 + 8 + 8 * 4 + 1) / np.median(tc) / 1e6}
    # config 5: hazard disc at 30% of the start->goal line
    start = (N // 5, N // 4)
    c = (int(start[0] + 0.3 * (goal[0] - start[0])), int(start[1] + 0.3 * (goal[1] - start[1])))
    r = 20
    hd = np.zeros((N, N))
    eng.d2h(hd, st["hazard"])
    hd0 = hd.copy()
    jj, ii = np.mgrid[c[1] - r - 1:c[1] + r + 2, c[0] - r - 1:c[0] + r + 2]
    d2 = (ii - c[0]) ** 2 + (jj - c[1]) ** 2
    sub = hd[c[1] - r - 1:c[1] + r + 2, c[0] - r - 1:c[0] + r + 2]
    inner, ring = d2 <= r * r, (d2 > r * r) & (d2 <= (r + 1) ** 2)
    sub[inner] = np.minimum(1.0, sub[inner] + 1.0)
    sub[ring] = np.minimum(1.0, sub[ring] + 0.1)
    eng.solve_device(dF, dT0, N, N, N, *goal)  # converged map of the old speed
    eng.h2d(st["hazard"], hd)
    eng.pack_speed(N, N, N, 1.0, st, dF)
    i0, j0, w = c[0] - r - 1, c[1] - r - 1, 2 * r + 3
    tw, sw = [], None
    T0 = np.empty((N, N))
    eng.d2h(T0, dT0)
    for _ in range(reps):
        eng.h2d(dT, T0)
        eng.d2h(np.empty(1), dT)  # drain
        t = time.perf_counter()
        sw = eng.resolve_window_device(dF, dT, N, N, N, goal[0], goal[1], i0, j0, w, w)
        tw.append((time.perf_counter() - t) * 1e3)  # raise front + re-solve, wall
    us = eng.last_update_stats()
    Tw = np.empty((N, N))
    eng.d2h(Tw, dT)
    # A/B: the round-2 theta reset (every cell at or above theta) on the same bump
    os.environ["DYMU_RAISE"] = "0"
    eng_r = dymu.Engine()
    del os.environ["DYMU_RAISE"]
    tr, sr = [], None
    for _ in range(reps):
        eng_r.h2d(dT, T0)
        eng_r.d2h(np.empty(1), dT)
        t = time.perf_counter()
        sr = eng_r.resolve_window_device(dF, dT, N, N, N, goal[0], goal[1], i0, j0, w, w)
        tr.append((time.perf_counter() - t) * 1e3)
    eng_r.close()
    tcold, sc = [], None
    for _ in range(reps):
        eng.d2h(np.empty(1), dT)
        t = time.perf_counter()
        sc = eng.solve_device(dF, dT, N, N, N, *goal)
        tcold.append((time.perf_counter() - t) * 1e3)
    Tc = np.empty((N, N))
    eng.d2h(Tc, dT)
    # the disc cleared again: a decrease-only change (no reset, window tiles seeded)
    eng.h2d(st["hazard"], hd0)
    eng.pack_speed(N, N, N, 1.0, st, dF)
    eng.solve_device(dF, dT0, N, N, N, *goal)
    T0c = np.empty((N, N))
    eng.d2h(T0c, dT0)  # reference point: the cold solve of the cleared speed
    eng.h2d(st["hazard"], hd)
    eng.pack_speed(N, N, N, 1.0, st, dF)
    eng.solve_device(dF, dT0, N, N, N, *goal)
    Tb = np.empty((N, N))
    eng.d2h(Tb, dT0)  # converged map with the disc
    eng.h2d(st["hazard"], hd0)
    eng.pack_speed(N, N, N, 1.0, st, dF)
    td, sd = [], None
    for _ in range(reps):
        eng.h2d(dT, Tb)
        eng.d2h(np.empty(1), dT)
        t = time.perf_counter()
        sd = eng.update_window_device(dF, dT, N, N, N, goal[0], goal[1], i0, j0, w, w, True)
        td.append((time.perf_counter() - t) * 1e3)
    Td = np.empty((N, N))
    eng.d2h(Td, dT)
    tcold2 = []
    for _ in range(reps):
        eng.d2h(np.empty(1), dT)
        t = time.perf_counter()
        eng.solve_device(dF, dT, N, N, N, *goal)
        tcold2.append((time.perf_counter() - t) * 1e3)
    fin0 = np.isfinite(T0c)
    out["config5_clear"] = {
        "decrease_only_ms": float(np.median(td)), "cold_ms": float(np.median(tcold2)),
        "speedup": float(np.median(tcold2) / np.median(td)),
        "decrease_only_tile_visits": sd["tile_visits"], "passes": sd["passes"],
        "inf_mask_equal": bool(np.array_equal(np.isinf(Td), np.isinf(T0c))),
        "max_rel_diff_vs_cold": float((np.abs(Td[fin0] - T0c[fin0]) /
                                       np.maximum(1, T0c[fin0])).max()),
    }
    fin = np.isfinite(Tc)
    out["config5"] = {
        "window": [i0, j0, w, w], "windowed_ms": float(np.median(tw)),
        "cold_ms": float(np.median(tcold)), "speedup": float(np.median(tcold) / np.median(tw)),
        "windowed_tile_visits": sw["tile_visits"], "cold_tile_visits": sc["tile_visits"],
        "windowed_passes": sw["passes"], "raise": us,
        "theta_reset_ms": float(np.median(tr)), "theta_reset_tile_visits": sr["tile_visits"],
        "theta_reset_passes": sr["passes"],
        "timing": "wall clock around the blocking C-ABI call (raise front included)",
        "inf_mask_equal": bool(np.array_equal(np.isinf(Tw), np.isinf(Tc))),
        "max_rel_diff_vs_cold": float((np.abs(Tw[fin] - Tc[fin]) / np.maximum(1, Tc[fin])).max()),
        "bitwise_equal_frac": float((Tw == Tc).mean()),
    }
    for p in (dE, dTr, dF, dT, dT0, *st.values()):
        eng.free(p)
    eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4096)
