"""Generates the committed golden fixtures under tests/golden/.

Inputs are synthetic (the reference ships no fixtures and no tests); expected
outputs come from the CPU restatement in oracle/ (exact reference pop order),
which is itself pinned by the reference-run KAT checksums of SURVEY.md s8(c)
(tests/test_oracle.py::test_kat_reference_checksums).  Run from the repo root:
    python tests/golden/gen_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_ffi  # noqa: E402


def terrain_inputs(N):
    """Config-2 style terrain: sinusoid + ramp elevation,
    checkerboard terrain ids 1/2, 3 terrains x 1 mode x 5 slopes LUT."""
    j, i = np.mgrid[0:N, 0:N].astype(np.float64)
    elev = 3.0 * np.sin(0.05 * i) * np.cos(0.07 * j) + 0.002 * i
    terr = 1.0 + (((i.astype(np.int64) // 16) + (j.astype(np.int64) // 16)) % 2)
    lut = np.array([100.0] * 5 + [1, 1.5, 2, 3, 5] + [2, 2.5, 3, 4, 6], dtype=np.float64)
    slopes = np.array([0.0, 5.0, 10.0, 15.0, 20.0])
    return elev, terr, lut, slopes


def valuenoise(N, seed=2, cell=64):
    """Bilinear value noise on a `cell`-spaced lattice of U(0,1) draws (SURVEY s8(d)
    config 2's elevation term)."""
    L = N // cell + 2
    rng = np.random.default_rng(seed)
    lat = rng.uniform(0.0, 1.0, (L, L))
    x = np.arange(N) / cell
    i0 = np.floor(x).astype(int)
    f = x - i0
    rows = lat[:, i0] * (1 - f) + lat[:, i0 + 1] * f          # [L, N] along x
    return rows[i0, :] * (1 - f)[:, None] + rows[i0 + 1, :] * f[:, None]


def config2_inputs(N):
    """BASELINE config 2: elevation 3 sin(0.05 i) cos(0.07 j) + 0.002 i +
    0.5 valuenoise(seed 2, 64-cell lattice); terrain 1 + ((i/16 + j/16) mod 2); LUT
    3 terrains x "Wheel" x slopes {0,5,10,15,20} deg."""
    elev, terr, lut, slopes = terrain_inputs(N)
    return elev + 0.5 * valuenoise(N), terr, lut, slopes


def main():
    o = oracle_ffi.load()
    out = {}
    # 1) setCostMap path: mt19937_64(2) U(1,5) with 5% obstacles (cost -1)
    N = 64
    cost = o.mt_uniform(N * N, seed=2).reshape(N, N)
    obs_u = o.mt_uniform(N * N, seed=3, lo=0.0, hi=1.0).reshape(N, N)
    cost[obs_u < 0.05] = -1.0
    g = (40, 21)
    cost[g[1] - 1:g[1] + 2, g[0] - 1:g[0] + 2] = np.abs(cost[g[1] - 1:g[1] + 2, g[0] - 1:g[0] + 2])
    st = o.new_state(N, N)
    o.lib.oracle_set_cost_map(cost.ravel(), cost.size, st["cost"].ravel(), st["is_obstacle"].ravel(),
                              st["traff"].ravel(), st["hazard"].ravel())
    F = o.pack_speed(st["cost"], st["hazard"], st["traff"], st["is_obstacle"], res=1.0)
    T, rc = o.fmm(F, g, linear=True)
    out["setcost64_cost"] = cost
    out["setcost64_goal"] = np.array(g, dtype=np.int64)
    out["setcost64_T"] = T
    # 2) computeCostMap path (terrain), 128^2, res 0.5, goal (96, 96)
    N = 128
    elev, terr, lut, slopes = terrain_inputs(N)
    st = o.new_state(N, N)
    o.compute_cost_map(st, 0.5, lut, slopes, 1, elev, terr)
    g = (96, 96)
    F = o.pack_speed(st["cost"], st["hazard"], st["traff"], st["is_obstacle"], res=0.5)
    T, rc = o.fmm(F, g, linear=True)
    out["terrain128_elev"] = elev
    out["terrain128_terrain"] = terr
    out["terrain128_cost"] = st["cost"].copy()
    out["terrain128_goal"] = np.array(g, dtype=np.int64)
    out["terrain128_T"] = T
    # 3) early-exit computeTotalCostMap on the 64^2 map: tentative T + closed
    F64 = o.pack_speed(*(lambda s: (s["cost"], s["hazard"], s["traff"], s["is_obstacle"]))(
        _state_from_cost(o, out["setcost64_cost"])), res=1.0)
    T, rc, closed = o.fmm(F64, tuple(out["setcost64_goal"]), start=(12, 50), linear=True,
                          want_closed=True)
    out["early64_T"] = T
    out["early64_closed"] = closed
    out["early64_rc"] = np.array([rc], dtype=np.int64)
    # 4) early exit far from the goal on a 256^2 map: U(1,5) from
    #    mt19937_64(5), 3% obstacles, goal (200, 190), start (30, 40)
    N = 256
    cost = o.mt_uniform(N * N, seed=5).reshape(N, N)
    obs_u = o.mt_uniform(N * N, seed=6, lo=0.0, hi=1.0).reshape(N, N)
    cost[obs_u < 0.03] = -1.0
    g, s = (200, 190), (30, 40)
    for (ci, cj) in (g, s):
        cost[cj - 1:cj + 2, ci - 1:ci + 2] = np.abs(cost[cj - 1:cj + 2, ci - 1:ci + 2])
    F = o.pack_speed(*(lambda t: (t["cost"], t["hazard"], t["traff"], t["is_obstacle"]))(
        _state_from_cost(o, cost)), res=1.0)
    T, rc, closed = o.fmm(F, g, start=s, linear=False, want_closed=True)
    out["early256_cost"] = cost
    out["early256_goal_start"] = np.array(g + s, dtype=np.int64)
    out["early256_T"] = T
    out["early256_closed"] = closed
    out["early256_rc"] = np.array([rc], dtype=np.int64)
    for k, v in out.items():
        np.save(os.path.join(HERE, k + ".npy"), v, allow_pickle=False)
    print("wrote", len(out), "fixtures")


def _state_from_cost(o, cost):
    N = cost.shape[0]
    st = o.new_state(N, N)
    o.lib.oracle_set_cost_map(np.ascontiguousarray(cost).ravel(), cost.size, st["cost"].ravel(),
                              st["is_obstacle"].ravel(), st["traff"].ravel(), st["hazard"].ravel())
    return st


if __name__ == "__main__":
    main()
