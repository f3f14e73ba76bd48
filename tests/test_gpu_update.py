"""GPU parity of the windowed re-propagation:
dymu_resolve_window / dymu_resolve_window_device after the speed changed in a
window must reach the map of a cold solve of the new speed -- compared with
the oracle FMM (tolerance 1e-12, identical +inf mask, as every engine test) and
with the engine's own cold solve."""
import numpy as np
import pytest

from gen_golden import terrain_inputs
from test_gpu_solver import assert_parity

pytestmark = pytest.mark.gpu


def disc(nx, ny, c, r):
    j, i = np.mgrid[0:ny, 0:nx]
    d2 = (i - c[0]) ** 2 + (j - c[1]) ** 2
    return d2 <= r * r, (d2 > r * r) & (d2 <= (r + 1) ** 2)


def window_of(mask):
    jj, ii = np.nonzero(mask)
    return int(ii.min()), int(jj.min()), int(ii.max() - ii.min() + 1), int(jj.max() - jj.min() + 1)


def modified(kind, F0, goal, rng):
    ny, nx = F0.shape
    F1 = F0.copy()
    if kind == "hazard":      # speed increase on a disc + ring, far from the goal
        inner, ring = disc(nx, ny, (nx // 5, ny // 3), 9)
        F1[inner] *= 1.5
        F1[ring] *= 1.05
        return F1, window_of(inner | ring)
    if kind == "obstacle":    # a blocked disc
        inner, _ = disc(nx, ny, (nx * 2 // 3, ny // 4), 7)
        F1[inner] = np.inf
        return F1, window_of(inner)
    if kind == "clear":       # obstacles removed in a box: speed decrease
        i0, j0, w, h = nx // 4, ny // 2, 40, 30
        box = F1[j0:j0 + h, i0:i0 + w]
        box[~np.isfinite(box)] = 2.0
        box *= 0.5
        return F1, (i0, j0, w, h)
    if kind == "mixed":       # random up / down factors
        i0, j0, w, h = nx // 2, ny // 8, 25, 35
        F1[j0:j0 + h, i0:i0 + w] *= rng.uniform(0.5, 2.0, (h, w))
        return F1, (i0, j0, w, h)
    if kind == "goal":        # window over the goal: everything but the goal resets
        i0, j0 = goal[0] - 5, goal[1] - 5
        F1[j0:j0 + 11, i0:i0 + 11] *= 1.3
        return F1, (i0, j0, 11, 11)
    if kind == "border":      # window clipped at the grid edge
        F1[ny - 6:, nx - 20:] *= 2.0
        return F1, (nx - 20, ny - 6, 500, 500)
    raise KeyError(kind)


KINDS = ["hazard", "obstacle", "clear", "mixed", "goal", "border"]


@pytest.mark.parametrize("kind", KINDS)
def test_resolve_window_matches_cold(kengine, oracle, kind):
    nx, ny, goal = 300, 260, (150, 200)
    rng = np.random.default_rng(17)
    F0 = oracle.synth_speed(nx, ny, seed=23, obst_frac=0.04, obst_seed=29, goal=goal)
    kengine.solve(F0, *goal)
    F1, (i0, j0, w, h) = modified(kind, F0, goal, rng)
    r = kengine.resolve_window(F1, goal[0], goal[1], i0, j0, w, h)
    Tref, _ = oracle.fmm(F1, goal)
    assert_parity(r.T, Tref)
    cold = kengine.solve(F1, *goal)
    assert_parity(r.T, cold.T)
    if kind in ("hazard", "obstacle", "mixed"):  # downstream of a small window only
        assert r.stats["tile_visits"] < cold.stats["tile_visits"]
    # a second update chains on the first (the engine keeps the staged state)
    F2 = F1.copy()
    F2[5:15, 5:25] *= 0.8
    r2 = kengine.resolve_window(F2, goal[0], goal[1], 5, 5, 20, 10)
    Tref2, _ = oracle.fmm(F2, goal)
    assert_parity(r2.T, Tref2)


def test_resolve_window_device_pitched(engine, oracle):
    nx, ny, ld, goal = 257, 190, 264, (30, 40)
    F0 = oracle.synth_speed(nx, ny, seed=3, obst_frac=0.03, obst_seed=7, goal=goal)
    inner, ring = disc(nx, ny, (200, 120), 12)
    F1 = F0.copy()
    F1[inner] = np.inf
    F1[ring] *= 1.2
    i0, j0, w, h = window_of(inner | ring)
    dF, dT = engine.alloc(8 * ny * ld), engine.alloc(8 * ny * ld)
    try:
        buf = np.zeros((ny, ld))
        buf[:, :nx] = F0
        engine.h2d(dF, buf)
        engine.solve_device(dF, dT, nx, ny, ld, *goal)
        buf[:, :nx] = F1
        engine.h2d(dF, buf)
        st = engine.resolve_window_device(dF, dT, nx, ny, ld, goal[0], goal[1], i0, j0, w, h)
        T = np.empty((ny, ld))
        engine.d2h(T, dT)
        Tref, _ = oracle.fmm(F1, goal)
        assert_parity(T[:, :nx], Tref)
        assert st["passes"] > 0
    finally:
        engine.free(dF)
        engine.free(dT)


def test_config5_hazard_bump(kengine, oracle):
    """SURVEY s8(d) config 5 (scaled to 512^2): config-2 terrain, a hazard disc of
    radius 20 at 30% along the start->goal line, hazard = min(1, hd+1) inside and
    min(1, hd+0.1) on the 1-cell ring (LocalPathRepairing.cpp:264-274)."""
    N, res = 512, 1.0
    elev, terr, lut, slopes = terrain_inputs(N)
    st = oracle.new_state(N, N)
    oracle.compute_cost_map(st, res, lut, slopes, 1, elev, terr)
    goal, start = (384, 384), (40, 60)
    F0 = oracle.pack_speed(st["cost"], st["hazard"], st["traff"], st["is_obstacle"], res=res)
    kengine.solve(F0, *goal)
    c = (int(start[0] + 0.3 * (goal[0] - start[0])), int(start[1] + 0.3 * (goal[1] - start[1])))
    inner, ring = disc(N, N, c, 20)
    hd = st["hazard"].copy()
    hd[inner] = np.minimum(1.0, hd[inner] + 1.0)
    hd[ring] = np.minimum(1.0, hd[ring] + 0.1)
    F1 = oracle.pack_speed(st["cost"], hd, st["traff"], st["is_obstacle"], res=res)
    i0, j0, w, h = window_of(inner | ring)
    r = kengine.resolve_window(F1, goal[0], goal[1], i0, j0, w, h)
    Tref, _ = oracle.fmm(F1, goal)
    assert_parity(r.T, Tref)
    cold = kengine.solve(F1, *goal)
    assert r.stats["tile_visits"] < cold.stats["tile_visits"]


def test_resolve_window_needs_previous_solve(dymu, oracle):
    eng = dymu.Engine()
    try:
        F = oracle.synth_speed(64, 64, seed=1, obst_frac=0.0, obst_seed=1, goal=(10, 10))
        with pytest.raises(dymu.DymuError):
            eng.resolve_window(F, 10, 10, 0, 0, 4, 4)
        eng.solve(F, 10, 10)
        with pytest.raises(dymu.DymuError):  # other goal
            eng.resolve_window(F, 11, 10, 0, 0, 4, 4)
        r = eng.resolve_window(F, 10, 10, 40, 40, 4, 4)  # nothing changed
        Tref, _ = oracle.fmm(F, (10, 10))
        assert_parity(r.T, Tref)
    finally:
        eng.close()


@pytest.mark.parametrize("kind", ["hazard", "obstacle", "mixed", "border"])
def test_raise_front_is_local(dymu, oracle, kind, monkeypatch):
    """Speed increases re-propagate only the window's dependency cone (the raise
    front), not every cell at or above theta as the round-2 reset
    did (DYMU_RAISE=0 keeps it for A/B): both reach the cold fixed point, the raise
    invalidates a subset of the reset region and visits fewer tiles."""
    nx, ny, goal = 300, 260, (150, 200)
    rng = np.random.default_rng(5)
    F0 = oracle.synth_speed(nx, ny, seed=23, obst_frac=0.04, obst_seed=29, goal=goal)
    F1, (i0, j0, w, h) = modified(kind, F0, goal, rng)
    T0, _ = oracle.fmm(F0, goal)
    Tref, _ = oracle.fmm(F1, goal)
    got = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("DYMU_RAISE", mode)
        eng = dymu.Engine(kernel=5, prio_target=16)
        try:
            eng.solve(F0, *goal)
            r = eng.resolve_window(F1, goal[0], goal[1], i0, j0, w, h)
            got[mode] = (r, eng.last_update_stats())
        finally:
            eng.close()
        assert_parity(got[mode][0].T, Tref)
    r1, us = got["1"]
    r0, us0 = got["0"]
    assert us0["raise_passes"] == 0 and us["raise_passes"] > 0
    wi0, wj0 = max(i0 - 1, 0), max(j0 - 1, 0)
    theta = T0[wj0:j0 + h + 1, wi0:i0 + w + 1].min()
    reset = int((np.isfinite(T0) & (T0 >= theta)).sum())
    assert 0 < us["cells_invalidated"] <= reset
    if kind in ("hazard", "obstacle"):  # a small cone behind a disc
        assert us["cells_invalidated"] < 0.5 * reset
        assert r1.stats["tile_visits"] < r0.stats["tile_visits"]
