"""Edge-case parity of every pass kernel against the oracle FMM: special speed
values and degenerate maps.

dymu_fim.h's contract: F >= 0 or +inf, and NaN counts as an obstacle (the
oracle's is_blocked, restating the reference's isObstacle skip at
src/DyMu_GlobalPathPlanning.cpp:463-465).  The kernels take the range-restricted
sqrt only when every speed of the tile is >= 2^-383; tiny speeds
exercise the library sqrt path, huge ones overflow 2*C^2 to +inf inside the
two-sided candidate (:531-535), exactly as the reference arithmetic does.
"""
import numpy as np
import pytest

from test_gpu_solver import assert_parity

pytestmark = pytest.mark.gpu


def _fmm(oracle, F, g):
    Tref, _ = oracle.fmm(F, g)
    return Tref


@pytest.mark.parametrize("case", ["nan", "zero", "tiny", "c2_near_max", "mixed_scales"])
def test_special_speeds(kengine, oracle, case):
    nx, ny, g = 200, 150, (70, 90)
    rng = np.random.default_rng(5)
    F = oracle.synth_speed(nx, ny, seed=17, obst_frac=0.03, obst_seed=19, goal=g)
    pick = rng.random((ny, nx)) < 0.05
    pick[g[1] - 1:g[1] + 2, g[0] - 1:g[0] + 2] = False
    if case == "nan":
        F[pick] = np.nan
    elif case == "zero":
        F[pick] = 0.0
    elif case == "tiny":
        F = F * 1e-300  # every tile below 2^-383: the library sqrt path
    elif case == "c2_near_max":
        F = np.where(np.isfinite(F), 7.0e153, F)  # 2*C^2 = 9.8e307 > 2^1023, still finite
    else:
        F[pick] = F[pick] * 1e-200
        F[rng.random((ny, nx)) < 0.02] *= 1e150
        F[g[1], g[0]] = 1.0
    F = np.ascontiguousarray(F)
    r = kengine.solve(F, *g)
    Tref = _fmm(oracle, F, g)
    assert_parity(r.T, Tref)
    if case == "nan":
        assert np.all(np.isinf(r.T[pick]))


def test_goal_walled_in(kengine, oracle):
    """Goal sealed by a ring of obstacles: only the goal is finite."""
    nx, ny, g = 97, 61, (40, 30)
    F = np.full((ny, nx), 2.0)
    F[g[1] - 2:g[1] + 3, g[0] - 2:g[0] + 3] = np.inf
    F[g[1] - 1:g[1] + 2, g[0] - 1:g[0] + 2] = 1.0
    F[g[1], g[0]] = 1.0
    r = kengine.solve(F, *g)
    fin = np.isfinite(r.T)
    assert np.count_nonzero(fin) == 9 and r.T[g[1], g[0]] == 0.0
    assert_parity(r.T, _fmm(oracle, F, g))


def test_everything_blocked_but_goal(kengine, oracle):
    nx, ny, g = 64, 48, (10, 20)
    F = np.full((ny, nx), np.inf)
    F[g[1], g[0]] = 3.0
    r = kengine.solve(F, *g)
    assert np.count_nonzero(np.isfinite(r.T)) == 1 and r.T[g[1], g[0]] == 0.0
    assert_parity(r.T, _fmm(oracle, F, g))


def test_goal_on_obstacle_cell(kengine, oracle):
    """The engine seeds T = 0 at the goal whatever its speed (the planner's setGoal
    rejects such goals, :346-351); its neighbours propagate from it."""
    nx, ny, g = 80, 80, (40, 40)
    F = oracle.synth_speed(nx, ny, seed=3, obst_frac=0.0, obst_seed=4, goal=g)
    F[g[1], g[0]] = np.inf
    r = kengine.solve(np.ascontiguousarray(F), *g)
    assert_parity(r.T, _fmm(oracle, F, g))


def test_overflowing_speed_terminates(kengine, oracle):
    """C > 1.34e154: 2*C^2 overflows, the two-sided candidate of :531-535 is +inf
    once both axis neighbours are finite, and the update is no longer monotone --
    whether a cell ever takes a finite (one-sided) value depends on the order in
    which its neighbours became finite, so the reference's own result depends on
    its pop order and no schedule-independent map exists (parity is stated for
    2*C^2 finite).  The engine still terminates, keeps the goal at
    0 and obstacles at +inf, and every finite value is a one-sided candidate of
    a finite neighbour (>= the smallest neighbour + C)."""
    nx, ny, g = 200, 150, (70, 90)
    F = np.ascontiguousarray(
        oracle.synth_speed(nx, ny, seed=17, obst_frac=0.03, obst_seed=19, goal=g) * 1e300)
    T = kengine.solve(F, *g).T
    assert T[g[1], g[0]] == 0.0
    assert np.all(np.isinf(T[~np.isfinite(F)]))
    inf = np.full((1, nx), np.inf)
    infc = np.full((ny, 1), np.inf)
    nbmin = np.minimum(np.minimum(np.vstack([inf, T[:-1]]), np.vstack([T[1:], inf])),
                       np.minimum(np.hstack([infc, T[:, :-1]]), np.hstack([T[:, 1:], infc])))
    fin = np.isfinite(T)
    fin[g[1], g[0]] = False
    assert np.all(T[fin] >= nbmin[fin] + F[fin])
