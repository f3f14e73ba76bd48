"""SURVEY s4.3 property tests on the GPU solve, at sizes the oracle cannot check
cell by cell in a test: each property holds for the reference FMM output
(propagateGlobalNode, src/DyMu_GlobalPathPlanning.cpp:500-546; the band only
grows through OPEN, non-obstacle 4-neighbours, :456-466), so it must hold for
the engine's map too.

* the finite mask is exactly the 4-connected component of non-obstacle cells
  that holds the goal (flood fill; scipy.ndimage.label as the checker);
* goal 0, obstacles +inf, every other finite cell > 0;
* monotone upwind: a finite non-goal cell is larger than the smallest of its
  4 neighbours (each candidate of :531-535 is >= min(Tx, Ty) + something > 0);
* mirror and transposition symmetry: the update is symmetric in Tx/Ty and in
  each axis (fmin, |Tx - Ty|, Tx + Ty), so a symmetric speed field with the goal
  on the symmetry axis gives a symmetric map -- up to the ulp-level freedom of
  the FIM fixed point, i.e. within the engine tolerance.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-12


def _flood_mask(F, goal):
    from scipy import ndimage

    free = np.isfinite(F)
    lab, _ = ndimage.label(free, structure=[[0, 1, 0], [1, 1, 1], [0, 1, 0]])
    return lab == lab[goal[1], goal[0]]


def _neighbour_min(T):
    inf = np.full_like(T[:1], np.inf)
    up = np.vstack([inf, T[:-1]])
    dn = np.vstack([T[1:], inf])
    infc = np.full_like(T[:, :1], np.inf)
    lf = np.hstack([infc, T[:, :-1]])
    rt = np.hstack([T[:, 1:], infc])
    return np.minimum(np.minimum(up, dn), np.minimum(lf, rt))


@pytest.mark.parametrize("N,frac", [(4096, 0.30), (8192, 0.02)])
def test_reachability_mask_and_invariants(dymu, oracle, N, frac):
    """30% obstacles at 4096^2: thousands of sealed pockets; 2% at 8192^2."""
    g = (N // 2 + 3, N // 2 - 5)
    F = oracle.synth_speed(N, N, seed=11, obst_frac=frac, obst_seed=13, goal=g)
    eng = dymu.Engine()
    try:
        T = eng.solve(F, *g).T
    finally:
        eng.close()
    fin = np.isfinite(T)
    reach = _flood_mask(F, g)
    assert np.array_equal(fin, reach), f"{np.count_nonzero(fin != reach)} cells differ"
    assert T[g[1], g[0]] == 0.0
    assert np.all(np.isinf(T[~np.isfinite(F)]))
    other = fin.copy()
    other[g[1], g[0]] = False
    assert np.all(T[other] > 0.0)
    # monotone upwind: strictly above the smallest neighbour
    assert np.all(T[other] > _neighbour_min(T)[other])


def _assert_close(a, b):
    assert np.array_equal(np.isinf(a), np.isinf(b))
    fin = np.isfinite(a)
    err = np.abs(a[fin] - b[fin]) / np.maximum(1.0, np.abs(b[fin]))
    assert err.max(initial=0.0) <= RTOL, f"max rel err {err.max()}"


@pytest.mark.parametrize("kernel", [3, 5])
def test_transpose_symmetry(dymu, oracle, kernel):
    N = 2048
    A = oracle.synth_speed(N, N, seed=21, obst_frac=0.03, obst_seed=22, goal=(N // 2, N // 2))
    F = np.minimum(A, A.T)  # +inf wins: obstacles symmetric too
    g = (N // 2, N // 2)
    eng = dymu.Engine(kernel=kernel)
    try:
        T = eng.solve(np.ascontiguousarray(F), *g).T
    finally:
        eng.close()
    _assert_close(T, T.T)


@pytest.mark.parametrize("kernel", [3, 5])
def test_mirror_symmetry(dymu, oracle, kernel):
    """Left-right mirror (odd width, goal on the middle column) and up-down."""
    nx, ny = 2049, 1537
    A = oracle.synth_speed(nx, ny, seed=31, obst_frac=0.03, obst_seed=32, goal=(nx // 2, ny // 2))
    F = np.ascontiguousarray(np.minimum(A, A[:, ::-1]))
    g = (nx // 2, ny // 3)
    F[g[1] - 1:g[1] + 2, g[0] - 1:g[0] + 2] = 1.0  # goal and its ring free, still symmetric
    eng = dymu.Engine(kernel=kernel)
    try:
        T = eng.solve(F, *g).T
        _assert_close(T, T[:, ::-1])
        ny2 = 2 * (ny // 2) + 1
        F2 = np.ascontiguousarray(np.minimum(A[:ny2], A[:ny2][::-1]))
        g2 = (nx // 3, ny2 // 2)
        F2[g2[1] - 1:g2[1] + 2, g2[0] - 1:g2[0] + 2] = 1.0
        T2 = eng.solve(F2, *g2).T
        _assert_close(T2, T2[::-1])
    finally:
        eng.close()
