"""Host planner (include/DyMu.hpp through include/dymu_planner.h) against the
oracle.  The cost-map and goal logic are host C++ and run on CPU; the solve
and path tests need the GPU (marked)."""
import os

import numpy as np
import pytest

from gen_golden import terrain_inputs

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RTOL = 1e-12


def gold(name):
    return np.load(os.path.join(GOLD, name + ".npy"), allow_pickle=False)


def oracle_global_cost(st):
    c = st["cost"] * (2 + st["hazard"] - st["traff"])
    return np.where(st["is_obstacle"] != 0, -1.0, c)


@pytest.mark.parametrize("res,N", [(0.5, 128), (1.0, 33), (0.5, 700)])
def test_compute_cost_map_bitwise(dymu, oracle, res, N):
    elev, terr, lut, slopes = terrain_inputs(N)
    p = dymu.Planner()
    assert p.initGlobalLayer(res, res / 4, N, N)
    st = oracle.new_state(N, N)
    for _ in range(2):  # second call exercises Q1 carry-over
        assert p.computeCostMap(lut, slopes, ["Wheel"], elev, terr)
        oracle.compute_cost_map(st, res, lut, slopes, 1, elev, terr)
        assert np.array_equal(p.getGlobalCostMatrix(), oracle_global_cost(st))
    assert np.array_equal(p.getHazardDensityMatrix(), st["hazard"])
    assert np.array_equal(p.getTrafficabilityMatrix(), st["traff"])
    assert p.getLocomotionMode((5 * res, 5 * res)) == "Wheel"


def test_compute_cost_map_multi_locomotion(dymu, oracle):
    N = 24
    j, i = np.mgrid[0:N, 0:N].astype(float)
    elev = 0.3 * np.sin(0.3 * i) + 0.1 * j
    terr = 1.0 + (i > 12)
    lut = np.array([50.0] * 6 + [1, 2, 4, 2, 2.5, 3] + [3, 3, 3, 1, 5, 9], dtype=float)
    slopes = np.array([0.0, 10.0, 20.0])
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    assert p.computeCostMap(lut, slopes, ["Wheel", "Walk"], elev, terr)
    st = oracle.new_state(N, N)
    oracle.compute_cost_map(st, 1.0, lut, slopes, 2, elev, terr)
    assert np.array_equal(p.getGlobalCostMatrix(), oracle_global_cost(st))
    for (x, y) in [(4, 4), (15, 7), (20, 20)]:
        m = st["loc_mode"][y, x]
        assert p.getLocomotionMode((x, y)) == (["Wheel", "Walk"][m] if m >= 0 else "DONT_CARE")


def test_set_cost_map_and_goal(dymu, oracle):
    cost = gold("setcost64_cost")
    N = cost.shape[0]
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N, offset=(10.0, -3.0))
    assert p.setCostMap(cost)
    obs = (cost <= 0).astype(np.uint8)
    for w in [(50.2, 18.1), (10.0, -3.0), (40.0, 30.0), (12.3, 44.4), (73.0, 60.0)]:
        ref = oracle.set_goal(N, N, 1.0, (10.0, -3.0), w, obs)
        assert p.setGoal(w) == (ref is not None), w
    assert not p.setCostMap(np.ones((N, N + 1)))  # size mismatch -> false (:112)


@pytest.mark.gpu
def test_entire_total_cost_map_setcost(dymu, oracle):
    cost = gold("setcost64_cost")
    g = tuple(int(x) for x in gold("setcost64_goal"))
    N = cost.shape[0]
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    p.setCostMap(cost)
    assert p.setGoal(g)
    assert p.computeEntireTotalCostMap()
    Tref = gold("setcost64_T")
    M = p.getTotalCostMatrix()
    ref = np.where(np.isinf(Tref), -1.0, Tref)
    assert np.array_equal(M == -1.0, ref == -1.0)
    fin = ref >= 0
    assert (np.abs(M[fin] - ref[fin]) / np.maximum(1, ref[fin])).max() <= RTOL
    st = p.lastStats()
    assert st["passes"] > 0


@pytest.mark.gpu
def test_entire_total_cost_map_terrain(dymu, oracle):
    elev, terr, lut, slopes = terrain_inputs(128)
    p = dymu.Planner()
    p.initGlobalLayer(0.5, 0.125, 128, 128)
    p.computeCostMap(lut, slopes, ["Wheel"], elev, terr)
    g = tuple(int(x) for x in gold("terrain128_goal"))
    assert p.setGoal((g[0] * 0.5, g[1] * 0.5))
    assert p.computeEntireTotalCostMap()
    T = p.totalCostRaw()
    Tref = gold("terrain128_T")
    assert np.array_equal(np.isinf(T), np.isinf(Tref))
    fin = np.isfinite(Tref)
    assert (np.abs(T[fin] - Tref[fin]) / np.maximum(1, Tref[fin])).max() <= RTOL


def _early_matches(M, Tt):
    """getTotalCostMatrix after computeTotalCostMap vs the reference's early-exit
    state: the never-reached mask (-1) exact, CLOSED values and the band's
    tentative values within the parity tolerance."""
    ref = np.where(np.isinf(Tt), -1.0, Tt)
    bad = np.argwhere((M == -1.0) != (ref == -1.0))
    assert bad.size == 0, (len(bad), [(tuple(b), M[tuple(b)], ref[tuple(b)]) for b in bad[:8]])
    fin = ref >= 0
    assert (np.abs(M[fin] - ref[fin]) / np.maximum(1, ref[fin])).max() <= RTOL


@pytest.mark.gpu
def test_compute_total_cost_map_returns(dymu, oracle):
    """computeTotalCostMap (:364-408) stops like the reference: the whole
    getTotalCostMatrix -- CLOSED values, the band's tentative values and -1 for
    the cells never reached -- equals the reference's early-exit state."""
    cost = gold("setcost64_cost")
    g = tuple(int(x) for x in gold("setcost64_goal"))
    N = cost.shape[0]
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    p.setCostMap(cost)
    p.setGoal(g)
    assert p.computeTotalCostMap((12, 50)) == bool(gold("early64_rc")[0])
    _early_matches(p.getTotalCostMatrix(), gold("early64_T"))
    assert p.lastBandSize() > 0
    assert not p.computeTotalCostMap((0.2, 30))        # border start: unsafe
    obs = np.argwhere(cost <= 0)[0]
    assert not p.computeTotalCostMap((obs[1], obs[0]))  # on an obstacle


@pytest.mark.gpu
def test_global_narrowband_after_early_exit(dymu, oracle):
    """global_narrowband (src/DyMu.hpp:445) after computeTotalCostMap holds the
    reference's band nodes -- reached but not CLOSED (early64_closed) -- and
    minCostGlobalNode (:548-567) pops them lowest total cost first."""
    cost = gold("setcost64_cost")
    g = tuple(int(x) for x in gold("setcost64_goal"))
    N = cost.shape[0]
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    p.setCostMap(cost)
    p.setGoal(g)
    assert p.computeTotalCostMap((12, 50))
    Tt, closed = gold("early64_T"), gold("early64_closed").astype(bool)
    ref = np.isfinite(Tt) & ~closed
    band = p.globalNarrowband()
    assert len(band) == p.lastBandSize() == int(ref.sum())
    got = np.zeros_like(ref)
    got[band[:, 1], band[:, 0]] = True
    assert np.array_equal(got, ref)
    M = p.getTotalCostMatrix()
    vals, gvals = np.sort(M[ref]), np.sort(Tt[ref])
    for k in range(3):
        (i, j), t = p.minCostGlobalNode()
        assert ref[j, i] and t == M[j, i] == vals[k]
        assert abs(t - gvals[k]) <= RTOL * max(1.0, t)
    assert p.lastBandSize() == int(ref.sum()) - 3


@pytest.mark.gpu
def test_early_exit_far_start_256(dymu, oracle):
    """A start far from the goal on a 256^2 map with obstacles (golden from the
    oracle's exact reference pop order)."""
    cost = gold("early256_cost")
    gi, gj, si, sj = (int(x) for x in gold("early256_goal_start"))
    N = cost.shape[0]
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    p.setCostMap(cost)
    assert p.setGoal((gi, gj))
    assert p.computeTotalCostMap((si, sj)) == bool(gold("early256_rc")[0])
    _early_matches(p.getTotalCostMatrix(), gold("early256_T"))
    # the state drives getTotalCost's CLOSED test (:873-876) like the reference's
    closed = gold("early256_closed").astype(bool)
    Tt = gold("early256_T")
    for (x, y) in [(si + 0.3, sj + 0.6), (gi - 2.5, gj + 0.25), (100.5, 100.5)]:
        i, j = int(x), int(y)
        a, b = x - i, y - j
        if closed[j, i] and closed[j, i + 1] and closed[j + 1, i] and closed[j + 1, i + 1]:
            w00, w10, w01, w11 = Tt[j, i], Tt[j, i + 1], Tt[j + 1, i], Tt[j + 1, i + 1]
            exp = w00 + (w10 - w00) * a + (w01 - w00) * b + (w11 + w00 - w10 - w01) * a * b
        else:
            exp = Tt[int(y + 0.5), int(x + 0.5)]
        got = p.getTotalCost((x, y))
        assert (np.isinf(exp) and np.isinf(got)) or abs(got - exp) <= RTOL * max(1, abs(exp))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_early_exit_random_vs_oracle(dymu, oracle, seed):
    """Random maps and starts against the oracle's early exit; a start next to
    the goal runs fewer passes than the full solve."""
    rng = np.random.default_rng(100 + seed)
    N = int(rng.integers(48, 160))
    g = (int(rng.integers(4, N - 4)), int(rng.integers(4, N - 4)))
    F = oracle.synth_speed(N, N, seed=200 + seed, obst_frac=0.04, obst_seed=300 + seed, goal=g)
    cost = np.where(np.isfinite(F), F, -1.0)
    for _ in range(200):
        s = (int(rng.integers(2, N - 2)), int(rng.integers(2, N - 2)))
        if np.isfinite(F[s[1] - 1:s[1] + 2, s[0] - 1:s[0] + 2]).all():
            break
    assert np.isfinite(F[s[1] - 1:s[1] + 2, s[0] - 1:s[0] + 2]).all()
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    p.setCostMap(cost)
    assert p.setGoal(g)
    Tt, rc, _ = oracle.fmm(F, g, start=s, want_closed=True)
    assert p.computeTotalCostMap(s) == bool(rc)
    _early_matches(p.getTotalCostMatrix(), Tt)
    # near start: fewer passes than computeEntireTotalCostMap
    near = (g[0] + 1, g[1])
    p.computeTotalCostMap(near)
    near_passes = p.lastStats()["passes"]
    p.computeEntireTotalCostMap()
    assert near_passes < p.lastStats()["passes"]


@pytest.mark.gpu
@pytest.mark.parametrize("inputs", ["splitmix", "mt19937"])
def test_config1_exact_call(dymu, oracle, inputs):
    """BASELINE config 1 as the caller makes it: a 512^2
    setCostMap grid without obstacles, goal (256, 256), computeTotalCostMap from
    the start (102, 128) (:364-408) -- the whole getTotalCostMatrix (CLOSED values,
    the band's tentative values, -1 never reached) against the oracle's exact
    early exit -- then computeEntireTotalCostMap (:443-468) on the same planner
    against the oracle's full FMM.  Both generators: the counter-based U(1,5) of
    the synthetic configs and the reference-run KAT input (mt19937_64(1))."""
    N, g, s = 512, (256, 256), (102, 128)
    if inputs == "splitmix":
        F = oracle.synth_speed(N, N, seed=1, obst_frac=0.0, obst_seed=3, goal=g)
    else:
        F = oracle.mt_uniform(N * N).reshape(N, N)
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    p.setCostMap(F)
    assert p.setGoal(g)
    Tt, rc, _ = oracle.fmm(F, g, start=s, want_closed=True)
    assert rc == 1  # the reference returns true: the band is not empty at the exit
    assert p.computeTotalCostMap(s)
    M = p.getTotalCostMatrix()
    _early_matches(M, Tt)
    assert 0 < p.lastBandSize() and (M == -1.0).any()  # stopped before the map was covered
    assert p.computeEntireTotalCostMap()
    Tref, _ = oracle.fmm(F, g)
    M = p.getTotalCostMatrix()
    assert np.array_equal(M == -1.0, np.isinf(Tref))
    assert (np.abs(M - Tref) / np.maximum(1, Tref)).max() <= RTOL
    if inputs == "mt19937":  # the reference-run KAT through the class surface
        assert f"{M.sum():.10e}" == "1.3467278246e+08"


@pytest.mark.gpu
@pytest.mark.parametrize("N,g,s", [(160, (80, 80), (20, 140)), (512, (256, 256), (102, 128)),
                                   (96, (48, 48), (48, 20)), (2048, (1024, 1024), (200, 1900)),
                                   (4096, (2048, 2048), (2867, 2457))])  # a 1:2 staircase front
def test_early_exit_ties_exact(dymu, oracle, N, g, s):
    """computeTotalCostMap on a constant-speed map, where every mirror image ties:
    which of the cells of exactly the exit value the reference closed, and so which
    cells it reached, depends on its insertion order (:551-568).  The planner
    rebuilds that order from the values (csrc/pop_order.hpp) instead of replaying
    the FMM: the never-reached mask and every node state are the reference's, the
    values within the parity tolerance, the band in the reference's insertion order
    (oracle_fmm_order's sequence), and no exact host replay ran."""
    F = np.ones((N, N))
    p = dymu.Planner()
    try:
        p.initGlobalLayer(1.0, 0.5, N, N)
        p.setCostMap(F)
        assert p.setGoal(g)
        Tl, rc, closed, seq = oracle.fmm_order(F, g, start=s)
        assert p.computeTotalCostMap(s) == bool(rc)
        info = p.lastEarlyExit()
        forced = os.environ.get("DYMU_EXACT_EXIT", "0") != "0"  # the exact replay's parity
        assert (forced or not info["exact_replay"]) and info["tied"] > 1 and info["band_exact"]
        M = p.getTotalCostMatrix()
        _early_matches(M, Tl)
        band = (closed == 0) & np.isfinite(Tl)
        assert p.lastBandSize() == int(band.sum())
        nb = p.globalNarrowband()
        bj, bi = np.nonzero(band)
        want = np.stack([bi, bj], 1)[np.argsort(seq[bj, bi], kind="stable")]
        assert np.array_equal(nb, want)  # the reference's band vector, in its order
        if N <= 512:
            for j in range(N):
                for i in range(0, N, 7 if N > 160 else 1):
                    assert p.getGlobalNode(i, j)["state"] == int(closed[j, i]), (i, j)
        for (i, j) in [s, g, (s[0] + 1, s[1]), tuple(nb[0]), tuple(nb[-1])]:
            assert p.getGlobalNode(int(i), int(j))["state"] == int(closed[j, i])
        (i, j), t = p.minCostGlobalNode()  # first strict minimum in insertion order
        vals = np.array([M[y, x] for x, y in nb])
        assert (i, j) == tuple(nb[int(np.argmin(vals))]) and t == vals.min()
    finally:
        p.close()


@pytest.mark.gpu
def test_early_exit_false_returns(dymu, oracle):
    """The reference returns false when the band is empty at exit (:399-403):
    a start enclosed by obstacles (unreachable), and a start whose neighbourhood
    closes last of all the reachable nodes (expensive start cells)."""
    N = 40
    cost = np.ones((N, N))
    cost[24:33, 24:33] = -1.0
    cost[25:32, 25:32] = 1.0   # a free room inside a wall: unreachable
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    p.setCostMap(cost)
    assert p.setGoal((8, 8))
    F = np.where(cost > 0, cost * 1.0, np.inf)
    Tt, rc, _ = oracle.fmm(F, (8, 8), start=(28, 28), want_closed=True)
    assert rc == 0
    assert not p.computeTotalCostMap((28, 28))
    _early_matches(p.getTotalCostMatrix(), Tt)
    cost2 = np.ones((N, N))
    for (i, j) in [(20, 20), (20, 19), (19, 20), (21, 20), (20, 21)]:
        cost2[j, i] = 1000.0  # the start and its nb4 close after everything else
    p2 = dymu.Planner()  # setCostMap never clears an obstacle flag (:117-123)
    p2.initGlobalLayer(1.0, 0.5, N, N)
    p2.setCostMap(cost2)
    assert p2.setGoal((8, 8))
    F2 = cost2 * 1.0
    Tt2, rc2, _ = oracle.fmm(F2, (8, 8), start=(20, 20), want_closed=True)
    assert rc2 == 0
    assert not p2.computeTotalCostMap((20, 20))
    _early_matches(p2.getTotalCostMatrix(), Tt2)


@pytest.mark.gpu
def test_get_path_matches_oracle(dymu, oracle):
    """getPath (:589-611) on GPU-produced T vs the oracle's restatement on the
    oracle's T: same waypoint count, positions within 1e-9."""
    N = 96
    F = oracle.synth_speed(N, N, seed=21, obst_frac=0.0, goal=(70, 60))
    cost = F.copy()
    p = dymu.Planner(risk_distance=0.5)
    p.initGlobalLayer(1.0, 0.5, N, N, offset=(100.0, 200.0))
    p.setCostMap(cost)
    assert p.setGoal((170.0, 260.0, 0.0, 1.25))
    assert p.computeEntireTotalCostMap()
    path = p.getPath((100.0 + 12.5, 200.0 + 20.25, 0.0, 0.3))
    Tref, _ = oracle.fmm(F, (70, 60))
    n, wp = oracle.global_path(Tref, (70, 60), res=1.0, start=(12.5, 20.25, 0.3),
                               risk_distance=0.5, goal_heading=1.25)
    assert n == len(path) and n > 20
    wp[:, 0] += 100.0
    wp[:, 1] += 200.0
    assert np.abs(path[:, :2] - wp[:, :2]).max() < 1e-9
    assert np.abs(path[:, 3] - wp[:, 3]).max() < 1e-9
    assert path[-1, 0] == 170.0 and path[-1, 1] == 260.0 and path[-1, 3] == 1.25


@pytest.mark.gpu
def test_get_total_cost_interpolation(dymu, oracle):
    N = 48
    F = oracle.synth_speed(N, N, seed=4, goal=(30, 30))
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    p.setCostMap(F)
    p.setGoal((30, 30))
    p.computeEntireTotalCostMap()
    T = p.totalCostRaw()
    x, y = 10.25, 7.5
    i, j, a, b = 10, 7, 0.25, 0.5
    w00, w10, w01, w11 = T[j, i], T[j, i + 1], T[j + 1, i], T[j + 1, i + 1]
    exp = w00 + (w10 - w00) * a + (w01 - w00) * b + (w11 + w00 - w10 - w01) * a * b
    assert p.getTotalCost((x, y)) == exp


@pytest.mark.gpu
def test_dynamic_hazard_feedback(dymu, oracle):
    """hazard_density / trafficability feed the next solve through the speed
    C = res*cost*(2+hd-tr) (:527-528), e.g. after a local repair."""
    N = 64
    F = oracle.synth_speed(N, N, seed=8, goal=(32, 32))
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    p.setCostMap(F)
    p.setGoal((32, 32))
    hd = np.zeros((N, N))
    hd[10:20, 10:20] = 1.0
    tr = np.ones((N, N))
    tr[40:50, 5:15] = 0.5
    assert p.setHazardDensity(hd) and p.setTrafficability(tr)
    p.computeEntireTotalCostMap()
    Fr = oracle.pack_speed(F, hd, tr, None, res=1.0)
    Tref, _ = oracle.fmm(Fr, (32, 32))
    T = p.totalCostRaw()
    fin = np.isfinite(Tref)
    assert (np.abs(T[fin] - Tref[fin]) / np.maximum(1, Tref[fin])).max() <= RTOL


@pytest.mark.gpu
def test_incremental_resolve_through_planner(dymu, oracle):
    """Config 5 through the class surface: a hazard bump on a disc (the local
    layer's write, LocalPathRepairing.cpp:264-274) followed by
    computeTotalCostMap re-propagates from the changed window only
    (lastSolveKind 1) and equals the cold solve / oracle; an unchanged speed
    reuses the map (2); a goal change solves cold (0)."""
    N = 200
    F = oracle.synth_speed(N, N, seed=12, obst_frac=0.02, obst_seed=13, goal=(150, 150))
    F[158:163, 38:43] = 2.0  # room for the second goal
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    p.setCostMap(np.where(np.isfinite(F), F, -1.0))
    assert p.setGoal((150, 150))
    assert p.computeEntireTotalCostMap() and p.lastSolveKind() == 0
    cold_visits = p.lastStats()["tile_visits"]
    assert p.computeEntireTotalCostMap() and p.lastSolveKind() == 2
    hd = p.getHazardDensityMatrix()
    j, i = np.mgrid[0:N, 0:N]
    inner = (i - 60) ** 2 + (j - 50) ** 2 <= 15 ** 2
    ring = ((i - 60) ** 2 + (j - 50) ** 2 <= 16 ** 2) & ~inner
    hd[inner] = np.minimum(1.0, hd[inner] + 1.0)
    hd[ring] = np.minimum(1.0, hd[ring] + 0.1)
    assert p.setHazardDensity(hd)
    p.computeEntireTotalCostMap()
    assert p.lastSolveKind() == 1
    assert p.lastStats()["tile_visits"] < cold_visits
    obst = ~np.isfinite(F)
    Fr = oracle.pack_speed(np.where(obst, -1.0, F), hd, p.getTrafficabilityMatrix(), obst,
                           res=1.0)
    Tref, _ = oracle.fmm(Fr, (150, 150))
    T = p.totalCostRaw()
    assert np.array_equal(np.isinf(T), np.isinf(Tref))
    fin = np.isfinite(Tref)
    assert (np.abs(T[fin] - Tref[fin]) / np.maximum(1, Tref[fin])).max() <= RTOL
    assert p.setGoal((40, 160))
    p.computeEntireTotalCostMap()
    assert p.lastSolveKind() == 0


@pytest.mark.gpu
def test_decrease_only_window_through_planner(dymu, oracle):
    """C = res*cost*(2+hd-tr) grows when the trafficability drops (the local
    layer's write on a replaced segment, LocalPathRepairing.cpp:389-394): an
    increase, re-propagated with the theta reset; restoring it is a decrease,
    re-propagated without any reset.  Both through the windowed setter; each
    result equals the oracle FMM of the new speed."""
    N = 160
    F = oracle.synth_speed(N, N, seed=17, obst_frac=0.02, obst_seed=19, goal=(120, 30))
    cost = np.where(np.isfinite(F), F, -1.0)
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    p.setCostMap(cost)
    assert p.setGoal((120, 30))
    p.computeEntireTotalCostMap()
    win = (40, 90, 12, 9)  # i0, j0, w, h
    i0, j0, w, h = win
    obst = ~np.isfinite(F)
    visits = {}
    for name, tr_val in (("up", 0.25), ("down", 1.0)):  # tr drop raises C; restoring lowers it
        assert p.setTrafficabilityWindow(i0, j0, np.full((h, w), tr_val))
        p.computeEntireTotalCostMap()
        assert p.lastSolveKind() == 1
        visits[name] = p.lastStats()["tile_visits"]
        Fr = oracle.pack_speed(cost, p.getHazardDensityMatrix(), p.getTrafficabilityMatrix(),
                               obst, res=1.0)
        Tref, _ = oracle.fmm(Fr, (120, 30))
        T = p.totalCostRaw()
        assert np.array_equal(np.isinf(T), np.isinf(Tref))
        fin = np.isfinite(Tref)
        assert (np.abs(T[fin] - Tref[fin]) / np.maximum(1, Tref[fin])).max() <= RTOL
    assert visits["down"] <= visits["up"]


def test_terrain_class_beyond_lut_is_obstacle(dymu, oracle):
    """A terrain class the LUT does not cover (an out-of-bounds read in the
    reference, :237-241 / :270-273) becomes an obstacle, on the host as in the
    device kernel (cost_kernels.hip); every other cell matches the oracle."""
    from gen_golden import terrain_inputs
    N = 32
    elev, terr, lut, slopes = terrain_inputs(N)  # LUT covers terrain 0..2
    terr = terr.copy()
    terr[10:14, 10:14] = 3.0
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    assert p.computeCostMap(lut, slopes, ["Wheel"], elev, terr)
    G = p.getGlobalCostMatrix()
    assert (G[10:14, 10:14] == -1.0).all()
    terr_ok = terr.copy()
    terr_ok[10:14, 10:14] = 1.0
    st = oracle.new_state(N, N)
    oracle.compute_cost_map(st, 1.0, lut, slopes, 1, elev, terr_ok)
    ref = oracle_global_cost(st)
    mask = np.ones((N, N), bool)
    mask[9:15, 9:15] = False  # the block and the ring its raw cost is smoothed into
    assert np.array_equal(G[mask], ref[mask])


@pytest.mark.gpu
def test_total_cost_readbacks_chunked(dymu, oracle):
    """copyTotalCost's chunked download (a stale mirror with >= 1024 rows goes down in
    16 row chunks, each copied out while the next downloads): raw and -1 forms, both
    orders, ragged last chunk, and blocks already fetched by a point query."""
    nx, ny, goal = 640, 1100, (300, 700)
    F = oracle.synth_speed(nx, ny, seed=12, obst_frac=0.03, obst_seed=13, goal=goal)
    Tref, _ = oracle.fmm(F, goal)
    Mref = np.where(np.isinf(Tref), -1.0, Tref)
    p = dymu.Planner()
    assert p.initGlobalLayer(1.0, 0.5, nx, ny)
    assert p.setCostMap(np.where(np.isfinite(F), F, -1.0))
    for first_raw in (True, False):
        assert p.setGoal(goal)
        assert p.computeEntireTotalCostMap()
        p.getTotalCost((17.0, 1050.0))  # one mirror block fetched on its own
        a = p.totalCostRaw() if first_raw else p.getTotalCostMatrix()
        b = p.getTotalCostMatrix() if first_raw else p.totalCostRaw()
        T, M = (a, b) if first_raw else (b, a)
        assert T.shape == (ny, nx) and M.shape == (ny, nx)
        assert np.array_equal(np.isinf(T), np.isinf(Tref))
        assert np.array_equal(M == -1.0, Mref == -1.0)
        fin = np.isfinite(Tref)
        assert (np.abs(T[fin] - Tref[fin]) / np.maximum(1, Tref[fin])).max() <= RTOL
        assert np.array_equal(np.where(np.isinf(T), -1.0, T), M)
        # a second solve with another goal leaves no stale rows behind
        assert p.setGoal((goal[0] + 1, goal[1]))
        assert p.computeEntireTotalCostMap()
        T2 = p.totalCostRaw()
        assert T2[goal[1], goal[0] + 1] == 0.0 and T2[goal[1], goal[0]] > 0.0
