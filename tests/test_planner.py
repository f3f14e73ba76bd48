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


@pytest.mark.parametrize("res,N", [(0.5, 128), (1.0, 33)])
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


@pytest.mark.gpu
def test_compute_total_cost_map_returns(dymu, oracle):
    cost = gold("setcost64_cost")
    g = tuple(int(x) for x in gold("setcost64_goal"))
    N = cost.shape[0]
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    p.setCostMap(cost)
    p.setGoal(g)
    # the golden early-exit run: reference returns 1 and has closed the start
    assert p.computeTotalCostMap((12, 50)) == bool(gold("early64_rc")[0])
    T = p.totalCostRaw()
    Tt, closed = gold("early64_T"), gold("early64_closed").astype(bool)
    # CLOSED cells hold final values in the reference; they must agree
    assert (np.abs(T[closed] - Tt[closed]) / np.maximum(1, Tt[closed])).max() <= RTOL
    assert not p.computeTotalCostMap((0.2, 30))        # border start: unsafe
    obs = np.argwhere(cost <= 0)[0]
    assert not p.computeTotalCostMap((obs[1], obs[0]))  # on an obstacle


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
