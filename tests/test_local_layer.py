"""The local layer (path repairing, src/DyMu_LocalPathRepairing.cpp) of the
product planner (csrc/local_layer.cpp through include/dymu_planner.h) against
the oracle restatement (oracle/oracle_local.c), bit for bit.

Both run on the host over the same global layer: the total-cost map comes
from the oracle's heap FMM (the reference's pop order) and is installed in the
planner with loadTotalCostMap -- the local layer only reads it -- so these
tests run on CPU.  The GPU-produced map feeds the same code in
tests/test_gpu_local.py.
"""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def same(a, b):
    """bitwise equality, NaN == NaN"""
    a = np.asarray(a)
    b = np.asarray(b)
    return a.shape == b.shape and np.array_equal(a, b, equal_nan=True)


def disc_image(rover, centre, radius, res, size):
    """size x size traversability image at res m/pixel centred on rover (image
    convention: row j at y = rover_y + res*size/2 - j*res, :225-238) with a disc
    of obstacles (value 1)."""
    img = np.zeros((size, size), dtype=np.uint8)
    ox = rover[0] - res * size / 2
    oy = rover[1] + res * size / 2
    j, i = np.mgrid[0:size, 0:size]
    px = ox + i * res
    py = oy - j * res
    img[(px - centre[0]) ** 2 + (py - centre[1]) ** 2 <= radius ** 2] = 1
    return img


def build(dymu, oracle, N, lres, approach, offset=(0.0, 0.0), seed=5, goal=(38, 34),
          obst_frac=0.0, risk_distance=1.0, reconnect_distance=1.5, risk_ratio=5.0):
    F = oracle.synth_speed(N, N, seed=seed, obst_frac=obst_frac, obst_seed=seed + 1, goal=goal)
    cost = np.where(np.isfinite(F), F, -1.0)
    T, _ = oracle.fmm(F, goal)
    p = dymu.Planner(risk_distance=risk_distance, reconnect_distance=reconnect_distance,
                     risk_ratio=risk_ratio, approach=approach)
    assert p.initGlobalLayer(1.0, lres, N, N, offset=offset)
    assert p.setCostMap(cost)
    assert p.setGoal((goal[0] + offset[0], goal[1] + offset[1], 0.0, 0.7))
    assert p.loadTotalCostMap(T)
    o = oracle.local(N, N, 1.0, lres, offset=offset, risk_distance=risk_distance,
                     reconnect_distance=reconnect_distance, risk_ratio=risk_ratio,
                     approach=approach)
    o.set_global((cost <= 0).astype(np.uint8), T, goal, goal_heading=0.7,
                 hazard=p.getHazardDensityMatrix(), traff=p.getTrafficabilityMatrix())
    return p, o


def compare_state(p, o, rover):
    hd_o, tr_o = o.hazard_traff()
    assert same(p.getHazardDensityMatrix(), hd_o)
    assert same(p.getTrafficabilityMatrix(), tr_o)
    mask = p.localMapMask()
    assert same(mask, o.map_mask())
    for j, i in np.argwhere(mask):
        a, b = p.localBlock(int(i), int(j)), o.block(int(i), int(j))
        for x, y in zip(a, b):
            assert same(x, y), (i, j)
    assert same(p.getRiskMatrix(rover), o.risk_matrix(rover[0], rover[1]))
    assert same(p.getDeviationMatrix(rover), o.deviation_matrix(rover[0], rover[1]))
    assert p.getReconnectingIndex() == o.reconnecting_index()
    assert same(p.current_path, o.path)


@pytest.mark.parametrize("approach", [0, 1], ids=["conservative", "sweeping"])
@pytest.mark.parametrize("lres", [0.25, 0.1])
def test_local_planning_matches_oracle(dymu, oracle, approach, lres):
    N = 48
    p, o = build(dymu, oracle, N, lres, approach)
    start = (8.3, 9.6, 0.0, 0.0)
    path = p.getPath(start)
    n_o, path_o = o.get_path(start)
    assert len(path) > 20 and n_o == len(path)
    assert same(path, path_o)
    # an obstacle disc on the path ~4 m ahead of the rover
    k = min(12, len(path) - 2)
    rover = tuple(path[2][:2])
    centre = tuple(path[k][:2])
    img = disc_image(rover, centre, 0.8, lres, int(round(9.0 / lres)))
    rep, traj, _ = p.computeLocalPlanning(rover + (0.0, 0.0), img, lres)
    rep_o, traj_o = o.local_planning(rover + (0.0, 0.0), img, lres)
    assert rep == rep_o
    assert rep, "the disc sits on the path: it must be repaired"
    assert same(traj, traj_o)
    compare_state(p, o, rover)
    # the repaired path avoids the disc
    d = np.hypot(traj[:, 0] - centre[0], traj[:, 1] - centre[1])
    assert d.min() > 0.8
    # getPath after the repair walks evaluatePath over the local maps
    path2 = p.getPath(start)
    n2, path2_o = o.get_path(start)
    assert same(path2, path2_o)
    compare_state(p, o, rover)


def test_local_planning_offset_and_obstacles(dymu, oracle):
    """A non-zero map offset (the reference subtracts it again inside the local
    layer's global lookups, kept) and global obstacles next to the rover."""
    N = 40
    off = (3.0, -2.0)
    p, o = build(dymu, oracle, N, 0.2, 0, offset=off, seed=9, goal=(30, 28), obst_frac=0.03)
    start = (6.1 + off[0], 7.2 + off[1])
    path = p.getPath(start)
    n_o, path_o = o.get_path(start)
    assert same(path, path_o)
    rover = tuple(path[1][:2])
    centre = tuple(path[min(10, len(path) - 2)][:2])
    img = disc_image((rover[0] + off[0], rover[1] + off[1]),
                     (centre[0] + off[0], centre[1] + off[1]), 0.6, 0.2, 40)
    w = (rover[0] + off[0], rover[1] + off[1], 0.0, 0.0)
    rep, traj, _ = p.computeLocalPlanning(w, img, 0.2)
    rep_o, traj_o = o.local_planning(w, img, 0.2)
    assert rep == rep_o
    assert same(traj, traj_o)
    compare_state(p, o, rover)


def test_local_planning_not_blocked(dymu, oracle):
    """Obstacles away from the path: hazard feedback only, no repair (:278-290)."""
    N = 40
    p, o = build(dymu, oracle, N, 0.25, 1, goal=(30, 30))
    start = (6.0, 6.0)
    path = p.getPath(start)
    o.get_path(start)
    rover = tuple(path[1][:2])
    img = disc_image(rover, (rover[0] + 3.0, rover[1] - 3.0), 0.5, 0.25, 32)
    rep, traj, _ = p.computeLocalPlanning(rover, img, 0.25)
    rep_o, _ = o.local_planning(rover, img, 0.25)
    assert not rep and not rep_o and len(traj) == 0
    compare_state(p, o, rover)
    assert p.getHazardDensityMatrix().max() > 0


@pytest.mark.parametrize("approach", [0, 1])
def test_repeated_planning_accumulates(dymu, oracle, approach):
    """Several local planning calls along the drive: the sub-grid, risk and
    hazard accumulate and repairs chain through reconnecting_index."""
    N = 56
    p, o = build(dymu, oracle, N, 0.25, approach, goal=(44, 40), seed=13)
    start = (6.4, 8.9)
    path = p.getPath(start)
    o.get_path(start)
    rng = np.random.default_rng(3)
    for step in range(3):
        cur = p.current_path
        if len(cur) < 8:
            break
        rover = tuple(cur[1][:2])
        k = min(len(cur) - 2, 6 + int(rng.integers(0, 4)))
        centre = tuple(cur[k][:2] + rng.normal(0, 0.3, 2))
        img = disc_image(rover, centre, 0.5 + 0.2 * step, 0.25, 40)
        rep, traj, _ = p.computeLocalPlanning(rover, img, 0.25)
        rep_o, traj_o = o.local_planning(rover, img, 0.25)
        assert rep == rep_o
        assert same(traj, traj_o)
        compare_state(p, o, rover)


def test_node_level_access(dymu, oracle):
    N = 24
    p, o = build(dymu, oracle, N, 0.5, 0, goal=(12, 12))
    n = p.getGlobalNode(12, 12)
    assert n["total_cost"] == 0.0 and n["state"] == 1 and not n["has_local_map"]
    assert p.getGlobalNode(N, 0) is None
    assert p.isSafeNode(12, 12) and p.isFullyClosedNode(12, 12)
    assert not p.isFullyClosedNode(0, 5)
    p.computeLocalPropagation((5.0, 5.0), (9.0, 9.0))
    assert p.getGlobalNode(5, 5)["has_local_map"]
    p.resetTotalCostMap()
    assert p.getGlobalNode(12, 12)["state"] == 0
    assert np.isinf(p.getGlobalNode(12, 12)["total_cost"])


def test_band_and_gradient_accessors(dymu, oracle):
    """resetGlobalNarrowBand / minCostGlobalNode (:487-498, :548-567) on an
    installed map, and gradientNode (:718-772) against the formula."""
    N = 24
    p, o = build(dymu, oracle, N, 0.5, 0, goal=(12, 12))
    assert len(p.globalNarrowband()) == 0 and p.minCostGlobalNode() is None
    p.resetGlobalNarrowBand()
    assert p.globalNarrowband().tolist() == [[12, 12]]
    assert p.minCostGlobalNode() == ((12, 12), 0.0)
    assert p.minCostGlobalNode() is None
    T = p.getTotalCostMatrix()
    T = np.where(T < 0, np.inf, T)
    for (i, j) in [(5, 7), (0, 3), (23, 10), (12, 12), (3, 0)]:
        def d(a, b, c, ha, hc):  # one axis of :718-772 (a below, c above)
            if (not ha and not hc) or (ha and hc and np.isinf(a) and np.isinf(c)):
                return 0.0
            if not ha or np.isinf(a):
                return c - b
            if not hc or np.isinf(c):
                return b - a
            return (c - a) * 0.5
        get = lambda x, y: T[y, x] if 0 <= x < N and 0 <= y < N else np.inf
        dx = d(get(i - 1, j), T[j, i], get(i + 1, j), i > 0, i + 1 < N)
        dy = d(get(i, j - 1), T[j, i], get(i, j + 1), j > 0, j + 1 < N)
        nrm = np.sqrt(dx * dx + dy * dy)
        want = (0.0, 0.0) if dx == 0 and dy == 0 else (dx / nrm, dy / nrm)
        assert p.gradientNode(i, j) == pytest.approx(want, abs=0, rel=1e-15)


def test_local_agent_and_dijkstra_step(dymu, oracle):
    """local_agent after a local propagation; computeLocalWaypointDijkstra
    (L:851-869) steps to an nb4 sub-cell (one local cell away)."""
    N = 24
    p, o = build(dymu, oracle, N, 0.25, 0, goal=(12, 12))
    assert p.localAgent() is None
    assert p.computeLocalPropagation((5.0, 5.0), (9.0, 9.0)) is not None
    ax, ay = p.localAgent()
    assert abs(ax - 5.0) <= 0.25 and abs(ay - 5.0) <= 0.25
    w = p.computeLocalWaypointDijkstra((5.5, 5.5))
    assert w is not None
    # an axis step of one local cell from the sub-cell holding (5.5, 5.5),
    # heading along it (the sub-cell's centre is within half a cell of 5.5)
    c = (w[0] - 0.25 * np.cos(w[3]), w[1] - 0.25 * np.sin(w[3]))
    assert min(abs(np.cos(w[3])), abs(np.sin(w[3]))) < 1e-12
    assert abs(c[0] - 5.5) <= 0.125 + 1e-12 and abs(c[1] - 5.5) <= 0.125 + 1e-12


def test_local_propagation_wall_clock_limit(dymu, oracle):
    """src/DyMu_LocalPathRepairing.cpp:685-696: past the time limit the local
    propagation gives up and returns NULL; without one it finds the set node."""
    N = 24
    p, o = build(dymu, oracle, N, 0.25, 0, goal=(12, 12))
    ref = p.computeLocalPropagation((5.0, 5.0), (9.0, 9.0))
    assert ref is not None
    p.setLocalPropagationTimeout(1e-9)  # checked every 256 settled sub-cells
    assert p.computeLocalPropagation((5.0, 5.0), (9.0, 9.0)) is None
    p.setLocalPropagationTimeout(0)  # disabled
    assert p.computeLocalPropagation((5.0, 5.0), (9.0, 9.0)) == ref
    p.setLocalPropagationTimeout(5.0)


@pytest.mark.parametrize("name,approach", [("cons", 0), ("sweep", 1)])
def test_local_golden_terrain(dymu, oracle, name, approach):
    """The committed local-layer fixtures (tests/golden/gen_golden_local.py):
    the oracle reproduces them, and so does the planner fed the same terrain
    through computeCostMap (waypoint z from the elevation)."""
    import gen_golden_local as G
    from gen_golden import terrain_inputs

    gold = {k: np.load(os.path.join(GOLD, f"local_{name}_{k}.npy"), allow_pickle=False)
            for k in ("path", "traj", "hazard", "traff", "risk", "dev", "rep")}
    res, (rover, img) = G.run_oracle(oracle, approach)
    for k, v in gold.items():
        assert same(res[k], v), k
    elev, terr, lut, slopes = terrain_inputs(G.N)
    _, _, T = G.scenario(oracle)
    p = dymu.Planner(approach=approach, **G.PARAMS)
    assert p.initGlobalLayer(1.0, G.LRES, G.N, G.N)
    assert p.computeCostMap(lut, slopes, ["Wheel"], elev, terr)
    assert p.setGoal((G.GOAL[0], G.GOAL[1], 0.0, 0.3))
    assert p.loadTotalCostMap(T)
    assert same(p.getPath(G.START), gold["path"])
    rep, traj, _ = p.computeLocalPlanning(rover, img, G.LRES)
    assert [int(rep), p.getReconnectingIndex()] == gold["rep"].tolist()
    assert same(traj, gold["traj"])
    assert np.abs(traj[:, 2]).max() > 0  # z interpolated from the elevation
    assert same(p.getHazardDensityMatrix(), gold["hazard"])
    assert same(p.getTrafficabilityMatrix(), gold["traff"])
    assert same(p.getRiskMatrix(rover), gold["risk"])
    assert same(p.getDeviationMatrix(rover), gold["dev"])


@pytest.mark.parametrize("approach", [0, 1])
def test_blocking_on_self_crossing_path(dymu, oracle, approach):
    """isBlockingObstacle (:441-471) takes the FIRST waypoint within
    risk_distance and the run of blocked waypoints after it: a current_path
    that loops back past the obstacle twice (the product finds that waypoint
    through a spatial index of the path, the oracle by the reference's scan)."""
    N = 48
    p, o = build(dymu, oracle, N, 0.25, approach, goal=(40, 40))
    t = np.linspace(0, 4 * np.pi, 160)
    loop = np.stack([20 + 8 * np.cos(t + np.pi) + 0.05 * t, 20 + 8 * np.sin(t + np.pi) + 0.05 * t,
                     np.zeros_like(t), np.zeros_like(t)], axis=1)
    path = np.concatenate([loop, np.stack([np.linspace(loop[-1, 0], 39, 60),
                                           np.linspace(loop[-1, 1], 39, 60),
                                           np.zeros(60), np.zeros(60)], axis=1)])
    p.current_path = path
    o.path = path
    rover = tuple(path[0, :2])
    centre = (28.3, 20.6)  # on the loop, passed twice
    img = disc_image(rover, centre, 0.9, 0.25, 160)
    rep, traj, _ = p.computeLocalPlanning(rover, img, 0.25)
    rep_o, traj_o = o.local_planning(rover, img, 0.25)
    assert rep and rep == rep_o
    assert len(traj) > 20
    assert same(traj, traj_o)
    compare_state(p, o, rover)
