"""The local layer on a GPU-produced total-cost map, and its feedback into the
next GPU solve (config 5 through the reference's own write path:
computeLocalPlanning's hazard bumps, src/DyMu_LocalPathRepairing.cpp:264-274,
and repairPath's trafficability drops, :389-394).

* the engine's map is checked against the oracle FMM (1e-12);
* the local layer on that map is compared bit for bit with the oracle's local
  restatement fed the same map;
* the next computeEntireTotalCostMap re-propagates only the changed window
  (lastSolveKind 1) and equals the oracle FMM of the new speed.
"""
import numpy as np
import pytest

from test_local_layer import compare_state, disc_image, same

RTOL = 1e-12


def close_T(T, Tref):
    assert np.array_equal(np.isinf(T), np.isinf(Tref))
    fin = np.isfinite(Tref)
    return (np.abs(T[fin] - Tref[fin]) / np.maximum(1, Tref[fin])).max() <= RTOL


def planner_on_gpu(dymu, oracle, N, goal, lres, approach, seed=31, obst_frac=0.02):
    F = oracle.synth_speed(N, N, seed=seed, obst_frac=obst_frac, obst_seed=seed + 1, goal=goal)
    cost = np.where(np.isfinite(F), F, -1.0)
    p = dymu.Planner(risk_distance=1.0, reconnect_distance=1.5, risk_ratio=5.0,
                     approach=approach)
    assert p.initGlobalLayer(1.0, lres, N, N)
    assert p.setCostMap(cost)
    assert p.setGoal((goal[0], goal[1], 0.0, 0.2))
    assert p.computeEntireTotalCostMap()
    Tref, _ = oracle.fmm(F, goal)
    T = p.totalCostRaw()
    assert close_T(T, Tref)
    o = oracle.local(N, N, 1.0, lres, risk_distance=1.0, reconnect_distance=1.5,
                     risk_ratio=5.0, approach=approach)
    o.set_global((cost <= 0).astype(np.uint8), T, goal, goal_heading=0.2,
                 hazard=p.getHazardDensityMatrix(), traff=p.getTrafficabilityMatrix())
    return p, o, cost


@pytest.mark.gpu
@pytest.mark.parametrize("approach", [0, 1], ids=["conservative", "sweeping"])
def test_local_repair_on_gpu_map(dymu, oracle, approach):
    N = 128
    goal = (100, 90)
    p, o, cost = planner_on_gpu(dymu, oracle, N, goal, 0.25, approach)
    start = (14.2, 20.7)
    path = p.getPath(start)
    _, path_o = o.get_path(start)
    assert len(path) > 50 and same(path, path_o)
    rover = tuple(path[3][:2])
    centre = tuple(path[15][:2])
    img = disc_image(rover, centre, 1.2, 0.25, 48)
    rep, traj, _ = p.computeLocalPlanning(rover, img, 0.25)
    rep_o, traj_o = o.local_planning(rover, img, 0.25)
    assert rep and rep_o
    assert same(traj, traj_o)
    compare_state(p, o, rover)
    # the feedback re-propagates from the changed window on the GPU
    assert p.computeEntireTotalCostMap()
    assert p.lastSolveKind() == 1
    obst = cost <= 0
    Fr = oracle.pack_speed(cost, p.getHazardDensityMatrix(), p.getTrafficabilityMatrix(),
                           obst, res=1.0)
    Tref2, _ = oracle.fmm(Fr, goal)
    assert close_T(p.totalCostRaw(), Tref2)
    # and the next path through evaluatePath keeps matching the oracle on the new map
    o.set_global(None, p.totalCostRaw(), goal, goal_heading=0.2)
    path2 = p.getPath(start)
    _, path2_o = o.get_path(start)
    assert same(path2, path2_o)


@pytest.mark.gpu
def test_config5_local_planning_4096(dymu, oracle):
    """BASELINE config 5 at size: 4096^2 config-2 terrain through
    computeCostMap, GPU solve, a 20-cell obstacle disc 30% along the path
    inserted by computeLocalPlanning (0.5 m local cells), the windowed GPU
    re-propagation of its hazard feedback vs the oracle FMM of the new speed."""
    from gen_golden import config2_inputs

    N = 4096
    elev, terr, lut, slopes = config2_inputs(N)
    goal = (3 * N // 4, 3 * N // 4)
    p = dymu.Planner(risk_distance=2.0, reconnect_distance=3.0, risk_ratio=5.0, approach=0)
    assert p.initGlobalLayer(1.0, 0.5, N, N)
    assert p.computeCostMap(lut, slopes, ["Wheel"], elev, terr)
    assert p.setGoal(goal)
    assert p.computeEntireTotalCostMap()
    cold_visits = p.lastStats()["tile_visits"]
    path = p.getPath((600.3, 700.6))
    assert len(path) > 100
    k = int(0.3 * len(path))
    rover = tuple(path[max(0, k - 75)][:2])  # ~30 m before the disc (0.4 m steps)
    centre = tuple(path[k][:2])
    img = disc_image(rover, centre, 20.0, 0.5, 160)
    rep, traj, t_local = p.computeLocalPlanning(rover, img, 0.5)
    assert rep and len(traj) > 10
    assert p.getHazardDensityMatrix().max() > 0.5
    assert p.computeEntireTotalCostMap()
    assert p.lastSolveKind() == 1
    assert p.lastStats()["tile_visits"] < cold_visits
    st = oracle.new_state(N, N)
    oracle.compute_cost_map(st, 1.0, lut, slopes, 1, elev, terr)
    Fr = oracle.pack_speed(st["cost"], p.getHazardDensityMatrix(), p.getTrafficabilityMatrix(),
                           st["is_obstacle"], res=1.0)
    Tref, _ = oracle.fmm(Fr, goal)
    assert close_T(p.totalCostRaw(), Tref)
