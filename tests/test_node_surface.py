"""The reference class's per-node surface at the product's class surface (VERDICT r3
"do this" 5): the public node lists (src/DyMu.hpp:445-454) and the per-node steps of
the loops the library otherwise runs whole -- propagateGlobalNode (:500-546),
maxRiskNode / propagateRisk (L:525-576), propagateLocalNode (L:700-750),
minCostLocalNode x2 (L:752-805) -- through the flat C-ABI (include/dymu_planner.h),
against the oracle restatements (oracle/oracle.c, oracle/oracle_local.c).

Host-only: the global map comes from the oracle (or from the per-node loop itself),
so these run on CPU.  setHorizonCost (src/DyMu.hpp:555) is declared but defined
nowhere in the reference; it has no counterpart to test."""
import os

import numpy as np
import pytest

from test_local_layer import build, disc_image, same

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NB4 = ((0, -1), (-1, 0), (1, 0), (0, 1))  # nb4List order (GlobalPathPlanning.cpp:76-80)


def drive_global_fmm(p, nx, ny):
    """computeEntireTotalCostMap (:443-468) written as a caller of the per-node
    surface: reset, then pop / close / propagate until the band is empty."""
    p.resetTotalCostMap()
    p.resetGlobalNarrowBand()
    pops = []
    while True:
        n = p.minCostGlobalNode()
        if n is None:
            break
        (i, j), _ = n
        pops.append((i, j))
        p.setGlobalNodeState(i, j, True)
        for di, dj in NB4:
            a, b = i + di, j + dj
            if 0 <= a < nx and 0 <= b < ny:
                q = p.getGlobalNode(a, b)
                if q["state"] == 0 and not q["is_obstacle"]:
                    p.propagateGlobalNode(a, b)
    return pops


def test_global_fmm_driven_node_by_node_is_the_reference(dymu, oracle):
    """The reference's own FMM loop, run through minCostGlobalNode /
    setGlobalNodeState / propagateGlobalNode on the 64^2 setCostMap golden, is the
    reference FMM bit for bit (the band keeps insertion order, so the pops are the
    reference's); global_propagated_nodes holds every reached node, goal first."""
    cost = np.load(os.path.join(GOLD, "setcost64_cost.npy"))
    goal = tuple(int(v) for v in np.load(os.path.join(GOLD, "setcost64_goal.npy")))
    Tgold = np.load(os.path.join(GOLD, "setcost64_T.npy"))
    ny, nx = cost.shape
    p = dymu.Planner()
    try:
        assert p.initGlobalLayer(1.0, 1.0, nx, ny)
        assert p.setCostMap(cost)
        assert p.setGoal((goal[0], goal[1], 0.0, 0.0))
        pops = drive_global_fmm(p, nx, ny)
        T = p.totalCostRaw()
        assert np.array_equal(T.view(np.uint64), Tgold.view(np.uint64))
        fin = np.isfinite(Tgold)
        assert len(pops) == int(fin.sum())
        assert all(p.getGlobalNode(i, j)["state"] == 1 for i, j in pops[:50])
        prop = p.globalPropagatedNodes()
        assert tuple(prop[0]) == goal and len(prop) == int(fin.sum())
        assert set(map(tuple, prop.tolist())) == {(int(i), int(j)) for j, i in np.argwhere(fin)}
        assert len(p.globalNarrowband()) == 0
    finally:
        p.close()


def test_propagate_global_node_single_update(dymu, oracle):
    """One propagateGlobalNode is the reference update (:500-546) of the node's
    current neighbours -- one-sided, two-sided, and at the border (a NULL neighbour:
    the other one alone) -- and joins the band / propagated list only when it was
    +inf (in insertion order, after the goal resetGlobalNarrowBand put there)."""
    N = 12
    cost = np.full((N, N), 2.0)
    cost[5, 4] = 2.5
    p = dymu.Planner()
    try:
        assert p.initGlobalLayer(1.0, 1.0, N, N)
        assert p.setCostMap(cost)
        assert p.setGoal((5, 6, 0.0, 0.0))
        p.resetTotalCostMap()
        p.resetGlobalNarrowBand()
        p.propagateGlobalNode(5, 5)  # below the goal: Ty = 0, Tx = +inf -> one-sided
        p.propagateGlobalNode(6, 5)  # Tx = T(5,5), Ty = +inf -> one-sided
        p.propagateGlobalNode(6, 6)  # Tx = T(5,6) = 0, Ty = T(6,5) -> two-sided
        T = p.totalCostRaw()
        assert T[5, 5] == 0.0 + cost[5, 5]
        assert T[5, 6] == T[5, 5] + cost[5, 6]
        assert T[6, 6] == oracle.eikonal(0.0, T[5, 6], cost[6, 6])
        p.propagateGlobalNode(4, 6)  # Tx = T(5,6) = 0 -> one-sided
        p.propagateGlobalNode(4, 5)  # Tx = T(5,5), Ty = T(4,6): both finite
        T = p.totalCostRaw()
        assert abs(T[5, 5] - T[6, 4]) < cost[5, 4]  # the two-sided branch (:531-533)
        assert T[5, 4] == oracle.eikonal(T[5, 5], T[6, 4], cost[5, 4])
        assert p.globalNarrowband().tolist() == [[5, 6], [5, 5], [6, 5], [6, 6], [4, 6], [4, 5]]
        before = p.getGlobalNode(5, 5)["total_cost"]
        p.propagateGlobalNode(5, 5)  # no lower value: unchanged, not queued again
        assert p.getGlobalNode(5, 5)["total_cost"] == before
        assert len(p.globalNarrowband()) == 6 and len(p.globalPropagatedNodes()) == 6
        assert p.getGlobalNode(5, 5)["state"] == 0  # OPEN until a caller closes it
        # the border: (5, 0) has no S neighbour (nb4List[0] NULL), so Ty = T(5, 1) alone
        for j in range(4, 0, -1):
            p.propagateGlobalNode(5, j)
        p.propagateGlobalNode(5, 0)
        T = p.totalCostRaw()
        assert np.isfinite(T[1, 5]) and T[0, 5] == T[1, 5] + cost[0, 5]
    finally:
        p.close()


def _node5(n):
    return np.array([n["global_x"], n["global_y"], n["deviation"], n["total_cost"], n["risk"]])


def _list5(nodes):
    return np.array([_node5(n) for n in nodes]).reshape(-1, 5)


def test_local_lists_and_risk_steps_match_oracle(dymu, oracle):
    """Obstacles off the path: computeLocalPlanning marks them and queues them in
    local_expandable_obstacles but does not repair (:278-290), so the queue is left
    full -- identical to the oracle's.  Then expandRisk is driven node by node on
    both (maxRiskNode, then propagateRisk on every non-obstacle nb4) and every pop
    and the final risk field agree bit for bit."""
    N = 40
    p, o = build(dymu, oracle, N, 0.25, 1, goal=(30, 30))
    try:
        start = (6.0, 6.0)
        path = p.getPath(start)
        o.get_path(start)
        rover = tuple(path[1][:2])
        img = disc_image(rover, (rover[0] + 3.0, rover[1] - 3.0), 0.5, 0.25, 32)
        assert not p.computeLocalPlanning(rover, img, 0.25)[0]
        assert not o.local_planning(rover, img, 0.25)[0]
        q = p.localExpandableObstacles()
        assert len(q) > 10 and same(_list5(q), o.node_list(1))
        assert all(n["risk"] == 1.0 and n["is_obstacle"] for n in q)
        pops = 0
        while True:
            n = p.maxRiskNode()
            n_o = o.max_risk_node()
            if n is None:
                assert n_o is None
                break
            assert same(_node5(n), n_o)
            pops += 1
            for d in range(4):
                nb = p.localNeighbour(n, d)
                if nb is not None and not nb["is_obstacle"]:
                    p.propagateRisk(nb)
                    assert o.propagate_risk(nb["global_x"], nb["global_y"])
            if pops % 64 == 0:
                assert same(_list5(p.localExpandableObstacles()), o.node_list(1))
        assert pops > len(q)  # risk spread beyond the obstacle cells
        for j, i in np.argwhere(p.localMapMask()):
            assert same(p.localBlock(int(i), int(j))[2], o.block(int(i), int(j))[2])
        assert same(p.getRiskMatrix(rover), o.risk_matrix(rover[0], rover[1]))
    finally:
        p.close()


@pytest.mark.parametrize("approach", [0, 1], ids=["conservative", "sweeping"])
def test_local_band_and_propagation_steps_match_oracle(dymu, oracle, approach):
    """After a repair, local_narrowband and local_propagated_nodes are the oracle's
    (order and values).  Then the local FMM continues node by node on both:
    minCostLocalNode (deviation key, or deviation + distance to a reach node),
    close it, propagateLocalNode on its open non-obstacle nb4 -- every pop agrees."""
    N = 48
    p, o = build(dymu, oracle, N, 0.25, approach)
    try:
        start = (8.3, 9.6, 0.0, 0.0)
        path = p.getPath(start)
        o.get_path(start)
        rover = tuple(path[2][:2])
        centre = tuple(path[min(12, len(path) - 2)][:2])
        img = disc_image(rover, centre, 0.8, 0.25, 36)
        assert p.computeLocalPlanning(rover + (0.0, 0.0), img, 0.25)[0]
        assert o.local_planning(rover + (0.0, 0.0), img, 0.25)[0]
        band, prop = p.localNarrowband(), p.localPropagatedNodes()
        assert len(band) > 0 and len(prop) > len(band)
        assert same(_list5(band), o.node_list(0))
        assert same(_list5(prop), o.node_list(2))
        reach = prop[len(prop) // 2] if approach == 0 else None
        for _ in range(200):
            if reach is not None:
                n = p.minCostLocalNode(reach=reach)
                n_o = o.min_cost(reach=(reach["global_x"], reach["global_y"]))
            else:
                n = p.minCostLocalNode(0.0, 1.0)
                n_o = o.min_cost()
            if n is None:
                assert n_o is None
                break
            assert same(_node5(n), n_o)
            p.setLocalNodeState(n, True)
            assert o.set_state(n["global_x"], n["global_y"], True)
            for d in range(4):
                nb = p.localNeighbour(n, d)
                if nb is not None and nb["state"] == 0 and not nb["is_obstacle"]:
                    p.propagateLocalNode(nb)
                    assert o.propagate_local(nb["global_x"], nb["global_y"])
        assert same(_list5(p.localNarrowband()), o.node_list(0))
        assert same(_list5(p.localPropagatedNodes()), o.node_list(2))
    finally:
        p.close()


def test_node_surface_empty_cases(dymu):
    """The reference's NULL cases: empty queues and bands, no local map."""
    p = dymu.Planner()
    try:
        assert p.initGlobalLayer(1.0, 0.5, 8, 8)
        assert p.maxRiskNode() is None
        assert p.minCostLocalNode(0.0, 1.0) is None
        assert p.localNarrowband() == [] and p.localExpandableObstacles() == []
        assert p.localPropagatedNodes() == []
        n = p.getLocalNode(3.2, 3.4)
        assert n is not None and p.localNeighbour(n, 0) is not None  # inside its block
        assert p.localNeighbour({"id": 10 ** 9}, 0) is None  # no such sub-cell
    finally:
        p.close()
