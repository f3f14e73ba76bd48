"""Config 5 through the class surface (development tool): config-2 terrain at N^2,
GPU solve, getPath, computeLocalPlanning with an obstacle disc 30% along the path
(the local layer on the host), then computeEntireTotalCostMap (the windowed GPU
re-propagation of the local layer's hazard / trafficability feedback) -- each
step timed.  Prints one JSON line per (N, approach, local resolution)."""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "planning-path_planning_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import numpy as np  # noqa: E402

import dymu  # noqa: E402
from gen_golden import config2_inputs  # noqa: E402
from test_local_layer import disc_image  # noqa: E402


def run(N, approach, lres, radius=20.0):
    elev, terr, lut, slopes = config2_inputs(N)
    goal = (3 * N // 4, 3 * N // 4)
    p = dymu.Planner(risk_distance=2.0, reconnect_distance=3.0, risk_ratio=5.0,
                     approach=approach)
    p.initGlobalLayer(1.0, lres, N, N)
    t = time.perf_counter()
    p.computeCostMap(lut, slopes, ["Wheel"], elev, terr)
    t_cost = time.perf_counter() - t
    p.setGoal(goal)
    p.computeEntireTotalCostMap()  # cold (first solve also sets up the engine)
    t = time.perf_counter()
    p.computeEntireTotalCostMap()
    t_reuse = time.perf_counter() - t
    p.setGoal((goal[0] - 1, goal[1]))
    t = time.perf_counter()
    p.computeEntireTotalCostMap()
    t_cold = time.perf_counter() - t
    cold = p.lastStats()
    start = (N * 0.15 + 0.3, N * 0.17 + 0.6)
    t = time.perf_counter()
    path = p.getPath(start)
    t_path = time.perf_counter() - t
    k = int(0.3 * len(path))
    rover = tuple(path[max(0, k - int(1.5 * radius / 0.4))][:2])
    centre = tuple(path[k][:2])
    size = int(4 * radius / lres)
    img = disc_image(rover, centre, radius, lres, size)
    t = time.perf_counter()
    rep, traj, t_local = p.computeLocalPlanning(rover, img, lres)
    t_lp = time.perf_counter() - t
    sub = int(p.localMapMask().sum())
    t = time.perf_counter()
    p.computeEntireTotalCostMap()
    t_win = time.perf_counter() - t
    win = p.lastStats()
    kind = p.lastSolveKind()
    t = time.perf_counter()
    path2 = p.getPath(start)
    t_path2 = time.perf_counter() - t
    print(json.dumps({
        "N": N, "approach": ["conservative", "sweeping"][approach], "local_res": lres,
        "image_px": size, "repaired": bool(rep), "trajectory": len(traj),
        "subdivided_global_nodes": sub, "sub_cells": sub * int(round(1 / lres)) ** 2,
        "ms": {"computeCostMap_host": 1e3 * t_cost, "cold_solve": 1e3 * t_cold,
               "reuse": 1e3 * t_reuse, "getPath": 1e3 * t_path,
               "computeLocalPlanning": 1e3 * t_lp, "repair_only": 1e3 * t_local,
               "windowed_resolve": 1e3 * t_win, "getPath_after": 1e3 * t_path2},
        "cold_passes": cold["passes"], "cold_visits": cold["tile_visits"],
        "window_passes": win["passes"], "window_visits": win["tile_visits"],
        "window_kind": kind, "path_len": len(path), "path_len_after": len(path2)}), flush=True)


if __name__ == "__main__":
    sizes = [int(a) for a in sys.argv[1:]] or [4096]
    for N in sizes:
        for approach in (0, 1):
            for lres in (0.5, 0.25):
                run(N, approach, lres)
