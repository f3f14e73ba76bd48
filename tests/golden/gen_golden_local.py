"""Generates the local-layer golden fixtures (tests/golden/local_*.npy).

Scenario: a 48x48 config-2 style terrain (elevation, so waypoint z is
exercised) through computeCostMap, goal (36, 32), the oracle's heap FMM for
the total cost, getPath from (7.3, 9.1), then computeLocalPlanning with a
0.8 m obstacle disc on the path 10 waypoints ahead (0.25 m local cells,
36x36 image), for CONSERVATIVE and SWEEPING.  Expected outputs come from the
local-layer restatement oracle/oracle_local.c (the reference has no tests and
ships no fixtures; parity of the local layer is unpinned beyond this
restatement).  Run from the repo root:
    python tests/golden/gen_golden_local.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import oracle_ffi  # noqa: E402
from gen_golden import terrain_inputs  # noqa: E402

N = 48
GOAL = (36, 32)
START = (7.3, 9.1, 0.0, 0.0)
LRES = 0.25
PARAMS = dict(risk_distance=1.0, reconnect_distance=1.5, risk_ratio=5.0)


def disc_image(rover, centre, radius, res, size):
    """size x size image at res m/pixel centred on rover (row j at
    y = rover_y + res*size/2 - j*res, reference :225-238), disc of value 1."""
    img = np.zeros((size, size), dtype=np.uint8)
    ox = rover[0] - res * size / 2
    oy = rover[1] + res * size / 2
    j, i = np.mgrid[0:size, 0:size]
    img[(ox + i * res - centre[0]) ** 2 + (oy - j * res - centre[1]) ** 2 <= radius ** 2] = 1
    return img


def scenario(o):
    """(state dict, total cost T) of the terrain global layer."""
    elev, terr, lut, slopes = terrain_inputs(N)
    st = o.new_state(N, N)
    o.compute_cost_map(st, 1.0, lut, slopes, 1, elev, terr)
    F = o.pack_speed(st["cost"], st["hazard"], st["traff"], st["is_obstacle"], res=1.0)
    T, _ = o.fmm(F, GOAL)
    return elev, st, T


def run_oracle(o, approach):
    elev, st, T = scenario(o)
    L = o.local(N, N, 1.0, LRES, approach=approach, **PARAMS)
    L.set_global(st["is_obstacle"], T, GOAL, goal_heading=0.3, elev=elev, hazard=st["hazard"],
                 traff=st["traff"])
    _, path = L.get_path(START)
    rover = tuple(path[2][:2])
    centre = tuple(path[10][:2])
    img = disc_image(rover, centre, 0.8, LRES, 36)
    rep, traj = L.local_planning(rover, img, LRES)
    hd, tr = L.hazard_traff()
    return {"path": path, "traj": traj, "hazard": hd, "traff": tr,
            "risk": L.risk_matrix(*rover), "dev": L.deviation_matrix(*rover),
            "rep": np.array([int(rep), L.reconnecting_index()], dtype=np.int64)}, (rover, img)


def main():
    o = oracle_ffi.load()
    for name, approach in (("cons", 0), ("sweep", 1)):
        res, _ = run_oracle(o, approach)
        for k, v in res.items():
            np.save(os.path.join(HERE, f"local_{name}_{k}.npy"), v, allow_pickle=False)
        print(name, {k: v.shape for k, v in res.items()}, "repaired", res["rep"].tolist())


if __name__ == "__main__":
    main()
