"""global_propagated_nodes (src/DyMu.hpp:447, :537-545) after a GPU solve: the time of
Planner.globalPropagatedNodes() -- the flat ABI's dymu_planner_global_propagated_nodes,
the list rebuilt in the reference's insertion order from the values (planner.cpp
insertionOrder) -- after computeEntireTotalCostMap and after a mid-distance
computeTotalCostMap, on the config-3 map (U(1,5) costs, 2% obstacles, goal centre).
usage: python tools/propagated_bench.py N [N ...]   (DYMU_LIBDIR: another build)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "planning-path_planning_amd"))
import dymu  # noqa: E402


def main():
    for N in [int(x) for x in sys.argv[1:]] or [4096]:
        rng = np.random.default_rng(5)
        c = rng.uniform(1.0, 5.0, size=(N, N))
        c[rng.random((N, N)) < 0.02] = -1.0
        g = (N // 2, N // 2)
        c[g[1] - 2:g[1] + 3, g[0] - 2:g[0] + 3] = 1.5
        s = (int(0.7 * N), int(0.6 * N))
        c[s[1] - 2:s[1] + 3, s[0] - 2:s[0] + 3] = 1.5
        p = dymu.Planner()
        p.initGlobalLayer(1.0, 0.5, N, N)
        p.setCostMap(c)
        assert p.setGoal(g)
        row = {"N": N, "lib": os.environ.get("DYMU_LIBDIR", "tree")}
        for kind in ("entire", "early"):
            t0 = time.perf_counter()
            assert p.computeEntireTotalCostMap() if kind == "entire" else p.computeTotalCostMap(s)
            row[kind + "_solve_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
            t0 = time.perf_counter()
            nodes = p.globalPropagatedNodes()
            row[kind + "_nodes_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
            row[kind + "_nodes"] = int(len(nodes))
            row[kind + "_head"] = nodes[:3].tolist()
            del nodes
        print(json.dumps(row), flush=True)
        p.close()


if __name__ == "__main__":
    main()
