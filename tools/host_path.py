"""PCIe-inclusive rate of the host-buffer path (dymu_solve: H2D of F, solve, D2H of T)
at the bench workload, beside the device-resident rate (dymu_solve_device).
Usage: python tools/host_path.py [N]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "planning-path_planning_amd"))
import dymu  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
g = (N // 2, N // 2)
eng = dymu.Engine()
dF, dT = eng.alloc(8 * N * N), eng.alloc(8 * N * N)
eng.synth_speed(dF, N, N, N, 0, 1, 0.02, 3, g[0], g[1])
F = np.empty((N, N))
eng.d2h(F, dF)
eng.solve_device(dF, dT, N, N, N, g[0], g[1])  # warm-up
t = time.perf_counter()
for _ in range(3):
    eng.solve_device(dF, dT, N, N, N, g[0], g[1])
dev = (time.perf_counter() - t) / 3
eng.free(dF)
eng.free(dT)
eng.solve(F, *g)  # warm-up (allocates the staging buffers)
t = time.perf_counter()
for _ in range(3):
    r = eng.solve(F, *g)
host = (time.perf_counter() - t) / 3
eng.close()
print(json.dumps({"grid": N, "device_resident_ms": dev * 1e3,
                  "device_resident_Mcells_s": N * N / dev / 1e6,
                  "host_buffers_ms": host * 1e3, "host_buffers_Mcells_s": N * N / host / 1e6,
                  "pcie_bytes": 16 * N * N, "note": "host path: pageable numpy F in, T out"}))
