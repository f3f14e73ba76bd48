"""Probe: where the class-surface readback of a 16384^2 map goes (solve, D2H into the
page-locked mirror, host copy into a fresh / a reused numpy buffer)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "planning-path_planning_amd"))
import numpy as np
import torch  # noqa: F401
import dymu

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
g = (N // 2, N // 2)
eng = dymu.Engine(device=0)
dF = eng.alloc(8 * N * N)
eng.synth_speed(dF, N, N, N, 0, 1, 0.02, 3, g[0], g[1])
F = np.empty((N, N))
t0 = time.perf_counter(); eng.d2h(F, dF); t_pageable = time.perf_counter() - t0
t0 = time.perf_counter(); eng.d2h(F, dF); t_pageable2 = time.perf_counter() - t0
eng.free(dF); eng.close()
p = dymu.Planner(device=0)
p.initGlobalLayer(1.0, 0.5, N, N)
p.setCostMap(np.where(np.isfinite(F), F, -1.0))
del F
p.setGoal(g)
p.computeEntireTotalCostMap()
for k in range(2):
    p.setGoal((g[0] + 1 - k, g[1]))
    t0 = time.perf_counter(); p.computeEntireTotalCostMap(); ts = time.perf_counter() - t0
    t0 = time.perf_counter(); T = p.totalCostRaw(); t1 = time.perf_counter() - t0
    t0 = time.perf_counter(); T2 = p.totalCostRaw(); t2 = time.perf_counter() - t0
    out = np.empty((N, N)); out.fill(0.0)
    lib = p._lib
    import ctypes
    t0 = time.perf_counter(); lib.dymu_planner_get_total_cost_raw(p.h, out); t3 = time.perf_counter() - t0
    print(f"solve {ts*1e3:.1f} ms | raw readback stale mirror, fresh buffer {t1*1e3:.1f} ms | "
          f"fresh mirror, fresh buffer {t2*1e3:.1f} ms | fresh mirror, touched buffer {t3*1e3:.1f} ms",
          flush=True)
    del T, T2, out
print(f"engine d2h 2 GiB into pageable numpy: {t_pageable*1e3:.1f} / {t_pageable2*1e3:.1f} ms "
      f"(first / touched), host threads {os.environ.get('OMP_NUM_THREADS')} nproc {os.cpu_count()}")
