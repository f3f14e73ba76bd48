import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "planning-path_planning_amd"), os.path.join(ROOT, "tests")]
os.environ["DYMU_ORDER_DEBUG"] = "1"
import dymu, oracle_ffi
o = oracle_ffi.load()
for N, g, s in [(160, (80, 80), (20, 140)), (96, (48, 48), (48, 20))]:
    F = np.ones((N, N))
    p = dymu.Planner()
    p.initGlobalLayer(1.0, 0.5, N, N)
    p.setCostMap(F)
    p.setGoal(g)
    Tt, rc, closed, seq = o.fmm_order(F, g, start=s)
    r = p.computeTotalCostMap(s)
    print(N, "rc", r, rc, p.lastEarlyExit(), flush=True)
    p.computeEntireTotalCostMap()
    M = p.getTotalCostMatrix()
    Tf, _ = o.fmm(F, g)
    d = M - Tf
    print("full map: max abs diff", np.abs(d).max(), "asym x", np.abs(M - M[:, ::-1][:, list(range(N - 2 * g[0] + 0, N)) + list(range(0, N - 2*g[0]))] ).max() if False else "")
    # symmetry about the goal
    h = min(g[0], N - 1 - g[0])
    sub = M[g[1]-h:g[1]+h+1, g[0]-h:g[0]+h+1]
    print("sym lr", np.abs(sub - sub[:, ::-1]).max(), "sym ud", np.abs(sub - sub[::-1, :]).max(), "sym diag", np.abs(sub - sub.T).max())
    p.close()
