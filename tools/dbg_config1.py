import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "planning-path_planning_amd"), os.path.join(ROOT, "tests")]
import dymu, oracle_ffi
o = oracle_ffi.load()
N, g, s = 512, (256, 256), (102, 128)
F = o.synth_speed(N, N, seed=1, obst_frac=0.0, obst_seed=3, goal=g)
p = dymu.Planner()
p.initGlobalLayer(1.0, 0.5, N, N)
p.setCostMap(F)
p.setGoal(g)
Tt, rc, closed, seq = o.fmm_order(F, g, start=s)
r = p.computeTotalCostMap(s)
print("rc", r, rc, p.lastEarlyExit(), "band", p.lastBandSize(), int(((closed == 0) & np.isfinite(Tt)).sum()))
M = p.getTotalCostMatrix()
bad = np.argwhere((M == -1.0) != np.isinf(Tt))
print("mask mismatches", len(bad), bad[:10], [ (M[j,i], Tt[j,i]) for j,i in bad[:10]])
fin = np.isfinite(Tt) & (M >= 0)
print("max rel", (np.abs(M[fin]-Tt[fin])/np.maximum(1,Tt[fin])).max())
