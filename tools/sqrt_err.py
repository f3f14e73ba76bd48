"""Max relative error of the device solve vs the oracle FMM at a few sizes
(development tool for numerics A/B; the oracle is the checker only)."""
import os, sys, json
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "planning-path_planning_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import dymu
import oracle_ffi

orc = oracle_ffi.load()
for N in [int(a) for a in sys.argv[1:]]:
    g = (N // 2, N // 2)
    F = orc.synth_speed(N, N, seed=1, obst_frac=0.02, obst_seed=3, goal=g)
    eng = dymu.Engine(kernel=5)
    r = eng.solve(F, g[0], g[1])
    Tref, _ = orc.fmm(F, g)
    fin = np.isfinite(Tref)
    same_mask = bool(np.array_equal(np.isfinite(r.T), fin))
    err = np.abs(r.T[fin] - Tref[fin]) / np.maximum(1.0, Tref[fin])
    print(json.dumps({"N": N, "same_inf_mask": same_mask, "max_rel_err": float(err.max()),
                      "mean_rel_err": float(err.mean())}), flush=True)
    eng.close()
