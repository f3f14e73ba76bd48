"""Minimal solve loop for the PMC passes (tools/pmc_round.sh): N^2 config-3 grid, reps solves."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "planning-path_planning_amd"))
import dymu
N = int(sys.argv[1]); reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
eng = dymu.Engine(); n = N * N
dF, dT = eng.alloc(8 * n), eng.alloc(8 * n)
eng.synth_speed(dF, N, N, N, 0, 1, 0.02, 3, N // 2, N // 2)
for r in range(reps):
    st = eng.solve_device(dF, dT, N, N, N, N // 2, N // 2)
    print(st, flush=True)
