"""Quick timing probe of the device-resident solve (development tool)."""
import os, sys, time, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "planning-path_planning_amd"))
import numpy as np
import dymu

def run(N, frac=0.02, reps=3, prof=False):
    eng = dymu.Engine()
    n = N * N
    dF, dT = eng.alloc(8 * n), eng.alloc(8 * n)
    g = (N // 2, N // 2)
    eng.synth_speed(dF, N, N, N, 0, 1, frac, 3, g[0], g[1])
    out = []
    for r in range(reps):
        eng.set_profiling(prof and r == reps - 1)
        t = time.perf_counter()
        st = eng.solve_device(dF, dT, N, N, N, g[0], g[1])
        dt = time.perf_counter() - t
        pm, pl = eng.last_pass_timing()
        st.update(wall_s=dt, mcells=n / dt / 1e6, pass_ms=pm, pass_launches=pl)
        out.append(st)
    T = np.empty((N, N)); eng.d2h(T, dT)
    fin = np.isfinite(T)
    print(json.dumps({"N": N, "runs": out, "sumT": float(T[fin].sum()), "T11": float(T[1,1])}), flush=True)
    eng.free(dF); eng.free(dT); eng.close()

if __name__ == "__main__":
    for a in sys.argv[1:]:
        run(int(a), prof=True)
