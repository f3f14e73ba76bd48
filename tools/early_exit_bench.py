"""Early-exit propagation (computeTotalCostMap, dymu_solve_until_device) timings:
goal at the centre of an N^2 config-3 grid, starts at increasing distances.
Prints one JSON object (per start: t_closed, passes, launches, ms median of 3).
usage: python tools/early_exit_bench.py [N ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "planning-path_planning_amd"))
import dymu  # noqa: E402


def main():
    out = {"pipeline": os.environ.get("DYMU_PIPELINE", "default")}
    for N in [int(x) for x in sys.argv[1:]] or [4096]:
        e = dymu.Engine()
        dF, dT = e.alloc(8 * N * N), e.alloc(8 * N * N)
        g = (N // 2, N // 2)
        e.synth_speed(dF, N, N, N, 0, 1, 0.02, 3, g[0], g[1])
        rows = []
        for d in (16, 256, N // 4, N // 2 - 1):
            s = (g[0] + d, g[1] + d // 2)
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                tc, st = e.solve_until_device(dF, dT, N, N, N, g[0], g[1], s[0], s[1])
                ts.append(time.perf_counter() - t0)
            rows.append({"start": s, "t_closed": tc, "passes": st["passes"],
                         "launches": st["launches"], "ms": round(sorted(ts)[1] * 1e3, 3)})
        full = []
        for _ in range(3):
            t0 = time.perf_counter()
            st = e.solve_device(dF, dT, N, N, N, g[0], g[1])
            full.append(time.perf_counter() - t0)
        out[str(N)] = {"early": rows, "full_ms": round(sorted(full)[1] * 1e3, 3),
                       "full_passes": st["passes"]}
        e.free(dF)
        e.free(dT)
        e.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
