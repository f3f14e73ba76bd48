"""Decompose a solve's passes (VERDICT r2 "do this" 3): kernel 5's per-pass
statistics (dymu_set_pass_stats) for the config-3 grid, summarised against the
geometric bound (largest Manhattan tile distance from the goal's tile).

  python tools/pass_decomp.py [--size N] [--out DIR] [--env K=V ...]

Prints one JSON line: totals of every field, the front's progress (the pass at
which the running maximum radius reached each decile of the bound, the passes in
which it did not grow), and the tail after the front reached the corners."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "planning-path_planning_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--obst", type=float, default=0.02)
    ap.add_argument("--out", default=None, help="directory for the raw per-pass records")
    ap.add_argument("--tag", default="decomp")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import dymu

    N = args.size
    g = (N // 2, N // 2)
    eng = dymu.Engine(device=0)
    dF, dT = eng.alloc(8 * N * N), eng.alloc(8 * N * N)
    eng.synth_speed(dF, N, N, N, 0, 1, args.obst, 3, g[0], g[1])
    eng.solve_device(dF, dT, N, N, N, g[0], g[1])  # warmup
    t0 = time.perf_counter()
    st0 = eng.solve_device(dF, dT, N, N, N, g[0], g[1])
    ms_plain = (time.perf_counter() - t0) * 1e3
    eng.set_pass_stats(True)
    recs = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        st = eng.solve_device(dF, dT, N, N, N, g[0], g[1])
        ms = (time.perf_counter() - t0) * 1e3
        recs.append((eng.last_pass_stats(), st, ms))
    eng.set_pass_stats(False)
    eng.free(dF)
    eng.free(dT)
    eng.close()
    tw = st0["tile_w"]
    ntx = (N + tw - 1) // tw
    gx = g[0] // tw
    bound = 2 * max(gx, ntx - 1 - gx)
    for k, (R, st, ms) in enumerate(recs):
        f = {name: R[:, i].astype(np.int64) for i, name in enumerate(dymu.Engine.PASS_STAT_FIELDS)}
        live = f["listed"] > 0
        P = int(live.sum())
        rmax = np.maximum.accumulate(np.where(f["visited"] > 0, f["radius_max"], 0))
        final = int(rmax[-1])
        reach = {}
        for q in range(1, 11):
            r = int(round(final * q / 10))
            idx = np.nonzero(rmax >= r)[0]
            reach[f"{q * 10}%"] = int(idx[0]) if len(idx) else None
        p_final = int(np.nonzero(rmax >= final)[0][0])
        grow = np.diff(np.concatenate([[0], rmax]))
        stalls = int(((grow == 0) & live)[:p_final + 1].sum())
        out = {
            "tag": args.tag, "grid": N, "rep": k, "ms_with_stats": round(ms, 3),
            "ms_without_stats": round(ms_plain, 3), "passes": P, "launches": int(st["launches"]),
            "geometric_bound": bound, "front_final_radius": final,
            "pass_front_reached_final": p_final, "front_stalls_before_final": stalls,
            "tail_passes_after_front": P - p_final - 1,
            "front_reach_pass_by_decile": reach,
            "totals": {name: int(v[live].sum()) for name, v in f.items()
                       if name not in ("radius_max", "radius_min", "bstar")},
            "tail_totals": {name: int(v[p_final + 1:].sum()) for name, v in f.items()
                            if name in ("listed", "visited", "capped", "deadline")},
            "stats": {kk: st[kk] for kk in ("passes", "tile_visits", "deferred", "inner_sweeps")},
        }
        # where the passes went: passes in which the frontier moved, by what stopped it
        out["passes_visit_capped_any"] = int((f["capped"][live] > 0).sum())
        out["passes_deadline_any"] = int((f["deadline"][live] > 0).sum())
        print(json.dumps(out), flush=True)
        if args.out:
            os.makedirs(args.out, exist_ok=True)
            np.save(os.path.join(args.out, f"{args.tag}_rep{k}.npy"), R)


if __name__ == "__main__":
    main()
