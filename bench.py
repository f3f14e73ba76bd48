"""bench.py -- global total-cost-map propagation throughput (Mcells/s).

Workload (BASELINE.json configs[2]): a 16384^2 synthetic grid, one goal at the
centre, F = 1 + 4*u(splitmix64) with 2% iid obstacles,
generated in HBM.  One "step" = one full solve (computeEntireTotalCostMap's
propagation: T initialised, relaxed to convergence, result in HBM).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--size S] [--obst P]

N > 1 runs under torch.distributed.run, one rank per GPU: the grid is cut in
row slabs, one per rank, with RCCL halo exchange driven from C++
(include/dymu_dist.h; bench_sharded.py); value is the whole-job rate
N^2 / max-over-ranks solve time.

Rank 0 prints ONE JSON line with the roofline of the dominant kernel
(k_fim_pass, per-launch HIP events over the timed region) and the CPU baseline
(the oracle's heap FMM, same pop order as the reference, one thread, on a
bounded sample), plus `cpu_reference_algorithm`: the reference's own
linear-scan narrow band (SURVEY s8(d) cpu_fmm_linear) on a 1024^2 sample.
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "planning-path_planning_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E spec peak
BYTES_PER_CELL_VISIT = 24  # read T 8 + read F 8 + write T 8
BYTES_PER_CELL_SOLVE = 16  # read F once + write T once
# The pass kernel's real limiter is the fp64 VALU (and the latency of its pass chain,
# DESIGN.md s4), not HBM.  Kernel 5's sweep loop issues 108 VALU instructions per pair
# of sweeps over a lane's 4 cells (ISA count of the fast path at v35, llvm-objdump of
# fim_kernels.hip; v32: 137): 13.5 per cell update, one of them v_rsq_f64 (issue cost
# ~3x a plain fp64 op, tools/valu_probe.hip).  Peak: MI355X fp64 vector 78.6 TFLOP/s =
# 256 CUs x 4 SIMDs x 16 lanes x 2.4 GHz = 39.3 T lane-instructions/s.
VALU_PER_CELL_UPDATE = {5: 108 / 8}
VALU_PEAK_T = 256 * 4 * 16 * 2.4e9 / 1e12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--obst", type=float, default=0.02)
    ap.add_argument("--cpu-sample", type=int, default=16384,
                    help="edge of the grid the CPU baseline solves (0 = skip)")
    ap.add_argument("--no-profile", action="store_true",
                    help="no per-launch events (roofline reported as null)")
    ap.add_argument("--backend", default="nccl",
                    help="N>1 only: 'nccl' (RCCL over xGMI) or 'gloo' (host-staged rehearsal)")
    ap.add_argument("--exchange", default="native",
                    choices=["native", "rccl", "ipc", "peer", "python"],
                    help="N>1: 'native' = the C++ loop of libdymu_dist with the transport "
                         "chosen on the node before the timed region: RCCL (or IPC when ranks "
                         "share a GPU) vs the GPU-initiated peer transport; 'rccl' / 'ipc' / "
                         "'peer' = that transport only (ipc / peer: N ranks may share one "
                         "GPU); 'python' = dymu.sharded over torch.distributed")
    ap.add_argument("--passes-per-exchange", type=int, default=0,
                    help="passes per exchange round (0: the native loop at N>1 times K = "
                         "2/4/8 before the timed region and keeps the fastest, 4 at N=1; 16 for "
                         "the python loop; tools/vdist_rehearsal.py)")
    ap.add_argument("--no-k-tune", action="store_true",
                    help="N>1 native loop: no transport / K choice before the timed region "
                         "(RCCL or IPC, K = 4)")
    ap.add_argument("--sharded", action="store_true",
                    help="run the row-slab path even at N=1 (exercises the RCCL code path)")
    ap.add_argument("--cpu-linear-size", type=int, default=2048,
                    help="edge of the grid the reference's linear-scan band is timed on")
    ap.add_argument("--sustain-s", type=float, default=8.0,
                    help="after the timed steps, keep solving for this many seconds (not "
                         "timed into `value`): the sustained rate and its spread, and a GPU "
                         "busy long enough for an outside sampler to see; 0 = off")
    ap.add_argument("--no-variants", action="store_true",
                    help="skip the exact-sqrt / deterministic re-runs of the headline solve")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the whole-map comparison with the cpu_baseline's oracle map")
    ap.add_argument("--no-planner", action="store_true",
                    help="skip the class-surface leg (computeEntireTotalCostMap through "
                         "libdymu_planner.so)")
    ap.add_argument("--fake-cpu", action="store_true",
                    help="tests only: the N-rank plumbing on CPU (gloo, numpy stand-in engine, "
                         "python exchange loop); no GPU is touched")
    return ap.parse_args()


def spawn_ranks(n):
    """`bench.py --gpus N` run without a launcher: start the N rank processes with
    torch.distributed.run (one per GPU) as children -- this process never touches the
    GPU -- and return their exit code.  Rank 0's JSON line is the run's output."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def host_cpu():
    """The host the CPU baseline ran on: logical CPUs and the model name."""
    model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "model": model}


def cpu_baseline(n_edge, obst, keep=None):
    """Oracle heap FMM (reference pop order) on an n_edge^2 config-3 grid, 1 thread.
    keep: a dict that receives the oracle's map (keep["T"]) for the parity check."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi

    o = oracle_ffi.load()
    g = (n_edge // 2, n_edge // 2)
    F = o.synth_speed(n_edge, n_edge, seed=1, obst_frac=obst, obst_seed=3, goal=g)
    t0 = time.perf_counter()
    T, _ = o.fmm(F, g)
    dt = time.perf_counter() - t0
    del F
    if keep is not None:
        keep["T"] = T
    return {
        "value": n_edge * n_edge / dt / 1e6,
        "unit": "Mcells/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{n_edge}x{n_edge} config-3 grid (2% obstacles, goal centre), oracle heap "
                  f"FMM with the reference's pop order, 1 thread, {dt:.1f}s",
        "host": host_cpu(),
    }


def oracle_parity(Tg, To, rtol=1e-12):
    """The headline map against the oracle heap FMM's on the same grid (both n x n):
    identical +inf mask, max |Tg - To| / max(1, To) over the finite cells (row blocks,
    so the temporaries stay small)."""
    n = Tg.shape[0]
    worst, finite, mism = 0.0, 0, 0
    for r0 in range(0, n, 1024):
        a, b = Tg[r0:r0 + 1024], To[r0:r0 + 1024]
        fa, fb = np.isfinite(a), np.isfinite(b)
        mism += int(np.count_nonzero(fa != fb))
        both = fa & fb
        finite += int(np.count_nonzero(fb))
        if both.any():
            d = np.abs(a[both] - b[both]) / np.maximum(1.0, b[both])
            worst = max(worst, float(d.max()))
    return {"reference": "oracle heap FMM (the reference's propagation, ported; 1 thread) on the "
                         "same grid, the cpu_baseline run",
            "max_rel": worst, "finite_cells": finite, "mismatched_cells": mism, "rtol": rtol,
            "ok": mism == 0 and worst <= rtol}


def cpu_reference_algorithm(n_edge, obst):
    """SURVEY s8(d) cpu_fmm_linear: the oracle's restatement of the reference's own
    narrow band (minCostGlobalNode, src/DyMu_GlobalPathPlanning.cpp:551-568: linear
    scan for the first strict minimum + vector::erase), 1 thread, bounded sample.
    Its cost is O(cells x band), so the rate falls as the grid grows."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi

    o = oracle_ffi.load()
    g = (n_edge // 2, n_edge // 2)
    F = o.synth_speed(n_edge, n_edge, seed=1, obst_frac=obst, obst_seed=3, goal=g)
    t0 = time.perf_counter()
    o.fmm(F, g, linear=True)
    dt = time.perf_counter() - t0
    return {
        "value": n_edge * n_edge / dt / 1e6,
        "unit": "Mcells/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{n_edge}x{n_edge} config-3 grid, oracle FMM with the reference's linear-scan "
                  f"narrow band (:551-568), 1 thread, {dt:.1f}s; the rate falls with grid size "
                  f"(O(cells x band))",
    }


def cpu_parallel(n_edge, obst):
    """SURVEY s8(d) cpu_fim_omp (optional): the same fixed point on ALL the host threads the
    job may use (OMP_NUM_THREADS, else every CPU) -- oracle_par.c's block FIM with a
    warm-started fast-marching solve per 64x64 tile."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi

    o = oracle_ffi.load()
    host = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS") or 0)
    threads = omp or host
    g = (n_edge // 2, n_edge // 2)
    F = o.synth_speed(n_edge, n_edge, seed=1, obst_frac=obst, obst_seed=3, goal=g)
    t0 = time.perf_counter()
    _, passes = o.fim_parallel(F, g, threads=threads)
    dt = time.perf_counter() - t0
    capped = threads < host
    return {
        "value": n_edge * n_edge / dt / 1e6,
        "unit": "Mcells/s",
        "cores": threads,
        "host_cpus": host,
        # SURVEY s8(d)(3) asks for all host cores; a shared GPU box gives this job a share of
        # them (OMP_NUM_THREADS), which is what is used -- the line says so
        "capped": (f"{threads} of {host} host CPUs: OMP_NUM_THREADS={omp}, the job's CPU share "
                   "on a shared box") if capped else None,
        "kind": "port",
        "sample": f"{n_edge}x{n_edge} config-3 grid, block FIM (64x64 tiles, local fast marching) "
                  f"on {threads} threads{' (capped, of ' + str(host) + ')' if capped else ''}, "
                  f"{passes} passes, {dt:.1f}s; same fixed point as the FMM",
    }


PROFILE_PERIOD = 64  # time every 64th pass launch with HIP events (sampled mean duration;
# ~150 launches over 5 steps; each sampled launch costs ~5-8 us of event overhead: every
# 8th added 3% to the solve, every 32nd 1.3%)
_EXACT = os.environ.get("DYMU_EXACT_SQRT", "0") not in ("", "0")  # dymu_opts.exact_sqrt
KERNEL_NAMES = {3: "k_fim_pass_rb", 4: "k_fim_pass_prio<8>",
                5: f"k_fim_pass_dyn<16, {'false' if _EXACT else 'true'}, false>"}


def geometric_bound(N, gi, gj, tw, th):
    """Largest Manhattan distance, in tiles, from the goal's tile to any tile."""
    nt_x, nt_y = (N + tw - 1) // tw, (N + th - 1) // th
    gx, gy = gi // tw, gj // th
    return max(gx, nt_x - 1 - gx) + max(gy, nt_y - 1 - gy)


def run_single(args):
    import dymu

    N = args.size
    eng = dymu.Engine(device=int(os.environ.get("LOCAL_RANK", "0")))
    n = N * N
    dF, dT = eng.alloc(8 * n), eng.alloc(8 * n)
    g = (N // 2, N // 2)
    eng.synth_speed(dF, N, N, N, 0, 1, args.obst, 3, g[0], g[1])
    for _ in range(args.warmup):
        eng.solve_device(dF, dT, N, N, N, g[0], g[1])
    prof = not args.no_profile
    eng.set_profiling(PROFILE_PERIOD if prof else 0)
    tot = {"passes": 0, "tile_visits": 0, "inner_sweeps": 0, "launches": 0, "deferred": 0}
    kern_ms, kern_n = 0.0, 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st = eng.solve_device(dF, dT, N, N, N, g[0], g[1])
        for k in tot:
            tot[k] += st[k]
        if prof:
            ms, nl = eng.last_pass_timing()
            kern_ms += ms
            kern_n += nl
    dt = time.perf_counter() - t0
    eng.set_profiling(False)
    T = np.empty(2)
    eng.d2h(T, dT)  # touch the result
    if args.sustain_s > 0:  # untimed for `value`: the same solve back to back
        per = []
        t1 = time.perf_counter()
        while time.perf_counter() - t1 < args.sustain_s:
            t2 = time.perf_counter()
            eng.solve_device(dF, dT, N, N, N, g[0], g[1])
            per.append((time.perf_counter() - t2) * 1e3)
        per.sort()
        tot["sustained"] = {"seconds": round(time.perf_counter() - t1, 2), "steps": len(per),
                            "ms_per_step_median": round(per[len(per) // 2], 3),
                            "ms_per_step_min": round(per[0], 3),
                            "ms_per_step_max": round(per[-1], 3),
                            "note": "back-to-back solves after the timed region (not in value)"}
    if getattr(args, "keep_result", False):  # the last timed solve's map, for oracle parity
        tot["T"] = np.empty((N, N))
        eng.d2h(tot["T"], dT)
    # the same solve with the arithmetic / schedule options the headline leaves off
    # (DESIGN.md s4): the correctly rounded sweep sqrt (every update bit-identical
    # to the reference formula, :531-535) and the bit-reproducible schedule
    variants = {}
    if not args.no_variants:
        for name, kw in (("exact_sqrt", dict(exact_sqrt=1)),
                         ("deterministic", dict(deterministic=1))):
            ev = dymu.Engine(device=int(os.environ.get("LOCAL_RANK", "0")), **kw)
            ev.solve_device(dF, dT, N, N, N, g[0], g[1])  # warmup
            n_v = max(2, min(args.steps, 5))
            t1 = time.perf_counter()
            for _ in range(n_v):
                sv = ev.solve_device(dF, dT, N, N, N, g[0], g[1])
            ms = (time.perf_counter() - t1) / n_v * 1e3
            variants[name] = {"ms_per_step": round(ms, 3), "value": round(N * N / ms / 1e3, 3),
                              "passes": sv["passes"], "steps": n_v}
            ev.close()
    eng.free(dF)
    eng.free(dT)
    eng.close()
    tot["variants"] = variants
    return dt, tot, kern_ms, kern_n, st


def planner_leg(N, obst, steps):
    """The drop-in class surface at the headline size: computeEntireTotalCostMap
    (reference :443-468) through libdymu_planner.so (include/DyMu.hpp), the call a
    Rock caller makes.  Each step moves the goal between two valid cells, so every
    step is a cold solve (no map reuse); the speed stays resident on the device and
    the total cost is not downloaded.  Returns ms per step and the same for a step
    that also reads the whole map back (getTotalCostMatrix's download)."""
    import dymu

    g = (N // 2, N // 2)
    eng = dymu.Engine(device=int(os.environ.get("LOCAL_RANK", "0")))
    dF = eng.alloc(8 * N * N)
    eng.synth_speed(dF, N, N, N, 0, 1, obst, 3, g[0], g[1])
    F = np.empty((N, N))
    eng.d2h(F, dF)
    eng.free(dF)
    eng.close()
    cost = np.where(np.isfinite(F), F, -1.0)
    del F
    p = dymu.Planner(device=int(os.environ.get("LOCAL_RANK", "0")))
    p.initGlobalLayer(1.0, 0.5, N, N)
    p.setCostMap(cost)
    goals = [g]
    for d in range(1, 64):  # a second valid goal next to the first
        if p.setGoal((g[0] + d, g[1])):
            goals.append((g[0] + d, g[1]))
            break
    del cost
    p.setGoal(goals[0])
    p.computeEntireTotalCostMap()  # uploads the speed once
    t0 = time.perf_counter()
    for k in range(steps):
        p.setGoal(goals[(k + 1) % len(goals)])
        p.computeEntireTotalCostMap()
    ms = (time.perf_counter() - t0) / steps * 1e3
    # solve + whole-map readback: one untimed step (first 2 GiB host allocation and
    # faults of the process), then the mean of two steps
    ms_read = []
    for k in range(3):
        t0 = time.perf_counter()
        p.setGoal(goals[k % len(goals)])
        p.computeEntireTotalCostMap()
        T = p.totalCostRaw()
        ms_read.append((time.perf_counter() - t0) * 1e3)
        del T
    ms_read = sum(ms_read[1:]) / 2
    kind = p.lastSolveKind()
    p.close()
    return ms, ms_read, kind


def main():
    args = parse()
    world = args.gpus
    env_world = os.environ.get("WORLD_SIZE")
    if world < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    if env_world is None and world > 1:
        sys.exit(spawn_ranks(world))
    if env_world is not None and int(env_world) != world:
        raise SystemExit(f"bench: WORLD_SIZE={env_world} but --gpus {world}: the line would "
                         "mislabel the run")
    rank = int(os.environ.get("RANK", "0"))
    if args.fake_cpu:
        args.exchange, args.backend = "python", "gloo"
    if world > 1 or args.sharded or args.fake_cpu:
        import torch  # noqa: F401  (before dymu: one HIP runtime in the process)
        import bench_sharded

        res = bench_sharded.run(args)
        if res is None:
            return
        dt, tot, kern_ms, kern_n, st = res
    else:
        # the whole map of the last timed solve is checked against the oracle's, which
        # the cpu_baseline leg computes on the same grid anyway
        args.keep_result = (args.cpu_sample == args.size and not args.no_parity)
        dt, tot, kern_ms, kern_n, st = run_single(args)
    if rank != 0:
        return
    N = args.size
    K = args.steps
    value = N * N * K / dt / 1e6
    roof = None
    if kern_n > 0 and kern_ms > 0:
        launch_s = kern_ms * 1e-3 / kern_n  # mean duration of a pass launch (sampled events)
        # (i) SURVEY s8(d)(i), the judged figure: 16 B per cell per solve (read F + write T
        # once), spread over the solve's pass launches
        cells = tot.get("slab_cells", N * N)  # N>1: rank 0's slab, rank 0's launches
        bytes_i = cells * BYTES_PER_CELL_SOLVE * K / tot["launches"]
        achieved = bytes_i / launch_s / 1e9
        # (ii) diagnostic sweep efficiency: 24 B per cell-visit in the launch
        visits = tot.get("rank0_tile_visits", tot["tile_visits"])
        cells_visited = visits * st["tile_w"] * st["tile_h"]
        bytes_ii = cells_visited * BYTES_PER_CELL_VISIT / tot["launches"]
        roof = {
            "bound": "hbm",
            "achieved": round(achieved, 3),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 6),
            "traffic": None,
            "kernel": KERNEL_NAMES.get(st.get("kernel", 3), "k_fim_pass_rb"),
            "per_unit": "16 B per cell per solve (SURVEY s8(d)(i)) / pass launches per solve",
            "bytes_per_launch": bytes_i,
            "avg_launch_us": launch_s * 1e6,
            "launches_per_solve": tot["launches"] / K,
            "timed_launches": f"{kern_n} of {tot['launches']} (1 in {PROFILE_PERIOD})",
            "sweep": {
                "per_unit": "24 B per cell-visit",
                "bytes_per_launch": bytes_ii,
                "achieved": round(bytes_ii / launch_s / 1e9, 3),
                "frac": round(bytes_ii / launch_s / 1e9 / HBM_PEAK_GBS, 6),
            },
            "headline_solve_GBs": round(N * N * BYTES_PER_CELL_SOLVE * K / dt / 1e9, 3),
        }
        vpu = VALU_PER_CELL_UPDATE.get(st.get("kernel"))
        if vpu:
            sweeps = tot.get("rank0_inner_sweeps", tot["inner_sweeps"])
            ops = sweeps * st["tile_w"] * st["tile_h"] * vpu / tot["launches"]
            roof["valu"] = {
                "per_unit": f"{vpu:.1f} fp64-VALU instructions per cell update x tile cells x "
                            "in-tile sweeps in the launch",
                "achieved": round(ops / launch_s / 1e12, 3),
                "peak": VALU_PEAK_T,
                "unit": "T lane-instr/s",
                "frac": round(ops / launch_s / 1e12 / VALU_PEAK_T, 4),
            }
    if roof is not None:
        # HBM bytes per launch from the PMC counters of the same kernel and
        # workload (tools/pmc_round.sh -> tools/pmc_summary.py), if committed
        import glob
        import re

        def natural(f):  # pmc_r01_v10 after pmc_r01_v9
            return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", f)]

        pm = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")), key=natural)
        for f in reversed(pm):  # newest summary of THIS kernel
            d = json.load(open(f))
            if d.get("kernel") and roof["kernel"] in d["kernel"] and d.get("grid", N) == N:
                roof["traffic"] = round(d["traffic_bytes_per_launch"])
                roof["traffic_unit"] = ("HBM bytes per launch (PMC FETCH_SIZE + WRITE_SIZE, "
                                        "calibrated: " + d.get("correction", "FETCH_SIZE x2") + ")")
                roof["traffic_source"] = os.path.basename(f)
                break
    line = {
        "metric": "global total-cost-map Mcells/s (16384^2 grid); iters to converge",
        "value": round(value, 3),
        "unit": "Mcells/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": round(dt / K * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": f"config 3: {N}x{N} grid, {world}x MI355X, splitmix64 U(1,5) speed, "
                        f"{args.obst:.0%} iid obstacles, goal centre, full solve",
            "grid": N,
            # what the headline computes in (DESIGN.md s4 "Sweep sqrt", s3 tolerance)
            "arith": ("fp64, correctly rounded sweep sqrt (DYMU_EXACT_SQRT=1)" if _EXACT else
                      "fp64, approx sweep sqrt (one Goldschmidt step, <= 36 ulp on the sqrt "
                      "term of each candidate; solve error vs the reference FMM <= 1e-14 rel)"),
            "schedule": "default (sweep deadline + first-insertion histogram: last ulps vary "
                        "run to run)",
            "parallelism": ("single" if world == 1 and not args.sharded else
                            f"row-slab x{world} ("
                            + {"rccl": "RCCL P2P + all-reduce, native C++ loop",
                               "ipc": "hipIpc rows + shared-memory board, native C++ loop",
                               "peer": "GPU-initiated peer pushes with sequence tags + status "
                                       "board, native C++ loop"}
                            .get(tot.get("transport"), f"{args.backend}, torch.distributed loop")
                            + ")"),
            "transport": tot.get("transport"),
            "exchange_rounds_per_solve": tot.get("rounds", 0) / K,
            "passes_per_exchange": tot.get("passes_per_exchange"),
            "passes_per_solve": tot["passes"] / K,
            # a tile is first relaxed one pass after its 4-neighbour that reaches it,
            # so no solve takes fewer passes than the largest Manhattan tile distance
            # from the goal's tile (1024 at 16384^2 with 16x16 tiles)
            "passes_geometric_bound": geometric_bound(N, N // 2, N // 2, st.get("tile_w", 16),
                                                      st.get("tile_h", 16)),
            "tile_visits_per_solve": tot["tile_visits"] / K,
            "entries_deferred_per_solve": tot.get("deferred", 0) / K,
            "inner_sweeps_per_solve": tot["inner_sweeps"] / K,
            "pass_kernel": st.get("kernel"),
            "ranks_seen": tot.get("ranks_seen", 1),
            "slabs": tot.get("slabs", [[0, 0, N]]),
        },
        "roofline": roof,
        "cpu_baseline": None,
    }
    if tot.get("k_autotune_ms"):  # untimed setup solves per candidate transport x K (max over ranks)
        line["config"]["k_autotune_ms"] = tot["k_autotune_ms"]
    if tot.get("transports_dropped"):  # candidates that failed on some rank before timing
        line["config"]["transports_dropped"] = tot["transports_dropped"]
    if tot.get("variants"):
        line["variants"] = tot["variants"]
    if tot.get("sustained"):
        line["sustained"] = tot["sustained"]
    if tot.get("parity") is not None:  # the sharded run's self-check (bench_sharded.self_check)
        line["parity"] = tot["parity"]
    if args.fake_cpu:
        line["data"] = "synthetic; --fake-cpu plumbing rehearsal (numpy engine, not a GPU number)"
    if world == 1 and not args.no_planner and not args.fake_cpu and not args.sharded:
        pms, pms_read, kind = planner_leg(N, args.obst, max(2, min(K, 5)))
        line["planner"] = {
            "api": "DyMuPathPlanner::computeEntireTotalCostMap via libdymu_planner.so (C-ABI)",
            "ms_per_step": round(pms, 3),
            "ratio_to_engine": round(pms / (dt / K * 1e3), 3),
            "ms_with_full_map_readback": round(pms_read, 3),
            "note": "goal alternates between two cells, so every step is a cold solve; the "
                    "readback step adds getTotalCostMatrix's 2 GiB D2H",
            "last_solve_kind": kind,
        }
    if world == 1 and args.cpu_sample > 0 and not args.fake_cpu:
        keep = {} if tot.get("T") is not None else None
        line["cpu_baseline"] = cpu_baseline(args.cpu_sample, args.obst, keep)
        if keep:
            line["parity"] = oracle_parity(tot.pop("T"), keep.pop("T"))
        line["cpu_reference_algorithm"] = cpu_reference_algorithm(args.cpu_linear_size, args.obst)
        line["cpu_parallel"] = cpu_parallel(args.cpu_sample, args.obst)
    print(json.dumps(line), flush=True)
    if line.get("parity") is not None and not line["parity"]["ok"]:
        sys.exit(f"bench: the map failed its parity check: {line['parity']}")


if __name__ == "__main__":
    main()
