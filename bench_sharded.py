"""Multi-GPU leg of bench.py: one rank per GPU (torch.distributed.run), the
16384^2 grid split in row slabs (dymu.slab_rows).

--exchange native (default): the C++ loop of libdymu_dist (dymu.dist.DistSolver);
    the transport is chosen on the node before the timed region among RCCL (its
    own communicator on the engine's stream; only when every rank has its own GPU)
    or IPC (ranks sharing a GPU) and the GPU-initiated peer transport (the pass
    kernels push the boundary rows themselves), together with the passes per
    round; torch.distributed (gloo) only carries the ids, barriers and the
    max-over-ranks time.
--exchange rccl | ipc | peer: that transport only (ipc / peer run N ranks on ONE
    GPU too, where RCCL refuses duplicate devices).
--exchange python: dymu.sharded.SlabSolver, the exchange loop in Python over
    torch.distributed ('nccl' = RCCL, or `--backend gloo` to rehearse N ranks on
    one GPU with host-staged rows).

After the timed steps every run checks the stitched map it produced (self_check):
each slab's fixed-point residual under the reference update (propagateGlobalNode,
src/DyMu_GlobalPathPlanning.cpp:500-546) against its ghost rows, the ghost rows
against the neighbours' real boundary rows, and the all-reduced sum / count of
the finite total costs against a single-GPU solve of the same grid on rank 0.
"""
import os
import sys
import time

import torch  # noqa: F401  (first: one HIP runtime for torch and libdymu_fim)
import torch.distributed as dist

import dymu

PROFILE_PERIOD = 64  # time every 64th pass launch of rank 0 (bench.py's roofline)


K_CANDIDATES = (2, 4, 8)  # passes per exchange round tried before the timed region (N > 1)
TUNE_TIMEOUT_S = 30.0  # bound on a host wait on a peer while candidates are timed


def _injected_failure(rank):
    """Test knob DYMU_BENCH_FAIL_CANDIDATE=transport:rank -- that rank makes the
    candidate's timing solves fail (a null speed slab: every rank's pre-flight refuses
    it), so tests can check that the bench drops it and still prints its line."""
    kv = os.environ.get("DYMU_BENCH_FAIL_CANDIDATE", "")
    if ":" not in kv:
        return None
    tr, r = kv.split(":", 1)
    return tr if int(r) == rank else None


def _env_defaults():
    # `bench.py --sharded` without torchrun: a world of one
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")


def run(args):
    _env_defaults()
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ["LOCAL_RANK"])
    fake = getattr(args, "fake_cpu", False)
    exchange = getattr(args, "exchange", "native")
    native = exchange in ("native", "rccl", "ipc", "peer") and not fake
    K = args.passes_per_exchange or (4 if native else 16)
    backend = "gloo" if (native or fake) else getattr(args, "backend", "nccl")
    if fake:  # CPU rehearsal of the rank plumbing (tests): numpy stand-in engine
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests"))
        from fake_engine import FakeEngine

        device = torch.device("cpu")
        dev_idx = 0
    else:
        ngpu = torch.cuda.device_count()
        dev_idx = local % max(ngpu, 1)
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=device)
    else:
        dist.init_process_group(backend)
    if dist.get_world_size() != args.gpus:
        raise SystemExit(f"bench: torch.distributed world {dist.get_world_size()} != --gpus "
                         f"{args.gpus}")
    N = args.size
    g = (N // 2, N // 2)
    row0, nrows = dymu.slab_rows(N, world, rank)
    if fake:
        eng = FakeEngine()
        F = torch.from_numpy(_fake_speed(N, row0, nrows, args.obst, g))
        T_buf = torch.empty((nrows + 2, N), dtype=torch.float64)
    else:
        eng = dymu.Engine(device=dev_idx)
        F = torch.empty((nrows, N), dtype=torch.float64, device=device)
        T_buf = torch.empty((nrows + 2, N), dtype=torch.float64, device=device)
        stream = torch.cuda.current_stream(device).cuda_stream
        eng.synth_speed(F.data_ptr(), N, nrows, N, row0, 1, args.obst, 3, g[0], g[1], stream)
        torch.cuda.synchronize()
    if native:
        from dymu import dist as ddist

        if exchange == "native":  # candidates, chosen on the node below
            # RCCL refuses two ranks on one GPU: ranks sharing a GPU compare IPC instead
            shared = world > max(torch.cuda.device_count(), 1) if not fake else True
            cands = ["ipc" if shared else "rccl", "peer"] if world > 1 else ["rccl"]
        else:
            cands = [exchange]
        solvers, dropped = {}, {}
        devs = [None] * world
        dist.all_gather_object(devs, dev_idx)
        for tr in cands:
            obj = [ddist.unique_id(tr) if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            ok = 1
            if tr == "peer":
                # the pass kernels store into the neighbours' memory: both neighbour
                # devices must be peer-accessible from this one (VERDICT r4 "do this" 4)
                nb = [devs[r] for r in (rank - 1, rank + 1) if 0 <= r < world]
                no = [d for d in nb if d != dev_idx and
                      not torch.cuda.can_device_access_peer(dev_idx, d)]
                if no:
                    dropped[tr] = f"device {dev_idx} has no peer access to device(s) {no}"
                    ok = 0
            if ok:
                try:
                    solvers[tr] = ddist.DistSolver(eng, dev_idx, obj[0], rank, world,
                                                   transport=tr)
                except dymu.DymuError as e:
                    dropped[tr] = str(e)
                    ok = 0
            if not _all_ok(ok) and len(cands) > 1:  # a candidate that fails anywhere is dropped
                dropped.setdefault(tr, "failed on another rank")
                if tr in solvers:
                    solvers.pop(tr).close()
            elif not ok:
                raise SystemExit(f"bench: transport {tr}: {dropped[tr]}")
        if not solvers:
            raise SystemExit(f"bench: no transport works: {dropped}")
        transport = next(iter(solvers))
        ranks_seen = min(sv.comm_count() for sv in solvers.values())  # what the transports see

        def solve(k=None, tr=None):
            return solvers[tr or transport].solve(F.data_ptr(), T_buf.data_ptr(), N, N, N, g[0],
                                                  g[1], k or K)
    else:
        from dymu.sharded import SlabSolver

        solver = SlabSolver(eng, N, N, rank, world, row0, nrows, device,
                            passes_per_exchange=K, check_every=4)
        ranks_seen = dist.get_world_size()

        def solve(k=None, tr=None):
            return solver.solve(F, T_buf, g[0], g[1])
    slabs = [None] * world
    dist.all_gather_object(slabs, [rank, row0, nrows])
    if ranks_seen != args.gpus or sorted(s[0] for s in slabs) != list(range(args.gpus)):
        raise SystemExit(f"bench: {ranks_seen} ranks seen by the communicator, --gpus "
                         f"{args.gpus}")
    for _ in range(args.warmup):
        for tr in (list(solvers) if native else [None]):
            if native and len(solvers) > 1:
                # a candidate whose solve fails on any rank (its peers fail fast through the
                # board's abort flag) is dropped on every rank before the timed region
                try:
                    solve(None, tr)
                    ok = 1
                except dymu.DymuError as e:
                    dropped[tr], ok = str(e), 0
                if not _all_ok(ok):
                    dropped.setdefault(tr, "failed on another rank")
                    solvers.pop(tr).close()
                    transport = next(iter(solvers))
            else:
                solve(None, tr)
    k_tune = None
    tune = native and world > 1 and not getattr(args, "no_k_tune", False)
    if tune:
        # transport and passes per round, chosen on this node before the timed region: a
        # round's exchange latency over xGMI is what the one-GPU rehearsal cannot see
        # (DESIGN.md s5); every rank runs every candidate (transport x K, or the given K),
        # the max over ranks of the best of two solves decides, and all ranks get the
        # same choice.  Every candidate solve is a full solve of the same grid.
        k_tune, sums = {}, {}
        ks = [args.passes_per_exchange] if args.passes_per_exchange else list(K_CANDIDATES)
        # a candidate that hangs (a peer or RCCL transport never tried across these GPUs)
        # gives up after TUNE_TIMEOUT_S instead of the 300-s default, fails on every rank
        # and is dropped with its reason: the line still prints (VERDICT r4 "do this" 4)
        ddist.set_timeout(min(TUNE_TIMEOUT_S, float(os.environ.get("DYMU_DIST_TIMEOUT_S") or 1e9)))
        fail_at = _injected_failure(rank)
        for tr in list(solvers):
            k_tune[tr] = {}
            failed = False
            for k in ks:
                best = float("inf")
                for _ in range(2):
                    dist.barrier()
                    torch.cuda.synchronize()
                    t = time.perf_counter()
                    ok = 1
                    try:
                        if fail_at == tr:  # test knob: this rank passes a null speed slab
                            solvers[tr].solve(0, T_buf.data_ptr(), N, N, N, g[0], g[1], k)
                        else:
                            solve(k, tr)
                    except dymu.DymuError as e:
                        dropped[tr], ok = f"failed while timing K={k}: {e}", 0
                    torch.cuda.synchronize()
                    el = torch.tensor([time.perf_counter() - t], dtype=torch.float64)
                    dist.all_reduce(el, op=dist.ReduceOp.MAX)
                    if not _all_ok(ok):
                        failed = True
                        break
                    best = min(best, float(el.item()))
                if failed:
                    break
                k_tune[tr][k] = round(best * 1e3, 3)
            if failed:
                dropped.setdefault(tr, "failed on another rank while timing")
                k_tune.pop(tr)
                solvers.pop(tr).close()
                continue
            sums[tr] = _map_checksum(T_buf, nrows)
        ddist.set_timeout(0)
        if not k_tune:
            raise SystemExit(f"bench: every transport failed while timing: {dropped}")
        # a candidate whose map disagrees with the first candidate's (finite-cell count, or
        # the sum beyond the tolerance) is dropped before the timed region; the timed
        # transport's own map is checked in full afterwards (self_check)
        first = next(iter(sums))
        for tr in list(k_tune)[1:]:
            (s0, n0), (s1, n1) = sums[first], sums[tr]
            if n1 != n0 or abs(s1 - s0) > RTOL * max(abs(s0), 1.0):
                dropped[tr] = f"map differs from {first}'s: sum {s1!r} vs {s0!r}, cells {n1} vs {n0}"
                k_tune.pop(tr)
        # identical on every rank (max-reduced times)
        transport, K = min(((tr, k) for tr in k_tune for k in k_tune[tr]),
                           key=lambda c: k_tune[c[0]][c[1]])
    prof = not args.no_profile and not fake
    if not fake:
        eng.set_profiling(PROFILE_PERIOD if prof else 0)
    kern_ms, kern_n = 0.0, 0
    tot = {"passes": 0, "tile_visits": 0, "inner_sweeps": 0, "launches": 0, "rounds": 0}
    sync = (lambda: None) if fake else torch.cuda.synchronize
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st = solve()
        for k in tot:
            tot[k] += st.get(k, 0)
        if prof:
            ms, nl = eng.last_pass_timing()
            kern_ms += ms
            kern_n += nl
    sync()
    dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                      device=device if backend == "nccl" else "cpu")
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    if os.environ.get("DYMU_BENCH_VERBOSE"):
        print(f"rank {rank}: rows {row0}+{nrows} {tot} {time.perf_counter() - t0:.4f}s",
              flush=True)
    tot["rank0_tile_visits"] = tot["tile_visits"]  # this rank's (rank 0 reports)
    tot["rank0_inner_sweeps"] = tot["inner_sweeps"]
    agg = torch.tensor([tot["tile_visits"], tot["inner_sweeps"], tot["passes"]],
                       dtype=torch.float64, device=dt.device)
    dist.all_reduce(agg)
    tot["tile_visits"], tot["inner_sweeps"] = int(agg[0]), int(agg[1])
    tot["passes_sum_ranks"] = int(agg[2])
    tot["slab_cells"] = nrows * N  # rank 0's slab: the roofline's per-launch bytes
    tot["ranks_seen"] = ranks_seen
    tot["passes_per_exchange"] = K
    if native:
        tot["transport"] = transport
        if dropped:
            tot["transports_dropped"] = dropped
        if transport == "peer" and k_tune is not None and len(sums) > 1:
            tot["peer_validated"] = (f"map checksum equal to {next(iter(sums))}'s before the "
                                     "timed region; self_check after it")
    if k_tune is not None:
        tot["k_autotune_ms"] = k_tune
    tot["slabs"] = sorted(slabs)
    if fake:
        _dump_fake(T_buf, row0, nrows, rank)
    else:
        eng.set_profiling(0)
    if native:
        for sv in solvers.values():
            sv.close()
    tot["parity"] = self_check(eng, F, T_buf, N, row0, nrows, rank, world, g, args.obst, fake,
                               dt.device)
    if not fake:
        eng.close()
    dist.destroy_process_group()
    if rank != 0:
        return None
    return float(dt.item()), tot, kern_ms, kern_n, st


def _map_checksum(T_buf, nrows):
    """(sum, count) of the finite owned total costs over all ranks (gloo all-reduce)"""
    own = T_buf[1:nrows + 1]
    fin = torch.isfinite(own)
    t = torch.tensor([float(own[fin].sum().item()), float(fin.sum().item())], dtype=torch.float64)
    dist.all_reduce(t)
    return float(t[0]), int(t[1])


def _all_ok(ok):
    """every rank's flag (gloo all-reduce MIN)"""
    t = torch.tensor([ok], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


RTOL = 1e-12  # SURVEY s8(c) / DESIGN.md s3 tolerance


def _update_rows(P, F):
    """The reference update (:504-535, restated in torch fp64, no FMA contraction:
    one op per kernel) of the rows of P[1:-1] against P (row 0 / -1: the halo rows)."""
    import torch

    inf = float("inf")
    own = P[1:-1]
    ty = torch.minimum(P[:-2], P[2:])
    pad = torch.full((own.shape[0], 1), inf, dtype=own.dtype, device=own.device)
    tx = torch.minimum(torch.cat([pad, own[:, :-1]], 1), torch.cat([own[:, 1:], pad], 1))
    d = tx - ty
    two = ((tx + ty) + torch.sqrt(2.0 * (F * F) - d * d)) * 0.5
    return torch.where(torch.abs(d) < F, two, torch.minimum(tx, ty) + F)


def self_check(eng, F, T_buf, N, row0, nrows, rank, world, g, obst, fake, red_dev):
    """The stitched map's parity, measured after the timed region (VERDICT r2 "do
    this" 1).  Returns rank 0's verdict dict (None elsewhere)."""
    import torch

    inf = float("inf")
    lo, hi = rank > 0, rank < world - 1
    P = T_buf.clone()  # ghost rows of the edge slabs are not part of the domain: +inf
    if not lo:
        P[0] = inf
    if not hi:
        P[-1] = inf
    worst, bad = 0.0, 0
    gl = g[1] - row0 if row0 <= g[1] < row0 + nrows else -1
    chunk = 1024
    for j0 in range(0, nrows, chunk):
        j1 = min(nrows, j0 + chunk)
        u = _update_rows(P[j0:j1 + 2], F[j0:j1])
        t = P[j0 + 1:j1 + 1]
        free = torch.isfinite(F[j0:j1])
        if j0 <= gl < j1:
            free[gl - j0, g[0]] = False
            bad += int(t[gl - j0, g[0]].item() != 0.0)
        bad += int((~torch.isinf(t[~torch.isfinite(F[j0:j1])])).sum())  # obstacles stay +inf
        tf, uf = t[free], u[free]
        bad += int((torch.isinf(tf) != torch.isinf(uf)).sum())  # reachability
        fin = torch.isfinite(tf) & torch.isfinite(uf)
        if bool(fin.any()):
            worst = max(worst, (torch.abs(tf[fin] - uf[fin]) /
                                torch.clamp(tf[fin], min=1.0)).max().item())
    # ghost rows == the neighbours' real boundary rows (after termination they must be)
    edge = torch.stack([T_buf[1], T_buf[nrows]]).to(red_dev)
    edges = [torch.empty_like(edge) for _ in range(world)]
    dist.all_gather(edges, edge)
    edges = [e.cpu() for e in edges]
    ghost = 0.0
    if lo:
        ghost = max(ghost, (T_buf[0].cpu() - edges[rank - 1][1]).abs().nan_to_num(0.0).max().item())
        bad += int((torch.isinf(T_buf[0].cpu()) != torch.isinf(edges[rank - 1][1])).sum())
    if hi:
        ghost = max(ghost, (T_buf[nrows + 1].cpu() - edges[rank + 1][0]).abs().nan_to_num(0.0)
                    .max().item())
        bad += int((torch.isinf(T_buf[nrows + 1].cpu()) != torch.isinf(edges[rank + 1][0])).sum())
    own = T_buf[1:nrows + 1]
    fin = torch.isfinite(own)
    agg = torch.tensor([float(own[fin].sum().item()), float(fin.sum().item()), float(bad)],
                       dtype=torch.float64, device=red_dev)
    dist.all_reduce(agg)
    res = torch.tensor([worst, ghost], dtype=torch.float64, device=red_dev)
    dist.all_reduce(res, op=dist.ReduceOp.MAX)
    if rank != 0:
        return None
    s_sh, n_sh, bad = float(agg[0]), int(agg[1]), int(agg[2])
    s_1, n_1 = _single_reference(eng, N, g, obst, fake, F.device)
    sum_rel = abs(s_sh - s_1) / max(abs(s_1), 1.0)
    out = {"residual": float(res[0]), "ghost_max_abs_diff": float(res[1]), "sum_rel": sum_rel,
           "finite_cells": n_sh, "finite_cells_single": n_1, "mismatched_cells": bad,
           "reference": "single-GPU dymu_solve_device of the same grid" if not fake else
           "numpy Jacobi of the same grid (--fake-cpu)", "rtol": RTOL}
    out["ok"] = bool(out["residual"] <= RTOL and sum_rel <= RTOL and n_sh == n_1 and bad == 0
                     and float(res[1]) == 0.0)
    return out


def _single_reference(eng, N, g, obst, fake, device):
    """Sum and count of the finite total costs of the whole grid solved on ONE
    device (rank 0): the value the stitched slabs must reproduce."""
    import torch

    if fake:
        from fake_engine import FakeEngine
        import numpy as np

        Fh = np.ascontiguousarray(_fake_speed(N, 0, N, obst, g))
        Tb = np.empty((N + 2, N))
        fe = FakeEngine()
        fe.dom_begin(Fh.ctypes.data, Tb.ctypes.data + 8 * N, N, N, N, 0, 0, g[0], g[1])
        while fe.dirty:
            fe.dom_run(64)
        T = Tb[1:N + 1]
        fin = np.isfinite(T)
        return float(T[fin].sum()), int(fin.sum())
    Ff = torch.empty((N, N), dtype=torch.float64, device=device)
    Tf = torch.empty((N, N), dtype=torch.float64, device=device)
    stream = torch.cuda.current_stream(device).cuda_stream
    eng.synth_speed(Ff.data_ptr(), N, N, N, 0, 1, obst, 3, g[0], g[1], stream)
    eng.solve_device(Ff.data_ptr(), Tf.data_ptr(), N, N, N, g[0], g[1], stream)
    torch.cuda.synchronize()
    fin = torch.isfinite(Tf)
    r = float(Tf[fin].sum().item()), int(fin.sum().item())
    del Ff, Tf
    torch.cuda.empty_cache()
    return r


def _fake_speed(N, row0, nrows, obst, g):
    """Rows [row0, row0+nrows) of the config-3 speed: the numbers k_synth writes on the
    GPU, from the numpy restatement of its generator in tests/fake_engine.py."""
    from fake_engine import synth_rows

    return synth_rows(N, row0, nrows, seed=1, obst_frac=obst, obst_seed=3, goal=g)


def _dump_fake(T_buf, row0, nrows, rank):
    """--fake-cpu: each rank's owned rows to $DYMU_BENCH_DUMP (the test compares them with
    the oracle; the bench itself never reads the oracle)."""
    import numpy as np

    d = os.environ.get("DYMU_BENCH_DUMP")
    if d:
        np.save(os.path.join(d, f"T_rank{rank}_row{row0}.npy"), T_buf[1:nrows + 1].numpy())
