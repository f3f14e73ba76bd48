"""Multi-GPU leg of bench.py: one rank per GPU (torch.distributed.run), the
16384^2 grid split in row slabs (dymu.slab_rows).

--exchange native (default): the C++ loop of libdymu_dist (dymu.dist.DistSolver)
    with its own RCCL communicator on the engine's stream; torch.distributed
    (gloo) only carries the communicator id, barriers and the max-over-ranks time.
--exchange python: dymu.sharded.SlabSolver, the exchange loop in Python over
    torch.distributed ('nccl' = RCCL, or `--backend gloo` to rehearse N ranks on
    one GPU with host-staged rows).
"""
import os
import sys
import time

import torch  # noqa: F401  (first: one HIP runtime for torch and libdymu_fim)
import torch.distributed as dist

import dymu

PROFILE_PERIOD = 64  # time every 64th pass launch of rank 0 (bench.py's roofline)


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
    native = getattr(args, "exchange", "native") == "native" and not fake
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

        obj = [ddist.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        solver = ddist.DistSolver(eng, dev_idx, obj[0], rank, world)
        ranks_seen = solver.comm_count()  # what RCCL itself sees

        def solve():
            return solver.solve(F.data_ptr(), T_buf.data_ptr(), N, N, N, g[0], g[1], K)
    else:
        from dymu.sharded import SlabSolver

        solver = SlabSolver(eng, N, N, rank, world, row0, nrows, device,
                            passes_per_exchange=K, check_every=4)
        ranks_seen = dist.get_world_size()

        def solve():
            return solver.solve(F, T_buf, g[0], g[1])
    slabs = [None] * world
    dist.all_gather_object(slabs, [rank, row0, nrows])
    if ranks_seen != args.gpus or sorted(s[0] for s in slabs) != list(range(args.gpus)):
        raise SystemExit(f"bench: {ranks_seen} ranks seen by the communicator, --gpus "
                         f"{args.gpus}")
    for _ in range(args.warmup):
        solve()
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
    tot["slabs"] = sorted(slabs)
    if fake:
        _dump_fake(T_buf, row0, nrows, rank)
    else:
        eng.set_profiling(0)
    if native:
        solver.close()
    if not fake:
        eng.close()
    dist.destroy_process_group()
    if rank != 0:
        return None
    return float(dt.item()), tot, kern_ms, kern_n, st


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
