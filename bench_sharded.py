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
    native = getattr(args, "exchange", "native") == "native"
    K = args.passes_per_exchange or (4 if native else 16)
    backend = "gloo" if native else getattr(args, "backend", "nccl")
    ngpu = torch.cuda.device_count()
    dev_idx = local % max(ngpu, 1)
    torch.cuda.set_device(dev_idx)
    device = torch.device("cuda", dev_idx)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=device)
    else:
        dist.init_process_group(backend)
    N = args.size
    g = (N // 2, N // 2)
    row0, nrows = dymu.slab_rows(N, world, rank)
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

        def solve():
            return solver.solve(F.data_ptr(), T_buf.data_ptr(), N, N, N, g[0], g[1], K)
    else:
        from dymu.sharded import SlabSolver

        solver = SlabSolver(eng, N, N, rank, world, row0, nrows, device,
                            passes_per_exchange=K, check_every=4)

        def solve():
            return solver.solve(F, T_buf, g[0], g[1])
    for _ in range(args.warmup):
        solve()
    prof = not args.no_profile
    eng.set_profiling(PROFILE_PERIOD if prof else 0)
    kern_ms, kern_n = 0.0, 0
    tot = {"passes": 0, "tile_visits": 0, "inner_sweeps": 0, "launches": 0, "rounds": 0}
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st = solve()
        for k in tot:
            tot[k] += st[k]
        if prof:
            ms, nl = eng.last_pass_timing()
            kern_ms += ms
            kern_n += nl
    torch.cuda.synchronize()
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
    eng.set_profiling(0)
    if native:
        solver.close()
    eng.close()
    dist.destroy_process_group()
    if rank != 0:
        return None
    return float(dt.item()), tot, kern_ms, kern_n, st
