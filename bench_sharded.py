"""Multi-GPU leg of bench.py: one rank per GPU (torch.distributed.run), the
16384^2 grid split in row slabs (dymu.slab_rows), solved by
dymu.sharded.SlabSolver with boundary-row exchange over RCCL ('nccl').
`--backend gloo` rehearses N ranks on one GPU with host-staged rows."""
import os
import time

import torch  # noqa: F401  (first: one HIP runtime for torch and libdymu_fim)
import torch.distributed as dist

import dymu
from dymu.sharded import SlabSolver

PROFILE_PERIOD = 8  # time every 8th pass launch of rank 0 (bench.py's roofline)


def run(args):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = getattr(args, "backend", "nccl")
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
    solver = SlabSolver(eng, N, N, rank, world, row0, nrows, device,
                        passes_per_exchange=args.passes_per_exchange, check_every=4)
    for _ in range(args.warmup):
        solver.solve(F, T_buf, g[0], g[1])
    prof = not args.no_profile
    eng.set_profiling(PROFILE_PERIOD if prof else 0)
    kern_ms, kern_n = 0.0, 0
    tot = {"passes": 0, "tile_visits": 0, "inner_sweeps": 0, "launches": 0, "rounds": 0}
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st = solver.solve(F, T_buf, g[0], g[1])
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
    tot["rank0_tile_visits"] = tot["tile_visits"]  # this rank's (rank 0 reports)
    agg = torch.tensor([tot["tile_visits"], tot["inner_sweeps"], tot["passes"]],
                       dtype=torch.float64, device=dt.device)
    dist.all_reduce(agg)
    tot["tile_visits"], tot["inner_sweeps"] = int(agg[0]), int(agg[1])
    tot["passes_sum_ranks"] = int(agg[2])
    tot["slab_cells"] = nrows * N  # rank 0's slab: the roofline's per-launch bytes
    eng.set_profiling(0)
    eng.close()
    dist.destroy_process_group()
    if rank != 0:
        return None
    return float(dt.item()), tot, kern_ms, kern_n, st
