"""The multi-rank path with the REAL engine: 2 ranks on one GPU (gloo backend,
host-staged boundary rows), dymu.sharded.SlabSolver on torch streams; the
gathered map must equal the oracle FMM.  (RCCL moves the same rows between
GPUs in bench_sharded.py; the orchestration is identical.)"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, nx, ny, goal, F_full, out_q, engine_kw):
    import sys
    import torch  # first: one HIP runtime for torch and libdymu_fim
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "planning-path_planning_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dymu
        from dymu.sharded import SlabSolver
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        row0, nrows = dymu.slab_rows(ny, world, rank)
        eng = dymu.Engine(device=0, **engine_kw)
        F = torch.from_numpy(np.ascontiguousarray(F_full[row0:row0 + nrows])).to(dev)
        T_buf = torch.empty((nrows + 2, nx), dtype=torch.float64, device=dev)
        solver = SlabSolver(eng, nx, ny, rank, world, row0, nrows, dev,
                            passes_per_exchange=2, check_every=2)
        for _ in range(2):  # repeat: workspace/epoch reuse across solves
            st = solver.solve(F, T_buf, goal[0], goal[1])
        torch.cuda.synchronize()
        out_q.put((rank, row0, T_buf[1:nrows + 1].cpu().numpy().copy(), st["rounds"],
                   st["tile_visits"]))
        eng.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nx,ny,goal,engine_kw", [
    (2, 300, 256, (150, 128), dict(kernel=3)),
    (3, 200, 230, (20, 30), dict(kernel=4, prio_target=32)),
    (2, 257, 300, (250, 3), dict(kernel=5, prio_target=8))])
def test_gpu_sharded_matches_oracle(oracle, world, nx, ny, goal, engine_kw):
    import torch.multiprocessing as mp
    F = oracle.synth_speed(nx, ny, seed=41, obst_frac=0.03, obst_seed=43, goal=goal)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nx, ny, goal, F, q, engine_kw))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    T = np.empty((ny, nx))
    for rank, row0, slab, rounds, visits in res:
        T[row0:row0 + slab.shape[0]] = slab
    Tref, _ = oracle.fmm(F, goal)
    assert np.array_equal(np.isinf(T), np.isinf(Tref))
    fin = np.isfinite(Tref)
    assert (np.abs(T[fin] - Tref[fin]) / np.maximum(1, Tref[fin])).max() <= 1e-12


@pytest.mark.parametrize("engine_kw", [dict(kernel=3), dict(kernel=5, prio_target=8)],
                         ids=["fim", "prio16"])
def test_native_rccl_world1_matches_oracle(dymu, oracle, engine_kw):
    """libdymu_dist's RCCL path in-process with a one-rank communicator
    (ncclCommInitRank + the lagged all-reduce; no peers, so no P2P): the
    native loop, the RCCL calls it makes at N=1 and its result vs the oracle.
    Two ranks cannot share one GPU under RCCL ('Duplicate GPU'), so the P2P
    rows are covered by dymu_vdist_solve (test_gpu_slabs.py) and gloo tests."""
    from dymu import dist

    nx, ny, goal = 203, 150, (31, 77)
    F = oracle.synth_speed(nx, ny, seed=5, obst_frac=0.03, obst_seed=6, goal=goal)
    eng = dymu.Engine(device=0, **engine_kw)
    solver = dist.DistSolver(eng, 0, dist.unique_id(), 0, 1)
    dF = eng.alloc(8 * nx * ny)
    dT = eng.alloc(8 * (ny + 2) * nx)
    eng.h2d(dF, F)
    for _ in range(2):  # reuse of the communicator and the workspace
        st = solver.solve(dF, dT, nx, nx, ny, goal[0], goal[1], 4)
    T = np.empty((ny, nx))
    eng.d2h(T, dT + 8 * nx)
    solver.close()
    eng.free(dF)
    eng.free(dT)
    eng.close()
    Tref, _ = oracle.fmm(F, goal)
    assert np.array_equal(np.isinf(T), np.isinf(Tref))
    fin = np.isfinite(Tref)
    assert (np.abs(T[fin] - Tref[fin]) / np.maximum(1, Tref[fin])).max() <= 1e-12
    assert st["rounds"] >= 2 and st["passes"] > 0
