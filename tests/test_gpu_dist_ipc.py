"""The native multi-rank loop across PROCESSES on one GPU: libdymu_dist's round
loop (run_rounds: pre-flight, fused rounds, mailbox posts of the reduced count,
termination) over the IPC transport -- rows pushed into the neighbours'
hipIpc-mapped receive rows, counts reduced through a /dev/shm board.  It is the
loop the RCCL bench runs (dymu_dist_solve), with RCCL's P2P and all-reduce
replaced: RCCL refuses two ranks on one GPU ("Duplicate GPU"), IPC does not.
The stitched map must equal the oracle FMM (reference
src/DyMu_GlobalPathPlanning.cpp:443-468 distributed as SURVEY.md s8(e))."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _worker(rank, world, uid, nx, ny, goal, F_full, out_q, engine_kw, bad_rank, bad_kind,
            transport):
    os.environ.setdefault("DYMU_DIST_TIMEOUT_S", "90")
    import sys
    import time
    t0 = time.monotonic()
    marks = []
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "planning-path_planning_amd"))
    import dymu
    from dymu import dist

    try:
        row0, nrows = dymu.slab_rows(ny, world, rank)
        eng = dymu.Engine(device=0, **engine_kw)
        solver = dist.DistSolver(eng, 0, uid, rank, world, transport=transport)
        marks.append(("joined", round(time.monotonic() - t0, 2)))
        seen = solver.comm_count()
        dF = eng.alloc(8 * nrows * nx)
        dT = eng.alloc(8 * (nrows + 2) * nx)
        eng.h2d(dF, np.ascontiguousarray(F_full[row0:row0 + nrows]))
        pre = None
        if bad_rank is not None:  # one rank passes an invalid slab / another K: all refuse
            bad = rank == bad_rank
            wide = nx + 64 if bad and bad_kind == "nx" else nx  # a wider grid (and pitch)
            K = 1 if bad_kind == "k1" else (3 if bad and bad_kind == "k" else 4)
            try:
                solver.solve(0 if bad and bad_kind == "slab" else dF, dT, wide, wide, ny, goal[0],
                             goal[1], K)
                pre = "solved"
            except dymu.DymuError as e:
                pre = e.status
            marks.append(("preflight", round(time.monotonic() - t0, 2)))
        sts = [solver.solve(dF, dT, nx, nx, ny, goal[0], goal[1], 4) for _ in range(2)]
        T = np.empty((nrows, nx))
        eng.d2h(T, dT + 8 * nx)
        solver.close()
        eng.free(dF)
        eng.free(dT)
        eng.close()
        out_q.put((rank, row0, T, [s["rounds"] for s in sts], seen, pre, None))
    except Exception as e:  # reported to the parent, which fails the test
        marks.append(("error", round(time.monotonic() - t0, 2)))
        out_q.put((rank, 0, None, None, 0, None, f"rank {rank}: {e!r} {marks}"))


def _run(oracle, world, nx, ny, goal, engine_kw, bad_rank=None, bad_kind="slab", transport="ipc",
         obst=0.03):
    import multiprocessing as mp
    from dymu import dist

    F = oracle.synth_speed(nx, ny, seed=71, obst_frac=obst, obst_seed=73, goal=goal)
    uid = dist.unique_id(transport)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, uid, nx, ny, goal, F, q, engine_kw, bad_rank, bad_kind,
                               transport))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    errs = [r[6] for r in res if r[6]]
    assert not errs, errs
    T = np.empty((ny, nx))
    for rank, row0, slab, rounds, seen, pre, _ in res:
        T[row0:row0 + slab.shape[0]] = slab
        assert seen == world
        assert min(rounds) >= 2
        if bad_rank is not None:
            assert pre == -1, f"rank {rank}: pre-flight gave {pre}"
    # every rank ran the same rounds (lock-step transports); the peer ranks all stop at
    # the same check but may have queued a different number of rounds by then
    if transport != "peer":
        assert len({tuple(r[3]) for r in res}) == 1
    Tref, _ = oracle.fmm(F, goal)
    assert np.array_equal(np.isinf(T), np.isinf(Tref))
    fin = np.isfinite(Tref)
    assert (np.abs(T[fin] - Tref[fin]) / np.maximum(1, Tref[fin])).max() <= 1e-12


@pytest.mark.parametrize("world,nx,ny,goal,engine_kw", [
    (2, 257, 300, (250, 3), dict(kernel=5, prio_target=8)),      # fused rounds
    (3, 300, 420, (150, 200), dict(kernel=5, prio_target=16)),   # goal in the middle slab
    (3, 200, 230, (20, 30), dict(kernel=4, prio_target=32)),     # exchange launch (no fusion)
], ids=["w2-fused", "w3-middle", "w3-k4"])
def test_ipc_loop_across_processes_matches_oracle(dymu, oracle, world, nx, ny, goal, engine_kw):
    _run(oracle, world, nx, ny, goal, engine_kw)


@pytest.mark.parametrize("bad_kind", ["slab", "k", "nx"])
def test_ipc_preflight_rejects_on_every_rank(dymu, oracle, bad_kind):
    """A rank-local argument error (a null speed slab on rank 1), a rank passing
    another K than its peers (which would run other rounds and leave them waiting),
    or a rank passing a wider grid (whose receive rows must not be re-allocated and
    re-published alone: ADVICE r3) fails every rank with DYMU_ERR_ARG through the
    collective pre-flight; the next solves work."""
    _run(oracle, 3, 160, 200, (80, 100), dict(kernel=5, prio_target=8), bad_rank=1,
         bad_kind=bad_kind)


# The GPU-initiated peer transport (dymu_dist_create_peer, DESIGN.md s5 "Peer
# transport"): the pass kernels push their boundary rows' decreases into the
# neighbours' receive rows with sequence tags, no host step per round; termination
# from the ranks' posted status.  Same processes-on-one-GPU harness and oracle.
@pytest.mark.parametrize("world,nx,ny,goal,engine_kw,obst", [
    (2, 257, 300, (250, 3), dict(kernel=5, prio_target=8), 0.03),
    (3, 300, 420, (150, 200), dict(kernel=5, prio_target=16), 0.03),   # goal in the middle
    (4, 512, 640, (40, 600), dict(kernel=5), 0.05),                     # 4 ranks, far goal
], ids=["w2", "w3-middle", "w4"])
def test_peer_loop_across_processes_matches_oracle(dymu, oracle, world, nx, ny, goal, engine_kw,
                                                   obst):
    _run(oracle, world, nx, ny, goal, engine_kw, transport="peer", obst=obst)


@pytest.mark.parametrize("bad_kind", ["slab", "nx", "k1"])
def test_peer_preflight_rejects_on_every_rank(dymu, oracle, bad_kind):
    """The peer transport's pre-flight (the same board as IPC): a rank-local error
    fails every rank with DYMU_ERR_ARG; the following solves reset the receive rows
    and match the oracle.  "k1": every rank asks for K = 1, which the peer transport's
    fused rounds cannot run -- rejected before any collective state changes, so the
    communicator survives (it used to abort every later solve)."""
    _run(oracle, 3, 160, 200, (80, 100), dict(kernel=5, prio_target=8), bad_rank=1,
         bad_kind=bad_kind, transport="peer")
