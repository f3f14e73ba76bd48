"""Row-slab domains on ONE GPU ("virtual slabs"): S engines,
each owning a slab with ghost rows, exchanging boundary rows through the host
until no slab has queued tiles.  The stitched map must equal the oracle FMM,
i.e. the sharded fixed point is the single-GPU one."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def solve_virtual_slabs(dymu, F, goal, S, K=8, **engine_kw):
    ny, nx = F.shape
    slabs = []
    for s in range(S):
        row0, nrows = dymu.slab_rows(ny, S, s)
        eng = dymu.Engine(**engine_kw)
        dF = eng.alloc(8 * nrows * nx)
        dT = eng.alloc(8 * (nrows + 2) * nx)
        stage = eng.alloc(16 * nx)
        eng.h2d(dF, np.ascontiguousarray(F[row0:row0 + nrows]))
        lo, hi = s > 0, s < S - 1
        gl = goal[1] - row0 if row0 <= goal[1] < row0 + nrows else -1
        eng.dom_begin(dF, dT + 8 * nx, nx, nrows, nx, lo, hi, goal[0] if gl >= 0 else 0, gl)
        slabs.append(dict(eng=eng, row0=row0, nrows=nrows, dF=dF, dT=dT, stage=stage, lo=lo,
                          hi=hi))
    rounds = 0
    row = np.empty(nx)
    while True:
        rounds += 1
        for sl in slabs:
            sl["eng"].dom_run(K)
        # boundary rows out (first / last owned rows), into neighbours' staging
        for s, sl in enumerate(slabs):
            e = sl["eng"]
            if sl["lo"]:
                e.d2h(row, sl["dT"] + 8 * nx)              # my first owned row
                slabs[s - 1]["eng"].h2d(slabs[s - 1]["stage"] + 8 * nx, row)   # their hi stage
            if sl["hi"]:
                e.d2h(row, sl["dT"] + 8 * nx * sl["nrows"])  # my last owned row
                slabs[s + 1]["eng"].h2d(slabs[s + 1]["stage"], row)            # their lo stage
        pending = 0
        for sl in slabs:
            sl["eng"].dom_merge_ghosts(sl["stage"] if sl["lo"] else 0,
                                       sl["stage"] + 8 * nx if sl["hi"] else 0, 0)
            pending += sl["eng"].dom_pending()
        if pending == 0 or rounds > 100000:
            break
    T = np.empty((ny, nx))
    for sl in slabs:
        buf = np.empty((sl["nrows"], nx))
        sl["eng"].d2h(buf, sl["dT"] + 8 * nx)
        T[sl["row0"]:sl["row0"] + sl["nrows"]] = buf
        sl["eng"].dom_finish()
        for k in ("dF", "dT", "stage"):
            sl["eng"].free(sl[k])
        sl["eng"].close()
    return T, rounds


@pytest.mark.parametrize("S,nx,ny,goal,frac", [(2, 200, 160, (100, 40), 0.02),
                                               (3, 130, 200, (7, 190), 0.05),
                                               (4, 256, 256, (128, 128), 0.0)])
@pytest.mark.parametrize("kw", [dict(kernel=3), dict(kernel=4, prio_target=32),
                                dict(kernel=5, prio_target=8)], ids=["fim", "prio", "prio16"])
def test_virtual_slabs_match_oracle(dymu, oracle, S, nx, ny, goal, frac, kw):
    F = oracle.synth_speed(nx, ny, seed=31, obst_frac=frac, obst_seed=5, goal=goal)
    T, rounds = solve_virtual_slabs(dymu, F, goal, S, **kw)
    Tref, _ = oracle.fmm(F, goal)
    assert np.array_equal(np.isinf(T), np.isinf(Tref))
    fin = np.isfinite(Tref)
    assert (np.abs(T[fin] - Tref[fin]) / np.maximum(1, Tref[fin])).max() <= 1e-12
    assert rounds > 1


def solve_vdist(dymu, F, goal, S, K=8, **engine_kw):
    """The native C++ sharded loop (libdymu_dist, dymu_vdist_solve): S slabs on
    one GPU, device-to-device row exchange, lagged termination check."""
    from dymu import dist

    ny, nx = F.shape
    engs, dFs, dTs, geo = [], [], [], []
    for s in range(S):
        row0, nrows = dymu.slab_rows(ny, S, s)
        eng = dymu.Engine(**engine_kw)
        dF = eng.alloc(8 * nrows * nx)
        dT = eng.alloc(8 * (nrows + 2) * nx)
        eng.h2d(dF, np.ascontiguousarray(F[row0:row0 + nrows]))
        engs.append(eng)
        dFs.append(dF)
        dTs.append(dT)
        geo.append((row0, nrows))
    stats = dist.vdist_solve(engs, dFs, dTs, nx, nx, ny, goal[0], goal[1], K)
    T = np.empty((ny, nx))
    for eng, dF, dT, (row0, nrows) in zip(engs, dFs, dTs, geo):
        buf = np.empty((nrows, nx))
        eng.d2h(buf, dT + 8 * nx)
        T[row0:row0 + nrows] = buf
        eng.free(dF)
        eng.free(dT)
        eng.close()
    return T, stats


@pytest.mark.parametrize("S,nx,ny,goal,frac,K", [(1, 96, 80, (10, 70), 0.02, 4),
                                                 (2, 200, 160, (100, 40), 0.02, 8),
                                                 (3, 130, 200, (7, 190), 0.05, 3),
                                                 (4, 256, 256, (128, 128), 0.0, 16),
                                                 (5, 64, 320, (32, 0), 0.03, 1)])
@pytest.mark.parametrize("kw", [dict(kernel=3), dict(kernel=5, prio_target=8)],
                         ids=["fim", "prio16"])
def test_native_vdist_matches_oracle(dymu, oracle, S, nx, ny, goal, frac, K, kw):
    F = oracle.synth_speed(nx, ny, seed=37, obst_frac=frac, obst_seed=9, goal=goal)
    T, stats = solve_vdist(dymu, F, goal, S, K=K, **kw)
    Tref, _ = oracle.fmm(F, goal)
    assert np.array_equal(np.isinf(T), np.isinf(Tref))
    fin = np.isfinite(Tref)
    assert (np.abs(T[fin] - Tref[fin]) / np.maximum(1, Tref[fin])).max() <= 1e-12
    assert len(stats) == S and all(st["rounds"] == stats[0]["rounds"] for st in stats)
    assert stats[0]["rounds"] >= 2  # at least the converged round + the lagged one


def test_native_vdist_large_matches_single(dymu):
    """4096^2 in 2 slabs with the default kernel choice (kernel 5 slabs): the
    stitched slabs equal the single-GPU solve's fixed point (both within ulps
    of each other)."""
    N, g = 4096, (700, 1500)
    eng = dymu.Engine()
    dF, dT = eng.alloc(8 * N * N), eng.alloc(8 * N * N)
    eng.synth_speed(dF, N, N, N, 0, 1, 0.02, 3, g[0], g[1])
    F = np.empty((N, N))
    eng.d2h(F, dF)
    eng.solve_device(dF, dT, N, N, N, g[0], g[1])
    T1 = np.empty((N, N))
    eng.d2h(T1, dT)
    eng.free(dF)
    eng.free(dT)
    eng.close()
    T, stats = solve_vdist(dymu, F, g, 2, K=4)
    assert stats[0]["kernel"] == 5
    assert np.array_equal(np.isinf(T), np.isinf(T1))
    fin = np.isfinite(T1)
    assert (np.abs(T[fin] - T1[fin]) / np.maximum(1, T1[fin])).max() <= 1e-12
