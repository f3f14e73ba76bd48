"""GPU parity tests of the HIP block-FIM engine through the C-ABI
(libdymu_fim.so: dymu_solve / dymu_solve_device) against the CPU oracle.

Tolerance: identical +inf mask and
|T_gpu - T_ref| <= 1e-12 * max(1, T_ref).  The reference FMM and the FIM fixed
point differ only at ulp level (measured <= 2.2e-15 relative)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-12


def assert_parity(T, Tref):
    inf_g, inf_r = np.isinf(T), np.isinf(Tref)
    assert np.array_equal(inf_g, inf_r), f"inf mask differs at {np.argwhere(inf_g != inf_r)[:5]}"
    fin = ~inf_r
    err = np.abs(T[fin] - Tref[fin]) / np.maximum(1.0, Tref[fin])
    assert err.max(initial=0.0) <= RTOL, f"max rel err {err.max()}"
    return err.max(initial=0.0)


def test_kat_mt19937_256(kengine, oracle):
    """SURVEY s8(c) KAT: reference sum(getTotalCostMatrix)=1.7066083890e+07,
    T[1][1]=479.2433625750 at N=256."""
    N = 256
    F = oracle.mt_uniform(N * N).reshape(N, N)
    r = kengine.solve(F, N // 2, N // 2)
    M = np.where(np.isinf(r.T), -1.0, r.T)
    assert f"{M.sum():.10e}" == "1.7066083890e+07"
    assert f"{r.T[1, 1]:.10f}" == "479.2433625750"
    Tref, _ = oracle.fmm(F, (N // 2, N // 2))
    assert_parity(r.T, Tref)


@pytest.mark.parametrize("N", [512, 1024])
def test_kat_mt19937(kengine, oracle, N):
    kat = {512: ("1.3467278246e+08", "972.7322452271"),
           1024: ("1.0666255888e+09", "1913.6136177798")}[N]
    F = oracle.mt_uniform(N * N).reshape(N, N)
    r = kengine.solve(F, N // 2, N // 2)
    M = np.where(np.isinf(r.T), -1.0, r.T)
    assert f"{M.sum():.10e}" == kat[0]
    assert f"{r.T[1, 1]:.10f}" == kat[1]


@pytest.mark.parametrize("nx,ny,frac,goal", [
    (64, 64, 0.0, (32, 32)),
    (128, 96, 0.02, (10, 80)),
    (33, 65, 0.05, (1, 1)),          # ragged tiles, goal near the corner
    (1, 1, 0.0, (0, 0)),             # single cell
    (1, 300, 0.0, (0, 150)),         # one column
    (300, 1, 0.0, (299, 0)),         # one row
    (257, 129, 0.10, (128, 64)),
    (500, 700, 0.25, (250, 350)),    # dense obstacles, disconnected pockets
])
def test_parity_random(kengine, oracle, nx, ny, frac, goal):
    F = oracle.synth_speed(nx, ny, seed=7, obst_frac=frac, obst_seed=11, goal=goal)
    r = kengine.solve(F, goal[0], goal[1])
    Tref, _ = oracle.fmm(F, goal)
    assert_parity(r.T, Tref)
    assert r.T[goal[1], goal[0]] == 0.0


@pytest.mark.parametrize("exact", [1, 0])
def test_constant_speed_closed_form(dymu, exact):
    """C=1: T on the axes equals the distance, T(+-1,+-1) = 1 + sqrt(2)/2 (:533) --
    bit for bit with the correctly rounded sweep sqrt (exact_sqrt=1), within the
    default candidate's 36-ulp bound otherwise."""
    N = 65
    F = np.ones((N, N))
    eng = dymu.Engine(exact_sqrt=exact)
    try:
        r = eng.solve(F, 32, 32)
    finally:
        eng.close()
    T = r.T
    for k in range(1, 20):
        assert T[32, 32 + k] == float(k) and T[32 - k, 32] == float(k)
    v = 1.0 + np.sqrt(2.0) / 2.0
    for dj, di in ((1, 1), (-1, 1), (1, -1), (-1, -1)):
        if exact:
            assert T[32 + dj, 32 + di] == v
        else:
            assert abs(T[32 + dj, 32 + di] - v) <= 36 * np.spacing(v)


def test_device_resident_and_synth(engine, oracle):
    """dymu_synth_speed on device == host generator; dymu_solve_device == oracle."""
    nx, ny, g = 384, 320, (200, 100)
    n = nx * ny
    dF = engine.alloc(8 * n)
    dT = engine.alloc(8 * n)
    try:
        engine.synth_speed(dF, nx, ny, nx, 0, 1, 0.02, 3, g[0], g[1])
        Fd = np.empty((ny, nx))
        engine.d2h(Fd, dF)
        Fh = oracle.synth_speed(nx, ny, seed=1, obst_frac=0.02, obst_seed=3, goal=g)
        assert np.array_equal(Fd, Fh)
        st = engine.solve_device(dF, dT, nx, ny, nx, g[0], g[1])
        T = np.empty((ny, nx))
        engine.d2h(T, dT)
        Tref, _ = oracle.fmm(Fh, g)
        assert_parity(T, Tref)
        assert st["passes"] > 0 and st["tile_visits"] >= st["passes"]
    finally:
        engine.free(dF)
        engine.free(dT)


def test_repeat_solves_reuse_context(kengine, oracle):
    """Epoch-stamped tile flags and priority keys survive across solves of
    different sizes."""
    for (nx, ny, g) in [(200, 200, (100, 100)), (64, 300, (3, 5)), (200, 200, (20, 180)),
                        (700, 500, (10, 490))]:
        F = oracle.synth_speed(nx, ny, seed=5, obst_frac=0.03, obst_seed=9, goal=g)
        r = kengine.solve(F, g[0], g[1])
        Tref, _ = oracle.fmm(F, g)
        assert_parity(r.T, Tref)


def test_priority_kernel_defers(dymu, oracle):
    """Kernel 4 with a small target relaxes fewer tiles than plain FIM and
    reaches the same map; the stats report which kernel ran."""
    nx = ny = 1024
    g = (512, 512)
    F = oracle.synth_speed(nx, ny, seed=2, obst_frac=0.02, obst_seed=4, goal=g)
    out = {}
    for k, kw in ((3, {}), (4, dict(prio_target=256)), (5, dict(prio_target=64))):
        eng = dymu.Engine(kernel=k, **kw)
        try:
            out[k] = eng.solve(F, g[0], g[1])
        finally:
            eng.close()
    assert [out[k].stats["kernel"] for k in (3, 4, 5)] == [3, 4, 5]
    assert out[4].stats["tile_visits"] < out[3].stats["tile_visits"]
    Tref, _ = oracle.fmm(F, g)
    for k in (3, 4, 5):
        assert_parity(out[k].T, Tref)


def test_auto_kernel_choice(dymu):
    """kernel=0 picks the 16x16 priority passes at every size (the checkerboard
    made them the faster kernel down to 256^2); kernel=3 still selects plain FIM."""
    eng = dymu.Engine()
    try:
        r = eng.solve(np.ones((64, 64)), 3, 3)
        assert r.stats["kernel"] == 5 and r.stats["tile_w"] == 16
        r = eng.solve(np.ones((2900, 2900)), 3, 3)
        assert r.stats["kernel"] == 5 and r.stats["tile_w"] == 16
        assert r.T[3, 13] == 10.0  # on the axis through the goal: the distance
    finally:
        eng.close()
    for k in (1, 2, 6, 7, -1):  # only 0 (auto) and 3-5 exist (kernels 1/2 were removed)
        with pytest.raises(dymu.DymuError):
            dymu.Engine(kernel=k)


def test_bad_args(engine, dymu):
    F = np.ones((8, 8))
    with pytest.raises(dymu.DymuError):
        engine.solve(F, 8, 0)


@pytest.mark.parametrize("fast", [True, False])
def test_update_arithmetic_bit_exact(engine, oracle, fast):
    """Every single update is bit-identical to the reference formula (:531-535)
    evaluated on the host (SSE2, no contraction): 2M random (Tx, Ty, C),
    including the one-sided, two-sided and infinite cases."""
    rng = np.random.default_rng(7)
    n = 1 << 21
    c = np.exp(rng.uniform(np.log(1e-3), np.log(1e3), n))
    tx = rng.uniform(0, 1e4, n)
    ty = tx + rng.normal(0, 1, n) * c  # many |Tx-Ty| < C (two-sided) cases
    ty = np.abs(ty)
    tx[::97] = np.inf
    ty[::89] = np.inf
    c[::101] = 1.0 + rng.uniform(0, 1e-12, c[::101].size)
    out = engine.eikonal_batch(tx, ty, c, fast=fast)
    ref = np.array([oracle.eikonal(a, b, cc) for a, b, cc in zip(tx[:200000], ty[:200000],
                                                                  c[:200000])])
    assert np.array_equal(out[:200000], ref)
    # vectorised reference for the rest (same op order, numpy is IEEE double)
    with np.errstate(invalid="ignore"):  # inf - inf in the unused branch
        d = tx - ty
        two = (np.abs(d) < c) & np.isfinite(tx) & np.isfinite(ty)
        r = np.where(two, (tx + ty + np.sqrt(2 * (c * c) - d * d)) / 2, np.minimum(tx, ty) + c)
    assert np.array_equal(out, r)


@pytest.mark.parametrize("fast", [2, 3, 4])
def test_update_arithmetic_approx_sqrt(engine, fast):
    """Kernel 5's sweep candidates: 2 = the default (monotone combine min + h,
    one Goldschmidt step after v_rsq_f64, the branch folded into h's argument
    min(|d|, C)), 3 = exact_sqrt (monotone combine, correctly rounded sqrt), 4 =
    v31's combine (two_sided_approx).  Each is within 40 ulp of the reference
    formula's candidate (the sqrt term within 36 ulp, tools/sqrt_probe.hip; the
    monotone combine rounds once where the reference rounds twice, <= 1 ulp apart),
    i.e. <= 1e-14 relative; with the correctly rounded sqrt within 2 ulp.  The
    infinite cases are identical; the one-sided ones bit for bit for 3 and 4, and
    for 2 (whose one-sided h is the approximate sqrt of ~C^2) within the same bound."""
    rng = np.random.default_rng(11)
    n = 1 << 21
    c = np.exp(rng.uniform(np.log(1e-3), np.log(1e3), n))
    tx = rng.uniform(0, 1e4, n)
    ty = np.abs(tx + rng.normal(0, 1, n) * c)
    tx[::97] = np.inf
    ty[::89] = np.inf
    out = engine.eikonal_batch(tx, ty, c, fast=fast)
    with np.errstate(invalid="ignore"):
        d = tx - ty
        two = (np.abs(d) < c) & np.isfinite(tx) & np.isfinite(ty)
        q = np.sqrt(2 * (c * c) - d * d)
        r = np.where(two, (tx + ty + q) / 2, np.minimum(tx, ty) + c)
    fin = np.isfinite(r)
    assert np.array_equal(np.isfinite(out), fin)
    chk = fin if fast == 2 else two
    if fast != 2:
        assert np.array_equal(out[~two], r[~two])
    ulps = 2 if fast == 3 else 40
    assert np.all(np.abs(out[chk] - r[chk]) <= ulps * np.spacing(r[chk]))
    assert np.max(np.abs(out[chk] - r[chk]) / r[chk]) <= 1e-14


def test_update_monotone_combine(engine):
    """The monotone combine (DESIGN.md s4 "Monotone combine"): raising Tx or Ty by
    one ulp almost never lowers the candidate, where the reference's two roundings
    at the scale of T -- RN(RN(Tx + Ty) + sqrt) / 2 -- lower it in a few percent of
    the two-sided cases.  That non-monotonicity is what the FIM's min over history
    turns into a bias along long paths (the 16384^2 maze, tests/test_gpu_maze.py)."""
    rng = np.random.default_rng(5)
    n = 1 << 20
    c = np.exp(rng.uniform(np.log(1e-1), np.log(1e1), n))
    tx = rng.uniform(0, 1e4, n)
    ty = np.abs(tx + rng.normal(0, 0.5, n) * c)
    two = np.abs(tx - ty) < c
    rate = {}
    for fast in (True, 4, 2, 3):
        a = engine.eikonal_batch(tx, ty, c, fast=fast)
        bx = engine.eikonal_batch(np.nextafter(tx, np.inf), ty, c, fast=fast)
        by = engine.eikonal_batch(tx, np.nextafter(ty, np.inf), c, fast=fast)
        rate[fast] = float(((bx < a) | (by < a))[two].mean())
    assert rate[True] > 0.01  # the reference arithmetic (kernels 3/4)
    assert rate[3] <= 1e-4, rate
    assert rate[2] <= rate[True] / 10, rate


def test_exact_sqrt_option(dymu, oracle):
    """dymu_opts.exact_sqrt = 1 (kernel 5 with the correctly rounded sweep sqrt)
    and the default both meet the parity bar on the same grid."""
    N = 1024
    F = oracle.synth_speed(N, N, seed=5, obst_frac=0.02, obst_seed=9, goal=(300, 700))
    Tref, _ = oracle.fmm(F, (300, 700))
    for ex in (0, 1):
        eng = dymu.Engine(kernel=5, exact_sqrt=ex)
        try:
            assert_parity(eng.solve(F, 300, 700).T, Tref)
        finally:
            eng.close()


def test_sampled_pass_timing(dymu, oracle):
    """dymu_set_profiling(period) times every period-th pass launch."""
    nx = ny = 512
    F = oracle.synth_speed(nx, ny, seed=3, obst_frac=0.02, obst_seed=5, goal=(256, 256))
    eng = dymu.Engine()
    try:
        eng.set_profiling(4)
        r = eng.solve(F, 256, 256)
        ms, n = eng.last_pass_timing()
        L = r.stats["launches"]
        assert n == (L + 3) // 4 and ms > 0.0
        eng.set_profiling(0)
        eng.solve(F, 256, 256)
        assert eng.last_pass_timing() == (0.0, 0)
        with pytest.raises(dymu.DymuError):
            eng.set_profiling(-1)
    finally:
        eng.close()


def serpentine_maze(F, period=64, offset=32):
    """SURVEY s8(d) config-3 stress variant: 1-cell walls every `period` rows,
    each with one gap, alternating between the left and the right end."""
    F = F.copy()
    ny, nx = F.shape
    for k, j in enumerate(range(offset, ny, period)):
        F[j, :] = np.inf
        F[j, 1 if k % 2 == 0 else nx - 2] = 2.0
    return F


@pytest.mark.parametrize("N,period", [(256, 16), (384, 32)])
def test_parity_serpentine_maze(kengine, oracle, N, period):
    g = (N // 2, N // 2 + 4)
    F = serpentine_maze(oracle.synth_speed(N, N, seed=9, obst_frac=0.01, obst_seed=2, goal=g),
                        period, period // 2)
    r = kengine.solve(F, *g)
    Tref, _ = oracle.fmm(F, g)
    assert_parity(r.T, Tref)
    assert r.stats["passes"] > 4 * N // (r.stats["tile_w"] * 2)  # the maze inflates the passes


@pytest.mark.parametrize("capfrac", ["0", "0.5", "0.9"])
def test_list_fraction_cap_same_fixed_point(dymu, oracle, monkeypatch, capfrac):
    """Kernel 5's per-pass target capped at a fraction of the active list
    (DYMU_PRIO_CAPFRAC; 0.9 by default, 0 = off) changes the schedule, not the map:
    the open grid and a serpentine maze (short lists, where the cap binds) both
    match the oracle FMM."""
    monkeypatch.setenv("DYMU_PRIO_CAPFRAC", capfrac)
    N, g = 320, (160, 164)
    F0 = oracle.synth_speed(N, N, seed=21, obst_frac=0.02, obst_seed=22, goal=g)
    eng = dymu.Engine(kernel=5, prio_target=64)
    try:
        for F in (F0, serpentine_maze(F0, 32, 16)):
            r = eng.solve(F, *g)
            Tref, _ = oracle.fmm(F, g)
            assert_parity(r.T, Tref)
    finally:
        eng.close()


@pytest.mark.parametrize("pack", ["0", "1"])
def test_packed_key_bins_same_fixed_point(dymu, oracle, monkeypatch, pack):
    """Kernel 5's list entries with (DYMU_PACK_BINS=1, default) and without their
    first-insertion key bin: the bin only moves the key gate before the tile loads, so
    the open grid and a serpentine maze (many key-deferred entries, re-queued without a
    bin by the capped visits) both reach the oracle's fixed point, with a small
    per-pass target so that the threshold binds."""
    monkeypatch.setenv("DYMU_PACK_BINS", pack)
    N, g = 384, (100, 250)
    F0 = oracle.synth_speed(N, N, seed=41, obst_frac=0.02, obst_seed=42, goal=g)
    eng = dymu.Engine(kernel=5, prio_target=16)
    try:
        for F in (F0, serpentine_maze(F0, 48, 16)):
            r = eng.solve(F, *g)
            Tref, _ = oracle.fmm(F, g)
            assert_parity(r.T, Tref)
            assert r.stats["deferred"] > 0
    finally:
        eng.close()


@pytest.mark.parametrize("mode", ["0", "1", "2"])
@pytest.mark.parametrize("kernel", [3, 5])
def test_convergence_check_modes(dymu, oracle, monkeypatch, mode, kernel):
    """DYMU_PIPELINE 0 (read-back after each batch), 1 (batch posts to the
    mailbox) and 2 (per-pass posts, 4 passes queued; the default) end on the
    same fixed point; the empty passes queued after convergence change nothing
    and are counted as launches, not passes (DESIGN.md s4 "Convergence checks")."""
    monkeypatch.setenv("DYMU_PIPELINE", mode)
    nx, ny, g = 640, 512, (100, 400)
    F = oracle.synth_speed(nx, ny, seed=12, obst_frac=0.04, obst_seed=13, goal=g)
    eng = dymu.Engine(kernel=kernel, prio_target=64 if kernel == 5 else 0)
    try:
        rs = [eng.solve(F, g[0], g[1]) for _ in range(2)]
    finally:
        eng.close()
    Tref, _ = oracle.fmm(F, g)
    for r in rs:
        assert_parity(r.T, Tref)
        assert r.stats["kernel"] == kernel
        assert r.stats["launches"] >= r.stats["passes"] > 0
        if mode == "2":  # at most the 4 queued-ahead passes run empty
            assert r.stats["launches"] <= r.stats["passes"] + 4 + 1


@pytest.mark.parametrize("mode", ["0", "2"])
def test_early_exit_modes(dymu, oracle, monkeypatch, mode):
    """dymu_solve_until_device with the batch read-back (0) and with the in-kernel
    probe posted every pass (2): the start and its nb4 are final when it returns,
    t_closed is their largest value, and every cell <= t_closed holds the oracle
    FMM value; the per-pass probe stops within the 4 queued passes of the first
    pass that sees them final."""
    monkeypatch.setenv("DYMU_PIPELINE", mode)
    N, g = 1024, (512, 512)
    F = oracle.synth_speed(N, N, seed=3, obst_frac=0.02, obst_seed=5, goal=g)
    Tref, _ = oracle.fmm(F, g)
    eng = dymu.Engine(kernel=5, prio_target=64)
    dF, dT = eng.alloc(8 * N * N), eng.alloc(8 * N * N)
    try:
        eng.h2d(dF, F)
        for s in ((g[0] + 3, g[1] + 2), (g[0] + 200, g[1] - 100), (1, 1)):
            tc, st = eng.solve_until_device(dF, dT, N, N, N, g[0], g[1], s[0], s[1])
            T = np.empty((N, N))
            eng.d2h(T, dT)
            cells = [(s[0] + di, s[1] + dj) for di, dj in ((0, 0), (1, 0), (-1, 0), (0, 1), (0, -1))
                     if 0 <= s[0] + di < N and 0 <= s[1] + dj < N]
            want = max(Tref[j, i] for i, j in cells)
            assert abs(tc - want) <= RTOL * max(1.0, want)
            closed = T <= tc
            assert all(closed[j, i] for i, j in cells)
            err = np.abs(T[closed] - Tref[closed]) / np.maximum(1.0, Tref[closed])
            assert err.max() <= RTOL
            assert st["passes"] > 0
    finally:
        eng.free(dF)
        eng.free(dT)
        eng.close()


def test_deterministic_mode_bit_reproducible(dymu, oracle):
    """dymu_opts.deterministic: checkerboard passes, no sweep deadline -- two
    contexts and two solves each give bit-identical maps, within the tolerance of
    the oracle; the default schedule reaches the same fixed point."""
    nx, ny, g = 1024, 768, (300, 500)
    F = oracle.synth_speed(nx, ny, seed=21, obst_frac=0.03, obst_seed=22, goal=g)
    maps, stats = [], []
    for _ in range(2):
        eng = dymu.Engine(deterministic=1, prio_target=64)
        try:
            for _ in range(2):
                r = eng.solve(F, g[0], g[1])
                maps.append(r.T)
                stats.append(r.stats)
        finally:
            eng.close()
    for T in maps[1:]:
        assert np.array_equal(T.view(np.uint64), maps[0].view(np.uint64))
    assert all(st["kernel"] == 5 for st in stats)
    assert len({(st["passes"], st["tile_visits"], st["inner_sweeps"]) for st in stats}) == 1
    Tref, _ = oracle.fmm(F, g)
    assert_parity(maps[0], Tref)


def test_deterministic_mode_large_grid(dymu):
    """At 8192^2 the default run uses the sweep deadline; deterministic mode drops
    it and repeats bit for bit (device-resident solve)."""
    N, g = 8192, (4096, 4096)
    eng = dymu.Engine(deterministic=1)
    dF, dT = eng.alloc(8 * N * N), eng.alloc(8 * N * N)
    try:
        eng.synth_speed(dF, N, N, N, 0, 1, 0.02, 3, g[0], g[1])
        outs = []
        for _ in range(2):
            st = eng.solve_device(dF, dT, N, N, N, g[0], g[1])
            T = np.empty((N, N))
            eng.d2h(T, dT)
            outs.append((T, st))
        assert np.array_equal(outs[0][0].view(np.uint64), outs[1][0].view(np.uint64))
        assert outs[0][1]["passes"] == outs[1][1]["passes"]
    finally:
        eng.free(dF)
        eng.free(dT)
        eng.close()


@pytest.mark.parametrize("checker", ["0", "1"])
def test_checkerboard_on_off(dymu, oracle, monkeypatch, checker):
    """Kernel 5 with and without checkerboard passes (DYMU_CHECKER) reaches the
    oracle's fixed point; the checkerboard relaxes fewer tiles."""
    monkeypatch.setenv("DYMU_CHECKER", checker)
    nx, ny, g = 768, 640, (200, 300)
    F = oracle.synth_speed(nx, ny, seed=31, obst_frac=0.03, obst_seed=32, goal=g)
    eng = dymu.Engine(kernel=5, prio_target=64)
    try:
        r = eng.solve(F, g[0], g[1])
    finally:
        eng.close()
    Tref, _ = oracle.fmm(F, g)
    assert_parity(r.T, Tref)
    assert r.stats["kernel"] == 5 and r.stats["tile_visits"] > 0


def test_plain_fim_kernel_still_selectable(dymu, oracle):
    """dymu_opts.kernel = 3 (plain block FIM, 8x8 tiles) remains a parity-green choice."""
    F = oracle.synth_speed(300, 200, seed=41, obst_frac=0.03, obst_seed=42, goal=(20, 150))
    eng = dymu.Engine(kernel=3)
    try:
        r = eng.solve(F, 20, 150)
    finally:
        eng.close()
    assert r.stats["kernel"] == 3 and r.stats["tile_w"] == 8
    Tref, _ = oracle.fmm(F, (20, 150))
    assert_parity(r.T, Tref)
