"""GPU parity of the device computeCostMap pre-pass (SURVEY s8(f)1,
dymu_compute_cost_map / dymu_pack_speed) against the CPU oracle's restatement
of reference src/DyMu_GlobalPathPlanning.cpp:145-308 (quirks Q1-Q4).

Exact: terrain classes, obstacle flags, locomotion modes, +inf mask of F.
Tolerance 1e-13 relative on slope / raw_cost / cost / F: the device atan
(ocml) may differ from glibc's in the last ulp.  Downstream,
the total-cost map from the device F matches the oracle FMM within the engine
tolerance 1e-12."""
import numpy as np
import pytest

from gen_golden import terrain_inputs
from test_gpu_solver import assert_parity

pytestmark = pytest.mark.gpu

RTOL = 1e-13

FIELDS = {"cost": np.float64, "raw_cost": np.float64, "slope": np.float64,
          "terrain": np.uint32, "is_obstacle": np.uint8, "hazard": np.float64,
          "traff": np.float64, "loc_mode": np.int32}


class DeviceState:
    """The planner node fields as device arrays (pitch ld >= nx)."""

    def __init__(self, eng, nx, ny, ld, host_state):
        self.eng, self.nx, self.ny, self.ld = eng, nx, ny, ld
        self.ptr = {}
        for f, dt in FIELDS.items():
            self.ptr[f] = eng.alloc(np.dtype(dt).itemsize * ny * ld)
            self.put(f, host_state[f])

    def put(self, f, a):
        buf = np.zeros((self.ny, self.ld), dtype=FIELDS[f])
        buf[:, :self.nx] = a
        self.eng.h2d(self.ptr[f], buf)

    def get(self, f):
        buf = np.empty((self.ny, self.ld), dtype=FIELDS[f])
        self.eng.d2h(buf, self.ptr[f])
        return buf[:, :self.nx].copy()

    def free(self):
        for p in self.ptr.values():
            self.eng.free(p)


def upload(eng, a, ld):
    ny, nx = a.shape
    buf = np.zeros((ny, ld))
    buf[:, :nx] = a
    p = eng.alloc(8 * ny * ld)
    eng.h2d(p, buf)
    return p


def close(a, b, rtol=RTOL):
    fin = np.isfinite(b)
    assert np.array_equal(np.isfinite(a), fin)
    err = np.abs(a[fin] - b[fin]) / np.maximum(1.0, np.abs(b[fin]))
    return err.max(initial=0.0) <= rtol, err.max(initial=0.0)


def case_inputs(name, N, rng):
    j, i = np.mgrid[0:N, 0:N].astype(np.float64)
    if name == "config2":  # 3 terrains x 1 mode x 5 slopes
        elev, terr, lut, slopes = terrain_inputs(N)
        return elev, terr, lut, slopes, 1
    if name == "multiloc":  # 3 terrains x 3 modes x 4 slopes, rough terrain (obstacles by slope)
        elev = 4.0 * np.sin(0.11 * i) * np.cos(0.09 * j) + rng.normal(0, 0.15, (N, N))
        terr = rng.integers(1, 3, (N, N)).astype(np.float64)
        lut = np.concatenate([np.full(12, 50.0), rng.uniform(1, 8, 24)])
        slopes = np.array([0.0, 10.0, 20.0, 30.0])
        return elev, terr, lut, slopes, 3
    if name == "range1":  # Q4: one slope value, LUT terrain*numLocs + i
        elev = 0.01 * i
        terr = rng.integers(1, 4, (N, N)).astype(np.float64)
        lut = np.concatenate([np.full(2, 9.0), rng.uniform(1, 5, 6)])
        return elev, terr, lut, np.array([0.0]), 2
    raise KeyError(name)


@pytest.mark.parametrize("name,nx,ny,ld,res", [
    ("config2", 160, 128, 160, 0.5),
    ("multiloc", 131, 97, 136, 1.0),
    ("range1", 64, 80, 64, 0.25),
])
def test_cost_map_matches_oracle(engine, oracle, name, nx, ny, ld, res):
    rng = np.random.default_rng(5)
    N = max(nx, ny)
    elev, terr, lut, slopes, n_locs = case_inputs(name, N, rng)
    elev, terr = elev[:ny, :nx].copy(), terr[:ny, :nx].copy()
    hst = oracle.new_state(nx, ny)
    dst = DeviceState(engine, nx, ny, ld, hst)
    dE, dTr = upload(engine, elev, ld), upload(engine, terr, ld)
    dF = engine.alloc(8 * ny * ld)
    try:
        for call in range(2):  # the second call compounds the smoothing (Q1)
            oracle.compute_cost_map(hst, res, lut, slopes, n_locs, elev, terr)
            engine.compute_cost_map(nx, ny, ld, res, lut, slopes, n_locs, dE, dTr, dst.ptr, dF)
            for f in ("terrain", "is_obstacle", "loc_mode", "hazard", "traff"):
                assert np.array_equal(dst.get(f), hst[f]), (call, f)
            for f in ("slope", "raw_cost", "cost"):
                ok, err = close(dst.get(f), hst[f])
                assert ok, (call, f, err)
            Fd = np.empty((ny, ld))
            engine.d2h(Fd, dF)
            Fh = oracle.pack_speed(hst["cost"], hst["hazard"], hst["traff"], hst["is_obstacle"],
                                   res=res)
            ok, err = close(Fd[:, :nx], Fh)
            assert ok, (call, "F", err)
        # downstream: the total-cost map of the device F
        g = (nx * 3 // 4, ny * 3 // 4)
        if hst["is_obstacle"][g[1], g[0]]:
            pytest.skip("goal on an obstacle for this draw")
        dT = engine.alloc(8 * ny * ld)
        try:
            engine.solve_device(dF, dT, nx, ny, ld, g[0], g[1])
            T = np.empty((ny, ld))
            engine.d2h(T, dT)
            Tref, _ = oracle.fmm(Fh, g)
            assert_parity(T[:, :nx], Tref)
        finally:
            engine.free(dT)
    finally:
        for p in (dE, dTr, dF):
            engine.free(p)
        dst.free()


def test_pack_speed_after_feedback(engine, oracle):
    """Hazard / trafficability feedback (LocalPathRepairing.cpp:264-274,
    :389-394) re-packed on the device equals the host packing bit-for-bit."""
    nx, ny = 96, 70
    rng = np.random.default_rng(9)
    hst = oracle.new_state(nx, ny)
    hst["cost"][:] = rng.uniform(1, 5, (ny, nx))
    hst["hazard"][:] = np.minimum(1.0, rng.uniform(0, 1.5, (ny, nx)))
    hst["traff"][:] = rng.uniform(0, 1, (ny, nx))
    hst["is_obstacle"][:] = rng.uniform(0, 1, (ny, nx)) < 0.03
    dst = DeviceState(engine, nx, ny, nx, hst)
    dF = engine.alloc(8 * nx * ny)
    try:
        engine.pack_speed(nx, ny, nx, 0.7, dst.ptr, dF)
        Fd = np.empty((ny, nx))
        engine.d2h(Fd, dF)
        Fh = oracle.pack_speed(hst["cost"], hst["hazard"], hst["traff"], hst["is_obstacle"],
                               res=0.7)
        assert np.array_equal(Fd, Fh)
    finally:
        engine.free(dF)
        dst.free()


def test_terrain_beyond_lut_is_obstacle(engine, oracle):
    """Terrain classes past the LUT (out-of-bounds reads in the reference) become
    obstacles instead of faulting."""
    nx = ny = 32
    hst = oracle.new_state(nx, ny)
    dst = DeviceState(engine, nx, ny, nx, hst)
    elev = np.zeros((ny, nx))
    terr = np.ones((ny, nx))
    terr[10, 10] = 7.0
    terr[11, 12] = -3.0
    lut = np.array([9.0, 9.0, 1.0, 2.0])  # 2 terrains x 1 mode x 2 slopes
    dE, dTr = upload(engine, elev, nx), upload(engine, terr, nx)
    try:
        engine.compute_cost_map(nx, ny, nx, 1.0, lut, [0.0, 10.0], 1, dE, dTr, dst.ptr)
        obs = dst.get("is_obstacle")
        assert obs[10, 10] == 1 and obs[11, 12] == 1 and obs[5, 5] == 0
        assert obs[0].all() and obs[:, 0].all()  # border forced to terrain 0 (:162-163)
    finally:
        engine.free(dE)
        engine.free(dTr)
        dst.free()


def test_cost_map_rejects_bad_args(engine, dymu):
    with pytest.raises(dymu.DymuError):
        engine.compute_cost_map(1, 8, 1, 1.0, [1.0], [0.0], 1, 0, 0,
                                {f: 0 for f in FIELDS})
