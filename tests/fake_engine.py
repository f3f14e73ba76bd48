"""CPU stand-in for dymu.Engine's dom_* primitives (TEST INFRASTRUCTURE).

Lets the gloo world_size>1 tests drive dymu.sharded.SlabSolver -- the real
multi-rank orchestration (partition, boundary-row exchange, ghost merge,
termination) -- without a GPU.  The local relaxation is a vectorised numpy
Jacobi of the reference update (:500-546); its fixed point is the one the HIP
kernels reach, so the gathered result must equal the oracle FMM."""
import ctypes

import numpy as np

INF = np.inf


def _view(ptr, n):
    return np.ctypeslib.as_array((ctypes.c_double * n).from_address(ptr))


def eikonal_np(tx, ty, c):
    d = tx - ty
    two = (np.abs(d) < c) & (tx < INF) & (ty < INF)
    with np.errstate(invalid="ignore", over="ignore"):
        r = 2 * (c * c) - d * d
        u2 = (tx + ty + np.sqrt(np.where(two, r, 0.0))) / 2
    u1 = np.minimum(tx, ty) + c
    return np.where(two, u2, u1)


_M64 = (1 << 64) - 1


def _splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return x ^ (x >> np.uint64(31))


def synth_rows(n, row0, nrows, seed=1, obst_frac=0.0, obst_seed=3, goal=(0, 0)):
    """Rows [row0, row0+nrows) of the synthetic config-3 speed: numpy
    restatement of k_synth (fim_kernels.hip) / oracle synth_speed -- U(1,5) from
    splitmix64(seed ^ k), obstacles where splitmix64(obst_seed ^ k) < obst_frac, the
    goal's 3x3 kept free."""
    with np.errstate(over="ignore"):
        j = np.arange(row0, row0 + nrows, dtype=np.uint64)[:, None]
        i = np.arange(n, dtype=np.uint64)[None, :]
        k = j * np.uint64(n) + i
        u = (_splitmix64(np.uint64(seed) ^ k) >> np.uint64(11)).astype(np.float64) * 2.0**-53
        F = 1.0 + 4.0 * u
        if obst_frac > 0:
            u2 = (_splitmix64(np.uint64(obst_seed) ^ k) >> np.uint64(11)).astype(np.float64)
            ob = u2 * 2.0**-53 < obst_frac
            near = (np.abs(i.astype(np.int64) - goal[0]) <= 1) & \
                (np.abs(j.astype(np.int64) - goal[1]) <= 1)
            F[ob & ~near] = np.inf
    return F


class FakeEngine:
    def dom_begin(self, F, T, nx, nrows, ld, ghost_lo, ghost_hi, goal_i, goal_j_local,
                  stream=0):
        self.nx, self.nrows, self.lo, self.hi = nx, nrows, ghost_lo, ghost_hi
        self.F = _view(F, nrows * ld).reshape(nrows, ld)[:, :nx]
        base = T - 8 * ld
        self.Tb = _view(base, (nrows + 2) * ld).reshape(nrows + 2, ld)[:, :nx]
        self.Tb[:] = INF
        if goal_j_local >= 0:
            self.Tb[goal_j_local + 1, goal_i] = 0.0
        self.dirty = goal_j_local >= 0
        self.passes = 0

    def dom_run(self, passes, stream=0):
        for _ in range(passes):
            if not self.dirty:
                return
            T = self.Tb
            own = T[1:-1]
            south = T[:-2].copy()
            north = T[2:].copy()
            if not self.lo:
                south[0] = INF
            if not self.hi:
                north[-1] = INF
            west = np.full_like(own, INF)
            east = np.full_like(own, INF)
            west[:, 1:] = own[:, :-1]
            east[:, :-1] = own[:, 1:]
            u = eikonal_np(np.minimum(west, east), np.minimum(north, south), self.F)
            imp = u < own
            own[imp] = u[imp]
            self.dirty = bool(imp.any())
            self.passes += 1

    def dom_merge_ghosts(self, new_lo=0, new_hi=0, pending=0, stream=0):
        if new_lo:
            v = _view(new_lo, self.nx)
            m = v < self.Tb[0]
            self.Tb[0][m] = v[m]
            self.dirty |= bool(m.any())
        if new_hi:
            v = _view(new_hi, self.nx)
            m = v < self.Tb[-1]
            self.Tb[-1][m] = v[m]
            self.dirty |= bool(m.any())
        if pending:
            ctypes.c_int32.from_address(pending).value = 1 if self.dirty else 0

    def dom_finish(self, stream=0):
        return {"passes": self.passes, "tile_visits": 0, "inner_sweeps": 0}
