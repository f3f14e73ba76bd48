"""ctypes binding of oracle/build/liboracle.so (TEST INFRASTRUCTURE ONLY).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker; never by the product path.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ODIR = os.path.join(ROOT, "oracle")
_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_u32, _u64, _i64, _d, _vp = (ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int64, ctypes.c_double,
                             ctypes.c_void_p)

_SIGS = {
    "oracle_fill_mt19937_uniform": (None, [_dp, _u64, _u64, _d, _d]),
    "oracle_u01": (_d, [_u64, _u64]),
    "oracle_fill_u01": (None, [_dp, _u64, _u64]),
    "oracle_pack_speed": (None, [_dp, _vp, _vp, _vp, _u64, _d, _dp]),
    "oracle_set_cost_map": (None, [_dp, _u64, _dp, _u8p, _dp, _dp]),
    "oracle_compute_cost_map": (None, [_u32, _u32, _d, _dp, ctypes.c_int, _dp, ctypes.c_int,
                                       ctypes.c_int, _dp, _dp, _dp, _dp, _dp, _u32p, _u8p, _dp,
                                       _dp, _i32p]),
    "oracle_set_goal": (ctypes.c_int, [_u32, _u32, _d, _d, _d, _d, _d, _vp,
                                       ctypes.POINTER(_u32), ctypes.POINTER(_u32)]),
    "oracle_eikonal": (_d, [_d, _d, _d]),
    "oracle_fmm_linear": (ctypes.c_int, [_dp, _u32, _u32, _u32, _u32, _i64, _i64, _dp, _vp,
                                         ctypes.POINTER(_u64)]),
    "oracle_fmm_heap": (ctypes.c_int, [_dp, _u32, _u32, _u32, _u32, _i64, _i64, _dp, _vp,
                                       ctypes.POINTER(_u64)]),
    "oracle_fmm_order": (ctypes.c_int, [_dp, _u32, _u32, _u32, _u32, _i64, _i64, _dp, _vp,
                                        np.ctypeslib.ndpointer(dtype=np.uint64,
                                                               flags="C_CONTIGUOUS")]),
    "oracle_jacobi": (ctypes.c_int, [_dp, _u32, _u32, _u32, _u32, _dp, ctypes.c_int]),
    "oracle_fim_parallel": (ctypes.c_int, [_dp, _u32, _u32, _u32, _u32, _dp, ctypes.c_int,
                                           ctypes.POINTER(_u64)]),
    "oracle_residual": (_d, [_dp, _dp, _u32, _u32, _u32, _u32, ctypes.POINTER(_u64)]),
    "oracle_total_cost_matrix": (None, [_dp, _u64, _dp]),
    "oracle_global_path": (ctypes.c_int, [_dp, _vp, _u32, _u32, _d, _u32, _u32, _d, _d, _d, _d,
                                          _d, _dp, ctypes.c_int]),
    "oracle_local_create": (_vp, [_u32, _u32, _d, _d, _d, _d, _d, _d, _d, ctypes.c_int]),
    "oracle_local_destroy": (None, [_vp]),
    "oracle_local_set_global": (None, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _d]),
    "oracle_local_get_global": (None, [_vp, _vp, _vp]),
    "oracle_local_set_path": (None, [_vp, _vp, ctypes.c_int]),
    "oracle_local_get_path": (ctypes.c_int, [_vp, _vp, ctypes.c_int]),
    "oracle_local_reconnecting_index": (ctypes.c_int, [_vp]),
    "oracle_local_planning": (ctypes.c_int, [_vp, _d, _d, _d, _d, _vp, _u32, _u32, _u32, _u32,
                                             _d]),
    "oracle_local_get_path_eval": (ctypes.c_int, [_vp, _d, _d, _d, _d, _vp, ctypes.c_int]),
    "oracle_local_risk_matrix": (None, [_vp, _d, _d, _vp]),
    "oracle_local_deviation_matrix": (None, [_vp, _d, _d, _vp]),
    "oracle_local_map_mask": (_u64, [_vp, _vp]),
    "oracle_local_block": (ctypes.c_int, [_vp, _u32, _u32, _vp, _vp, _vp, _vp, _vp]),
    "oracle_local_list": (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_int]),
    "oracle_local_max_risk_node": (ctypes.c_int, [_vp, _vp]),
    "oracle_local_propagate_risk_at": (ctypes.c_int, [_vp, _d, _d]),
    "oracle_local_propagate_local_at": (ctypes.c_int, [_vp, _d, _d]),
    "oracle_local_set_state_at": (ctypes.c_int, [_vp, _d, _d, ctypes.c_int]),
    "oracle_local_min_cost": (ctypes.c_int, [_vp, _d, _d, _vp]),
    "oracle_local_expand_risk": (None, [_vp]),
}


class OracleLocal:
    """The local-layer restatement (oracle/oracle_local.c) over a copy of a
    global layer: obstacle flags, total cost T (+inf unreachable), the CLOSED
    state (default: finite T), elevation, hazard / trafficability, goal."""

    def __init__(self, lib, nx, ny, gres, lres, offset=(0.0, 0.0), risk_distance=1.0,
                 reconnect_distance=1.0, risk_ratio=1.0, approach=0):
        self.lib = lib
        self.nx, self.ny = nx, ny
        self.r = int(gres / lres)
        self.off = offset
        self.h = lib.oracle_local_create(nx, ny, gres, lres, offset[0], offset[1], risk_distance,
                                         reconnect_distance, risk_ratio, approach)

    def close(self):
        if self.h:
            self.lib.oracle_local_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    @staticmethod
    def _p(a, dt):
        if a is None:
            return None, None
        a = np.ascontiguousarray(a, dtype=dt)
        return a, a.ctypes.data

    def set_global(self, obst, T, goal, goal_heading=0.0, closed=None, elev=None, hazard=None,
                   traff=None):
        if closed is None:
            closed = np.isfinite(T)
        keep = [self._p(obst, np.uint8), self._p(T, np.float64), self._p(closed, np.uint8),
                self._p(elev, np.float64), self._p(hazard, np.float64),
                self._p(traff, np.float64)]
        self.lib.oracle_local_set_global(self.h, *[k[1] for k in keep], goal[0], goal[1],
                                         goal_heading)

    def hazard_traff(self):
        hd = np.empty((self.ny, self.nx))
        tr = np.empty((self.ny, self.nx))
        self.lib.oracle_local_get_global(self.h, hd.ctypes.data, tr.ctypes.data)
        return hd, tr

    @property
    def path(self):
        n = self.lib.oracle_local_get_path(self.h, None, 0)
        buf = np.empty(4 * max(n, 1))
        self.lib.oracle_local_get_path(self.h, buf.ctypes.data, n)
        return buf[:4 * n].reshape(-1, 4).copy()

    @path.setter
    def path(self, wps):
        a = np.ascontiguousarray(np.asarray(wps, dtype=np.float64).reshape(-1, 4))
        self.lib.oracle_local_set_path(self.h, a.ctypes.data, len(a))

    def reconnecting_index(self):
        return self.lib.oracle_local_reconnecting_index(self.h)

    def local_planning(self, w, image, res):
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, wd = img.shape[:2]
        ps = img.shape[2] if img.ndim == 3 else 1
        w = tuple(w) + (0.0,) * (4 - len(w))
        r = self.lib.oracle_local_planning(self.h, w[0], w[1], w[2], w[3], img.ctypes.data, wd, h,
                                           wd * ps, ps, res)
        return bool(r), (self.path if r else np.empty((0, 4)))

    def get_path(self, w):
        w = tuple(w) + (0.0,) * (4 - len(w))
        n = self.lib.oracle_local_get_path_eval(self.h, w[0], w[1], w[2], w[3], None, 0)
        p = self.path
        p[:, 0] += self.off[0]
        p[:, 1] += self.off[1]
        return n, p

    def _window(self, fn, x, y):
        ls = 21 * self.r
        out = np.empty((ls, ls))
        fn(self.h, x, y, out.ctypes.data)
        return out

    def risk_matrix(self, x, y):
        return self._window(self.lib.oracle_local_risk_matrix, x, y)

    def deviation_matrix(self, x, y):
        return self._window(self.lib.oracle_local_deviation_matrix, x, y)

    def map_mask(self):
        m = np.zeros((self.ny, self.nx), dtype=np.uint8)
        self.lib.oracle_local_map_mask(self.h, m.ctypes.data)
        return m

    # per-node steps and the public lists (5 doubles per node: global x, global y,
    # deviation, total cost, risk)
    def node_list(self, which):
        n = self.lib.oracle_local_list(self.h, which, None, 0)
        out = np.empty((max(n, 1), 5))
        self.lib.oracle_local_list(self.h, which, out.ctypes.data, n)
        return out[:n]

    def max_risk_node(self):
        out = np.empty(5)
        return out if self.lib.oracle_local_max_risk_node(self.h, out.ctypes.data) else None

    def propagate_risk(self, x, y):
        return bool(self.lib.oracle_local_propagate_risk_at(self.h, x, y))

    def propagate_local(self, x, y):
        return bool(self.lib.oracle_local_propagate_local_at(self.h, x, y))

    def set_state(self, x, y, closed):
        return bool(self.lib.oracle_local_set_state_at(self.h, x, y, 1 if closed else 0))

    def min_cost(self, reach=None):
        out = np.empty(5)
        rx, ry = reach if reach is not None else (float("nan"), 0.0)
        return out if self.lib.oracle_local_min_cost(self.h, rx, ry, out.ctypes.data) else None

    def expand_risk(self):
        self.lib.oracle_local_expand_risk(self.h)

    def block(self, i, j):
        r = self.r
        dev, tc, risk = (np.empty((r, r)) for _ in range(3))
        st, ob = (np.empty((r, r), dtype=np.uint8) for _ in range(2))
        if not self.lib.oracle_local_block(self.h, i, j, dev.ctypes.data, tc.ctypes.data,
                                           risk.ctypes.data, st.ctypes.data, ob.ctypes.data):
            return None
        return dev, tc, risk, st, ob


class Oracle:
    def __init__(self, lib):
        self.lib = lib

    # generators
    def mt_uniform(self, n, seed=1, lo=1.0, hi=5.0):
        out = np.empty(n, dtype=np.float64)
        self.lib.oracle_fill_mt19937_uniform(out, n, seed, lo, hi)
        return out

    def u01(self, n, seed):
        out = np.empty(n, dtype=np.float64)
        self.lib.oracle_fill_u01(out, n, seed)
        return out

    def synth_speed(self, nx, ny, seed=1, obst_frac=0.0, obst_seed=3, goal=(0, 0)):
        """Host twin of dymu_synth_speed."""
        n = nx * ny
        F = 1.0 + 4.0 * self.u01(n, seed)
        if obst_frac > 0:
            o = self.u01(n, obst_seed) < obst_frac
            o = o.reshape(ny, nx)
            gi, gj = goal
            o[max(gj - 1, 0):gj + 2, max(gi - 1, 0):gi + 2] = False
            F = F.reshape(ny, nx)
            F[o] = np.inf
        return F.reshape(ny, nx)

    def fim_parallel(self, F, goal, threads=4):
        """All-cores block FIM (oracle_par.c): (T, passes)."""
        F = np.ascontiguousarray(F, dtype=np.float64)
        ny, nx = F.shape
        T = np.empty_like(F)
        passes = _u64()
        rc = self.lib.oracle_fim_parallel(F, nx, ny, goal[0], goal[1], T, threads,
                                          ctypes.byref(passes))
        assert rc == 0
        return T, passes.value

    def fmm(self, F, goal, start=None, linear=False, want_closed=False):
        F = np.ascontiguousarray(F, dtype=np.float64)
        ny, nx = F.shape
        T = np.empty_like(F)
        closed = np.zeros((ny, nx), dtype=np.uint8) if want_closed else None
        pops = _u64()
        si, sj = (start if start is not None else (-1, -1))
        fn = self.lib.oracle_fmm_linear if linear else self.lib.oracle_fmm_heap
        rc = fn(F, nx, ny, goal[0], goal[1], si, sj, T,
                closed.ctypes.data if closed is not None else None, ctypes.byref(pops))
        if rc < 0:
            raise ValueError("oracle fmm: bad args")
        if want_closed:
            return T, rc, closed
        return T, rc

    def fmm_order(self, F, goal, start=None):
        """The reference FMM (heap, the linear scan's pop order): T, the return code,
        the CLOSED mask and each node's band-insertion sequence (uint64 max = never)."""
        F = np.ascontiguousarray(F, dtype=np.float64)
        ny, nx = F.shape
        T = np.empty_like(F)
        closed = np.zeros((ny, nx), dtype=np.uint8)
        seq = np.empty((ny, nx), dtype=np.uint64)
        si, sj = (start if start is not None else (-1, -1))
        rc = self.lib.oracle_fmm_order(F, nx, ny, goal[0], goal[1], si, sj, T,
                                       closed.ctypes.data, seq)
        if rc < 0:
            raise ValueError("oracle fmm: bad args")
        return T, rc, closed, seq

    def jacobi(self, F, goal, max_sweeps=1 << 30):
        F = np.ascontiguousarray(F, dtype=np.float64)
        ny, nx = F.shape
        T = np.empty_like(F)
        sweeps = self.lib.oracle_jacobi(F, nx, ny, goal[0], goal[1], T, max_sweeps)
        return T, sweeps

    def residual(self, F, T, goal):
        F = np.ascontiguousarray(F, dtype=np.float64)
        T = np.ascontiguousarray(T, dtype=np.float64)
        ny, nx = F.shape
        cnt = _u64()
        r = self.lib.oracle_residual(F, T, nx, ny, goal[0], goal[1], ctypes.byref(cnt))
        return r, cnt.value

    def eikonal(self, tx, ty, c):
        return self.lib.oracle_eikonal(tx, ty, c)

    def pack_speed(self, cost, hazard=None, traff=None, is_obstacle=None, res=1.0):
        cost = np.ascontiguousarray(cost, dtype=np.float64)
        F = np.empty_like(cost)
        keep = []

        def ptr(a, dt):
            if a is None:
                return None
            a = np.ascontiguousarray(a, dtype=dt)
            keep.append(a)
            return a.ctypes.data

        self.lib.oracle_pack_speed(cost.ravel(), ptr(hazard, np.float64), ptr(traff, np.float64),
                                   ptr(is_obstacle, np.uint8), cost.size, res, F.ravel())
        return F

    def set_goal(self, nx, ny, res, off, w, is_obstacle=None):
        gi, gj = _u32(), _u32()
        obs = None
        if is_obstacle is not None:
            is_obstacle = np.ascontiguousarray(is_obstacle, dtype=np.uint8)
            obs = is_obstacle.ctypes.data
        ok = self.lib.oracle_set_goal(nx, ny, res, off[0], off[1], w[0], w[1], obs,
                                      ctypes.byref(gi), ctypes.byref(gj))
        return (gi.value, gj.value) if ok else None

    def compute_cost_map(self, state, res, lut, slopes, n_locs, elevation, terrain_map):
        """state: dict of planner SoA arrays (mutated in place, carries Q1 state)."""
        ny, nx = elevation.shape
        lut = np.ascontiguousarray(lut, dtype=np.float64)
        slopes = np.ascontiguousarray(slopes, dtype=np.float64)
        self.lib.oracle_compute_cost_map(
            nx, ny, res, lut, len(lut), slopes, len(slopes), n_locs,
            np.ascontiguousarray(elevation, dtype=np.float64).ravel(),
            np.ascontiguousarray(terrain_map, dtype=np.float64).ravel(),
            state["raw_cost"].ravel(), state["cost"].ravel(), state["slope"].ravel(),
            state["terrain"].ravel(), state["is_obstacle"].ravel(), state["traff"].ravel(),
            state["hazard"].ravel(), state["loc_mode"].ravel())

    @staticmethod
    def new_state(nx, ny):
        return {
            "raw_cost": np.zeros((ny, nx)), "cost": np.zeros((ny, nx)),
            "slope": np.zeros((ny, nx)), "terrain": np.zeros((ny, nx), dtype=np.uint32),
            "is_obstacle": np.zeros((ny, nx), dtype=np.uint8),
            "traff": np.ones((ny, nx)), "hazard": np.zeros((ny, nx)),
            "loc_mode": np.full((ny, nx), -1, dtype=np.int32),
        }

    def global_path(self, T, goal, res=1.0, start=(0.0, 0.0, 0.0), risk_distance=1.0,
                    goal_heading=0.0, elev=None, max_wp=1 << 20):
        T = np.ascontiguousarray(T, dtype=np.float64)
        ny, nx = T.shape
        wp = np.empty(4 * max_wp, dtype=np.float64)
        e = None
        if elev is not None:
            elev = np.ascontiguousarray(elev, dtype=np.float64)
            e = elev.ctypes.data
        n = self.lib.oracle_global_path(T, e, nx, ny, res, goal[0], goal[1], goal_heading,
                                        risk_distance, start[0], start[1], start[2], wp, max_wp)
        if n < 0:
            return n, None
        return n, wp[:4 * n].reshape(n, 4).copy()

    def local(self, nx, ny, gres, lres, **kw):
        return OracleLocal(self.lib, nx, ny, gres, lres, **kw)


_cached = None


def load():
    global _cached
    if _cached is None:
        path = os.path.join(ODIR, "build", "liboracle.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-s"], cwd=ODIR, check=True)
        lib = ctypes.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _cached = Oracle(lib)
    return _cached
