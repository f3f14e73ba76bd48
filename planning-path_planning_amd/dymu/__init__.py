"""dymu -- Python binding of the MI355X DyMu total-cost propagation engine.

Thin ctypes layer over the two in-tree shared libraries:

* ``lib/libdymu_fim.so``     -- HIP kernels + C-ABI (include/dymu_fim.h)
* ``lib/libdymu_planner.so`` -- host C++ ``PathPlanning_lib::DyMuPathPlanner``
                                (include/DyMu.hpp) behind include/dymu_planner.h
* ``lib/libdymu_dist.so``    -- row-slab sharded solve over RCCL
                                (include/dymu_dist.h; binding in dymu.dist)

There is no CPU fallback: if the HIP library is missing or no device is
visible, every entry point raises ``DymuError``.  The CPU oracle under
``oracle/`` is test infrastructure and is never imported from here.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# DYMU_LIBDIR: load the libraries from another directory (A/B builds)
_LIBDIR = os.environ.get("DYMU_LIBDIR") or os.path.normpath(os.path.join(_HERE, "..", "lib"))

DYMU_OK = 0
_ERRS = {
    -1: "invalid argument",
    -2: "HIP runtime error",
    -3: "device out of memory",
    -4: "pass cap reached before convergence",
    -5: "no HIP device",
    -6: "RCCL error",
    -7: "call out of sequence",
}


class DymuError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"dymu status {status} ({_ERRS.get(status, 'unknown')}) {what}".strip())


class DymuOpts(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int),
        ("passes_per_check", ctypes.c_int),
        ("max_passes", ctypes.c_int),
        ("max_inner", ctypes.c_int),
        ("grid_blocks", ctypes.c_int),
        ("kernel", ctypes.c_int),
        ("prio_target", ctypes.c_int),
        ("exact_sqrt", ctypes.c_int),
        ("deterministic", ctypes.c_int),
    ]


class DymuDomain(ctypes.Structure):
    _fields_ = [
        ("F", ctypes.c_void_p),
        ("T", ctypes.c_void_p),
        ("ld", ctypes.c_uint64),
        ("nx", ctypes.c_uint32),
        ("nrows", ctypes.c_uint32),
        ("ghost_lo", ctypes.c_int32),
        ("ghost_hi", ctypes.c_int32),
    ]


class DymuCostState(ctypes.Structure):
    """dymu_cost_state: device pointers of the planner node fields."""
    FIELDS = ("cost", "raw_cost", "slope", "terrain", "is_obstacle", "hazard", "traff",
              "loc_mode")
    _fields_ = [(f, ctypes.c_void_p) for f in FIELDS]


class DymuRegion(ctypes.Structure):
    _fields_ = [("i0", ctypes.c_uint32), ("j0", ctypes.c_uint32), ("i1", ctypes.c_uint32),
                ("j1", ctypes.c_uint32), ("n_range", ctypes.c_uint64), ("r_const", ctypes.c_double)]


class DymuStats(ctypes.Structure):
    _fields_ = [
        ("passes", ctypes.c_uint64),
        ("launches", ctypes.c_uint64),
        ("tile_visits", ctypes.c_uint64),
        ("inner_sweeps", ctypes.c_uint64),
        ("max_active", ctypes.c_uint64),
        ("rounds", ctypes.c_uint64),
        ("ms", ctypes.c_double),
        ("tile_w", ctypes.c_int),
        ("tile_h", ctypes.c_int),
        ("kernel", ctypes.c_int),
        ("reserved", ctypes.c_int),
        ("deferred", ctypes.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_u32, _u64, _i32, _vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p

# name -> (restype, argtypes)
FIM_SYMBOLS = {
    "dymu_create": (_i32, [ctypes.POINTER(_vp), ctypes.POINTER(DymuOpts)]),
    "dymu_destroy": (_i32, [_vp]),
    "dymu_solve": (_i32, [_vp, _dp, _u32, _u32, _u32, _u32, _dp, ctypes.POINTER(DymuStats)]),
    "dymu_solve_device": (_i32, [_vp, _vp, _vp, _u32, _u32, _u64, _u32, _u32, _vp,
                                 ctypes.POINTER(DymuStats)]),
    "dymu_synth_speed": (_i32, [_vp, _vp, _u32, _u32, _u64, _u64, _u64, ctypes.c_double, _u64,
                                _u32, _u32, _vp]),
    "dymu_device_alloc": (_i32, [_vp, ctypes.c_size_t, ctypes.POINTER(_vp)]),
    "dymu_device_free": (_i32, [_vp, _vp]),
    "dymu_memcpy_d2h": (_i32, [_vp, _vp, _vp, ctypes.c_size_t]),
    "dymu_memcpy_h2d": (_i32, [_vp, _vp, _vp, ctypes.c_size_t]),
    "dymu_set_profiling": (_i32, [_vp, _i32]),
    "dymu_set_pass_stats": (_i32, [_vp, _i32]),
    "dymu_last_update_stats": (_i32, [_vp, ctypes.POINTER(_u64)]),
    "dymu_last_pass_stats": (_i32, [_vp, _vp, _u64, ctypes.POINTER(_u64)]),
    "dymu_eikonal_batch": (_i32, [_vp, _vp, _vp, _vp, _vp, _u64, _i32]),
    "dymu_slab_rows": (_i32, [_u32, _u32, _u32, ctypes.POINTER(_u32), ctypes.POINTER(_u32)]),
    "dymu_dom_begin": (_i32, [_vp, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, _vp]),
    "dymu_dom_run": (_i32, [_vp, _u32, _vp]),
    "dymu_dom_merge_ghosts": (_i32, [_vp, _vp, _vp, _vp, _vp]),
    "dymu_dom_pending": (_i32, [_vp, _vp, ctypes.POINTER(_u64)]),
    "dymu_dom_exchange": (_i32, [_vp, _vp, _vp, _vp, _vp]),
    "dymu_dom_round_supported": (_i32, [_vp, _u32]),
    "dymu_dom_round_capable": (_i32, [_vp, _u32, _u32, _u32]),
    "dymu_dom_round": (_i32, [_vp, _u32, _vp, _vp, _vp, _vp]),
    "dymu_dom_round_peer": (_i32, [_vp, _u32, _vp, _vp]),
    "dymu_count_equal": (_i32, [_vp, _vp, _u32, _u32, _u64, ctypes.c_double,
                                ctypes.POINTER(_u64), _vp]),
    "dymu_find_equal": (_i32, [_vp, _vp, _u32, _u32, _u64, ctypes.c_double, _vp, _u64,
                               ctypes.POINTER(_u64), _vp]),
    "dymu_dom_post_status": (_i32, [_vp, _vp, _vp, _u32]),
    "dymu_dom_post": (_i32, [_vp, _vp, ctypes.POINTER(_u32)]),
    "dymu_dom_wait_post": (_i32, [_vp, _u32, ctypes.c_double, ctypes.POINTER(ctypes.c_int32),
                                  _vp]),
    "dymu_dom_finish": (_i32, [_vp, _vp, ctypes.POINTER(DymuStats)]),
    "dymu_last_pass_timing": (_i32, [_vp, ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_uint64)]),
    "dymu_compute_cost_map": (_i32, [_vp, _u32, _u32, _u64, ctypes.c_double, _dp, _i32, _dp,
                                     _i32, _i32, _vp, _vp, ctypes.POINTER(DymuCostState), _vp,
                                     _vp]),
    "dymu_pack_speed": (_i32, [_vp, _u32, _u32, _u64, ctypes.c_double,
                               ctypes.POINTER(DymuCostState), _vp, _vp]),
    "dymu_resolve_window_device": (_i32, [_vp, _vp, _vp, _u32, _u32, _u64, _u32, _u32, _u32,
                                          _u32, _u32, _u32, _vp, ctypes.POINTER(DymuStats)]),
    "dymu_update_window_device": (_i32, [_vp, _vp, _vp, _u32, _u32, _u64, _u32, _u32, _u32,
                                         _u32, _u32, _u32, _i32, _vp,
                                         ctypes.POINTER(DymuStats)]),
    "dymu_resolve_window": (_i32, [_vp, _dp, _u32, _u32, _u32, _u32, _u32, _u32, _u32, _u32,
                                   _dp, ctypes.POINTER(DymuStats)]),
    "dymu_solve_until_device": (_i32, [_vp, _vp, _vp, _u32, _u32, _u64, _u32, _u32, _u32, _u32,
                                       _vp, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(DymuStats)]),
    "dymu_early_exit_mask": (_i32, [_vp, _vp, _vp, _u32, _u32, _u64, ctypes.c_double, _vp, _u64,
                                    ctypes.POINTER(_u64), _vp]),
    "dymu_scatter": (_i32, [_vp, _vp, _u32, _u64, _vp, _vp, _u64, _vp]),
    "dymu_region_stats": (_i32, [_vp, _vp, _vp, _u32, _u32, _u64, _u32, _u32, ctypes.c_double,
                                 ctypes.c_double, ctypes.c_double, ctypes.POINTER(DymuRegion),
                                 _vp]),
    "dymu_memcpy2d_d2h": (_i32, [_vp, _vp, ctypes.c_size_t, _vp, ctypes.c_size_t,
                                 ctypes.c_size_t, ctypes.c_size_t]),
    "dymu_memcpy2d_h2d": (_i32, [_vp, _vp, ctypes.c_size_t, _vp, ctypes.c_size_t,
                                 ctypes.c_size_t, ctypes.c_size_t]),
    "dymu_host_register": (_i32, [_vp, _vp, ctypes.c_size_t]),
    "dymu_host_unregister": (_i32, [_vp, _vp]),
    "dymu_get_stream": (_vp, [_vp]),
    "dymu_strerror": (ctypes.c_char_p, [_i32]),
    "dymu_last_error": (ctypes.c_char_p, [_vp]),
    "dymu_abi_version": (_i32, []),
    "dymu_device_count": (_i32, []),
}

_fim = None


def lib_path(name: str) -> str:
    return os.path.join(_LIBDIR, name)


def load_fim() -> ctypes.CDLL:
    """Load libdymu_fim.so (RTLD_GLOBAL so the planner library resolves it)."""
    global _fim
    if _fim is None:
        path = lib_path("libdymu_fim.so")
        if not os.path.exists(path):
            raise DymuError(-5, f"HIP extension missing: {path} (run __graft_entry__.build())")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        ab_build = "DYMU_LIBDIR" in os.environ  # an older A/B build may lack newer symbols
        for name, (res, args) in FIM_SYMBOLS.items():
            if ab_build and not hasattr(lib, name):
                continue
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _fim = lib
    return _fim


def _check(rc: int, ctx=None):
    if rc != DYMU_OK:
        what = ""
        if ctx is not None:
            msg = load_fim().dymu_last_error(ctx)
            what = msg.decode() if msg else ""
        raise DymuError(rc, what)


@dataclass
class SolveResult:
    T: np.ndarray
    stats: dict


class Engine:
    """One HIP context (stream + workspace) on one device."""

    def __init__(self, device: int = -1, passes_per_check: int = 0, max_passes: int = 0,
                 max_inner: int = 0, grid_blocks: int = 0, kernel: int = 0,
                 prio_target: int = 0, exact_sqrt: int = 0, deterministic: int = 0):
        lib = load_fim()
        self._lib = lib
        opts = DymuOpts(device, passes_per_check, max_passes, max_inner, grid_blocks, kernel,
                        prio_target, exact_sqrt, deterministic)
        ctx = _vp()
        rc = lib.dymu_create(ctypes.byref(ctx), ctypes.byref(opts))
        if rc != DYMU_OK:
            raise DymuError(rc, "dymu_create")
        self.ctx = ctx

    def close(self):
        if getattr(self, "ctx", None):
            self._lib.dymu_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- host-buffer solve (planner path) --
    def solve(self, F: np.ndarray, goal_i: int, goal_j: int) -> SolveResult:
        F = np.ascontiguousarray(F, dtype=np.float64)
        if F.ndim != 2:
            raise ValueError("F must be 2-D [ny, nx]")
        ny, nx = F.shape
        T = np.empty_like(F)
        st = DymuStats()
        _check(self._lib.dymu_solve(self.ctx, F, nx, ny, goal_i, goal_j, T, ctypes.byref(st)),
               self.ctx)
        return SolveResult(T, st.as_dict())

    def resolve_window(self, F: np.ndarray, goal_i: int, goal_j: int, i0: int, j0: int, w: int,
                       h: int) -> SolveResult:
        """Windowed re-propagation after F changed inside [i0,i0+w) x [j0,j0+h);
        the previous solve on this engine must be of the same grid and goal."""
        F = np.ascontiguousarray(F, dtype=np.float64)
        ny, nx = F.shape
        T = np.empty_like(F)
        st = DymuStats()
        _check(self._lib.dymu_resolve_window(self.ctx, F, nx, ny, goal_i, goal_j, i0, j0, w, h, T,
                                             ctypes.byref(st)), self.ctx)
        return SolveResult(T, st.as_dict())

    def resolve_window_device(self, dF: int, dT: int, nx: int, ny: int, ld: int, goal_i: int,
                              goal_j: int, i0: int, j0: int, w: int, h: int,
                              stream: int = 0) -> dict:
        st = DymuStats()
        _check(self._lib.dymu_resolve_window_device(self.ctx, dF, dT, nx, ny, ld, goal_i, goal_j,
                                                    i0, j0, w, h, stream or None,
                                                    ctypes.byref(st)), self.ctx)
        return st.as_dict()

    def update_window_device(self, dF: int, dT: int, nx: int, ny: int, ld: int, goal_i: int,
                             goal_j: int, i0: int, j0: int, w: int, h: int,
                             decrease_only: bool, stream: int = 0) -> dict:
        st = DymuStats()
        _check(self._lib.dymu_update_window_device(self.ctx, dF, dT, nx, ny, ld, goal_i, goal_j,
                                                   i0, j0, w, h, int(bool(decrease_only)),
                                                   stream or None, ctypes.byref(st)), self.ctx)
        return st.as_dict()

    # -- device-resident solve --
    def solve_device(self, dF: int, dT: int, nx: int, ny: int, ld: int, goal_i: int,
                     goal_j: int, stream: int = 0) -> dict:
        st = DymuStats()
        _check(self._lib.dymu_solve_device(self.ctx, dF, dT, nx, ny, ld, goal_i, goal_j,
                                           stream or None, ctypes.byref(st)), self.ctx)
        return st.as_dict()

    def solve_until_device(self, dF: int, dT: int, nx: int, ny: int, ld: int, goal_i: int,
                           goal_j: int, start_i: int, start_j: int, stream: int = 0):
        """computeTotalCostMap's propagation: stops once the start and its nb4 are final.
        Returns (t_closed, stats)."""
        st = DymuStats()
        tc = ctypes.c_double()
        _check(self._lib.dymu_solve_until_device(self.ctx, dF, dT, nx, ny, ld, goal_i, goal_j,
                                                 start_i, start_j, stream or None,
                                                 ctypes.byref(tc), ctypes.byref(st)), self.ctx)
        return tc.value, st.as_dict()

    def synth_speed(self, dF: int, nx: int, ny: int, ld: int, row0: int = 0, seed: int = 1,
                    obst_frac: float = 0.0, obst_seed: int = 3, goal_i: int = 0,
                    goal_j: int = 0, stream: int = 0):
        _check(self._lib.dymu_synth_speed(self.ctx, dF, nx, ny, ld, row0, seed, obst_frac,
                                          obst_seed, goal_i, goal_j, stream or None), self.ctx)

    def find_equal(self, dT: int, nx: int, ny: int, ld: int, value: float, cap: int):
        """Cells whose value is bitwise `value` (dymu_find_equal): (count, indices of the
        first min(count, cap) of them, j * nx + i, in no particular order)."""
        idx = np.zeros(max(1, cap), dtype=np.uint64)
        n = _u64()
        _check(self._lib.dymu_find_equal(self.ctx, dT, nx, ny, ld, float(value), idx.ctypes.data,
                                         cap, ctypes.byref(n), None), self.ctx)
        return n.value, idx[:min(n.value, cap)]

    def scatter(self, dT: int, nx: int, ld: int, idx: np.ndarray, vals: np.ndarray):
        """T[idx // nx, idx % nx] = vals on the device (dymu_scatter)."""
        idx = np.ascontiguousarray(idx, dtype=np.uint64)
        vals = np.ascontiguousarray(vals, dtype=np.float64)
        if idx.shape != vals.shape:
            raise ValueError("idx and vals differ in shape")
        _check(self._lib.dymu_scatter(self.ctx, dT, nx, ld, idx.ctypes.data, vals.ctypes.data,
                                      idx.size, None), self.ctx)

    def region_stats(self, dF: int, dT: int, nx: int, ny: int, ld: int, goal_i: int,
                     goal_j: int, thr: float, lo: float, hi: float) -> dict:
        """dymu_region_stats: bounding box (inclusive) of the cells with T <= thr, the
        number with lo <= T <= hi, the distance from the goal to the nearest cell of
        another speed."""
        r = DymuRegion()
        _check(self._lib.dymu_region_stats(self.ctx, dF, dT, nx, ny, ld, goal_i, goal_j, thr, lo,
                                           hi, ctypes.byref(r), None), self.ctx)
        return {"box": (r.i0, r.j0, r.i1, r.j1), "n_range": r.n_range, "r_const": r.r_const}

    def alloc(self, nbytes: int) -> int:
        p = _vp()
        _check(self._lib.dymu_device_alloc(self.ctx, nbytes, ctypes.byref(p)), self.ctx)
        return p.value

    def free(self, p: int):
        _check(self._lib.dymu_device_free(self.ctx, p), self.ctx)

    def d2h(self, dst: np.ndarray, src: int):
        _check(self._lib.dymu_memcpy_d2h(self.ctx, dst.ctypes.data, src, dst.nbytes), self.ctx)

    def h2d(self, dst: int, src: np.ndarray):
        src = np.ascontiguousarray(src)
        _check(self._lib.dymu_memcpy_h2d(self.ctx, dst, src.ctypes.data, src.nbytes), self.ctx)

    # -- row-slab domain primitives (multi-GPU sharding, dymu.sharded) --
    def dom_begin(self, F: int, T: int, nx: int, nrows: int, ld: int, ghost_lo: bool,
                  ghost_hi: bool, goal_i: int, goal_j_local: int, stream: int = 0):
        d = DymuDomain(F, T, ld, nx, nrows, int(ghost_lo), int(ghost_hi))
        self._dom = d  # keep alive
        _check(self._lib.dymu_dom_begin(self.ctx, ctypes.addressof(d), goal_i, goal_j_local,
                                        stream or None), self.ctx)

    def dom_run(self, passes: int, stream: int = 0):
        _check(self._lib.dymu_dom_run(self.ctx, passes, stream or None), self.ctx)

    def dom_merge_ghosts(self, new_lo: int = 0, new_hi: int = 0, pending: int = 0,
                         stream: int = 0):
        _check(self._lib.dymu_dom_merge_ghosts(self.ctx, new_lo or None, new_hi or None,
                                               pending or None, stream or None), self.ctx)

    def dom_pending(self, stream: int = 0) -> int:
        n = ctypes.c_uint64()
        _check(self._lib.dymu_dom_pending(self.ctx, stream or None, ctypes.byref(n)), self.ctx)
        return n.value

    def dom_finish(self, stream: int = 0) -> dict:
        st = DymuStats()
        _check(self._lib.dymu_dom_finish(self.ctx, stream or None, ctypes.byref(st)), self.ctx)
        return st.as_dict()

    def eikonal_batch(self, tx: np.ndarray, ty: np.ndarray, c: np.ndarray,
                      fast=True) -> np.ndarray:
        """The kernels' update arithmetic on the GPU (bit-level self-test).
        fast: False = sqrt(), True = the correctly rounded sqrt in the reference's
        combine (kernels 3/4), 2 = kernel 5's default sweep candidate (monotone
        combine, approximate sqrt), 3 = kernel 5's exact_sqrt sweep candidate
        (monotone combine, correctly rounded sqrt), 4 = v31's sweep candidate."""
        arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (tx, ty, c)]
        n = arrs[0].size
        ptrs = [self.alloc(8 * n) for _ in range(4)]
        try:
            for p, a in zip(ptrs, arrs):
                self.h2d(p, a)
            _check(self._lib.dymu_eikonal_batch(self.ctx, ptrs[0], ptrs[1], ptrs[2], ptrs[3], n,
                                                fast if fast in (2, 3, 4) else 1 if fast else 0),
                   self.ctx)
            out = np.empty(n)
            self.d2h(out, ptrs[3])
            return out
        finally:
            for p in ptrs:
                self.free(p)

    # ---- computeCostMap on the device ----
    @staticmethod
    def cost_state(ptrs: dict) -> DymuCostState:
        """ptrs: field name -> device pointer (int), see DymuCostState.FIELDS."""
        return DymuCostState(*[ptrs[f] for f in DymuCostState.FIELDS])

    def compute_cost_map(self, nx, ny, ld, res, lut, slopes, n_locs, d_elev, d_terrain,
                         state: dict, dF=0, stream=0):
        lut = np.ascontiguousarray(lut, dtype=np.float64)
        slopes = np.ascontiguousarray(slopes, dtype=np.float64)
        st = self.cost_state(state)
        _check(self._lib.dymu_compute_cost_map(self.ctx, nx, ny, ld, res, lut, len(lut), slopes,
                                               len(slopes), n_locs, d_elev, d_terrain,
                                               ctypes.byref(st), dF or None, stream or None),
               self.ctx)

    def pack_speed(self, nx, ny, ld, res, state: dict, dF, stream=0):
        st = self.cost_state(state)
        _check(self._lib.dymu_pack_speed(self.ctx, nx, ny, ld, res, ctypes.byref(st), dF,
                                         stream or None), self.ctx)

    def set_profiling(self, period):
        """Time every `period`-th pass launch (True = every launch, 0/False = off)."""
        _check(self._lib.dymu_set_profiling(self.ctx, int(period)), self.ctx)

    PASS_STAT_FIELDS = ("listed", "visited", "colour_deferred", "key_deferred", "capped",
                        "deadline", "radius_max", "sweeps", "bstar", "radius_min", "enqueued")

    def last_update_stats(self) -> dict:
        """The last windowed update's raise front (dymu_last_update_stats)."""
        out = (_u64 * 4)()
        _check(self._lib.dymu_last_update_stats(self.ctx, out), self.ctx)
        return {"raise_passes": out[0], "raise_visits": out[1], "cells_invalidated": out[2]}

    def set_pass_stats(self, on=True):
        """Kernel 5 per-pass statistics for the next solves (diagnostics)."""
        _check(self._lib.dymu_set_pass_stats(self.ctx, int(bool(on))), self.ctx)

    def last_pass_stats(self) -> np.ndarray:
        """(passes, 12) uint32 records of the last solve (fields: PASS_STAT_FIELDS)."""
        n = _u64()
        cap = 1 << 14
        out = np.zeros((cap, 12), dtype=np.uint32)
        _check(self._lib.dymu_last_pass_stats(self.ctx, out.ctypes.data, cap, ctypes.byref(n)),
               self.ctx)
        return out[:n.value].copy()

    def last_pass_timing(self):
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        _check(self._lib.dymu_last_pass_timing(self.ctx, ctypes.byref(ms), ctypes.byref(n)),
               self.ctx)
        return ms.value, n.value


def slab_rows(ny: int, nranks: int, rank: int):
    """(row0, nrows) of `rank`'s row slab (boundaries on multiples of 32 rows)."""
    r0, n = ctypes.c_uint32(), ctypes.c_uint32()
    _check(load_fim().dymu_slab_rows(ny, nranks, rank, ctypes.byref(r0), ctypes.byref(n)))
    return r0.value, n.value


def device_count() -> int:
    return load_fim().dymu_device_count()


# ---------------------------------------------------------------------------
# host planner: PathPlanning_lib::DyMuPathPlanner behind include/dymu_planner.h
# ---------------------------------------------------------------------------
_d = ctypes.c_double
PLANNER_SYMBOLS = {
    "dymu_planner_create": (_i32, [ctypes.POINTER(_vp), _d, _d, _d, _i32]),
    "dymu_planner_destroy": (None, [_vp]),
    "dymu_planner_set_engine_options": (_i32, [_vp, ctypes.POINTER(DymuOpts)]),
    "dymu_planner_init_global_layer": (_i32, [_vp, _d, _d, _u32, _u32, _d, _d]),
    "dymu_planner_set_cost_map": (_i32, [_vp, _dp, _u32, _u32]),
    "dymu_planner_compute_cost_map": (_i32, [_vp, _dp, _i32, _dp, _i32,
                                             ctypes.POINTER(ctypes.c_char_p), _i32, _dp, _dp]),
    "dymu_planner_set_goal": (_i32, [_vp, _d, _d, _d, _d]),
    "dymu_planner_compute_total_cost_map": (_i32, [_vp, _d, _d, _d, _d]),
    "dymu_planner_compute_entire_total_cost_map": (_i32, [_vp]),
    "dymu_planner_get_total_cost_matrix": (_i32, [_vp, _dp]),
    "dymu_planner_get_global_cost_matrix": (_i32, [_vp, _dp]),
    "dymu_planner_get_hazard_density_matrix": (_i32, [_vp, _dp]),
    "dymu_planner_get_trafficability_matrix": (_i32, [_vp, _dp]),
    "dymu_planner_get_total_cost_raw": (_i32, [_vp, _dp]),
    "dymu_planner_get_total_cost": (_i32, [_vp, _d, _d, _d, _d, ctypes.POINTER(_d)]),
    "dymu_planner_get_path": (_i32, [_vp, _d, _d, _d, _d, _dp, _i32]),
    "dymu_planner_get_locomotion_mode": (_i32, [_vp, _d, _d, _d, _d, ctypes.c_char_p, _i32]),
    "dymu_planner_set_hazard_density": (_i32, [_vp, _dp]),
    "dymu_planner_set_trafficability": (_i32, [_vp, _dp]),
    "dymu_planner_last_stats": (_i32, [_vp, ctypes.POINTER(DymuStats)]),
    "dymu_planner_last_solve_kind": (_i32, [_vp]),
    "dymu_planner_last_early_exit": (_i32, [_vp, _dp]),
    "dymu_planner_last_early_exit_ex": (_i32, [_vp, _vp, _u32]),
    "dymu_planner_get_node_states": (_i32, [_vp, _vp]),
    "dymu_planner_set_hazard_density_window": (_i32, [_vp, _u32, _u32, _u32, _u32, _dp]),
    "dymu_planner_set_trafficability_window": (_i32, [_vp, _u32, _u32, _u32, _u32, _dp]),
    "dymu_planner_last_band_size": (ctypes.c_int64, [_vp]),
    "dymu_planner_get_global_node": (_i32, [_vp, _u32, _u32, _vp]),
    "dymu_planner_is_safe_node": (_i32, [_vp, _u32, _u32]),
    "dymu_planner_is_fully_closed_node": (_i32, [_vp, _u32, _u32]),
    "dymu_planner_global_narrowband": (ctypes.c_int64, [_vp, _vp, ctypes.c_int64]),
    "dymu_planner_min_cost_global_node": (_i32, [_vp, _vp, _dp]),
    "dymu_planner_reset_global_narrow_band": (_i32, [_vp]),
    "dymu_planner_gradient_node": (_i32, [_vp, _u32, _u32, _dp]),
    "dymu_planner_local_waypoint_dijkstra": (_i32, [_vp, _dp, _dp]),
    "dymu_planner_local_agent": (_i32, [_vp, _dp]),
    "dymu_planner_reset_total_cost_map": (_i32, [_vp]),
    "dymu_planner_load_total_cost_map": (_i32, [_vp, _dp]),
    "dymu_planner_set_current_path": (_i32, [_vp, _vp, _i32]),
    "dymu_planner_get_current_path": (_i32, [_vp, _dp, _i32]),
    "dymu_planner_compute_local_planning": (_i32, [_vp, _d, _d, _d, _d, _vp, _u32, _u32, _u32,
                                                   _u32, _d, _dp, _i32, ctypes.POINTER(_i32),
                                                   ctypes.POINTER(_d)]),
    "dymu_planner_repair_path": (_i32, [_vp, _d, _d, _d, _d, _u32]),
    "dymu_planner_evaluate_path": (_i32, [_vp, _u32]),
    "dymu_planner_expand_risk": (_i32, [_vp]),
    "dymu_planner_compute_local_propagation": (_i32, [_vp, _dp, _dp, _dp]),
    "dymu_planner_set_local_timeout": (_i32, [_vp, ctypes.c_double]),
    "dymu_planner_get_risk_matrix": (_i32, [_vp, _d, _d, _d, _d, _dp]),
    "dymu_planner_get_deviation_matrix": (_i32, [_vp, _d, _d, _d, _d, _dp]),
    "dymu_planner_get_reconnecting_index": (_i32, [_vp]),
    "dymu_planner_res_ratio": (_i32, [_vp]),
    "dymu_planner_local_map_mask": (ctypes.c_int64, [_vp, _vp]),
    "dymu_planner_local_block": (_i32, [_vp, _u32, _u32, _vp, _vp, _vp, _vp, _vp]),
    "dymu_planner_propagate_global_node": (_i32, [_vp, _u32, _u32]),
    "dymu_planner_set_global_node_state": (_i32, [_vp, _u32, _u32, _i32]),
    "dymu_planner_global_propagated_nodes": (ctypes.c_int64, [_vp, _vp, ctypes.c_int64]),
    "dymu_planner_get_local_node": (_i32, [_vp, _d, _d, _vp]),
    "dymu_planner_max_risk_node": (_i32, [_vp, _vp]),
    "dymu_planner_local_neighbour": (_i32, [_vp, _u64, _i32, _vp]),
    "dymu_planner_propagate_risk": (_i32, [_vp, _u64]),
    "dymu_planner_propagate_local_node": (_i32, [_vp, _u64]),
    "dymu_planner_set_local_node_state": (_i32, [_vp, _u64, _i32]),
    "dymu_planner_min_cost_local_node": (_i32, [_vp, _d, _d, _vp]),
    "dymu_planner_min_cost_local_node_reach": (_i32, [_vp, _u64, _vp]),
    "dymu_planner_local_list": (ctypes.c_int64, [_vp, _i32, _vp, ctypes.c_int64]),
}


class DymuGlobalNode(ctypes.Structure):
    _fields_ = [("elevation", _d), ("slope", _d), ("raw_cost", _d), ("cost", _d),
                ("hazard_density", _d), ("trafficability", _d), ("total_cost", _d),
                ("terrain", _u32), ("state", _i32), ("is_obstacle", _i32),
                ("has_local_map", _i32)]

class DymuLocalNode(ctypes.Structure):
    _fields_ = [("global_x", _d), ("global_y", _d), ("deviation", _d), ("total_cost", _d),
                ("risk", _d), ("parent_i", _u32), ("parent_j", _u32), ("li", _u32),
                ("lj", _u32), ("state", _i32), ("is_obstacle", _i32), ("id", _u64)]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


_pl = None


def load_planner() -> ctypes.CDLL:
    global _pl
    if _pl is None:
        load_fim()
        path = lib_path("libdymu_planner.so")
        if not os.path.exists(path):
            raise DymuError(-5, f"planner library missing: {path} (run __graft_entry__.build())")
        lib = ctypes.CDLL(path)
        for name, (res, args) in PLANNER_SYMBOLS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _pl = lib
    return _pl


def _b_int(rc: int) -> int:
    if rc < 0:
        raise DymuError(rc)
    return rc


def _b(rc: int) -> bool:
    if rc < 0:
        raise DymuError(rc)
    return bool(rc)


class Planner:
    """Python mirror of PathPlanning_lib::DyMuPathPlanner (reference
    src/DyMu.hpp:397-609, global layer).  Method names follow the reference;
    waypoints are (x, y[, z, heading]) tuples; grids are numpy [ny, nx]."""

    CONSERVATIVE, SWEEPING = 0, 1

    def __init__(self, risk_distance=1.0, reconnect_distance=1.0, risk_ratio=1.0,
                 approach=CONSERVATIVE, device: int = -1):
        self._lib = load_planner()
        h = _vp()
        rc = self._lib.dymu_planner_create(ctypes.byref(h), risk_distance, reconnect_distance,
                                           risk_ratio, approach)
        if rc != DYMU_OK:
            raise DymuError(rc, "dymu_planner_create")
        self.h = h
        self.nx = self.ny = 0
        if device >= 0:
            o = DymuOpts(device, 0, 0, 0, 0)
            _check(self._lib.dymu_planner_set_engine_options(self.h, ctypes.byref(o)))

    def close(self):
        if getattr(self, "h", None):
            self._lib.dymu_planner_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _wp(w):
        w = tuple(w) + (0.0,) * (4 - len(w))
        return float(w[0]), float(w[1]), float(w[2]), float(w[3])

    def _grid(self, a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        if a.shape != (self.ny, self.nx):
            raise ValueError(f"expected [{self.ny}, {self.nx}] grid, got {a.shape}")
        return a

    def initGlobalLayer(self, globalres, localres, nx, ny, offset=(0.0, 0.0)) -> bool:
        self.nx, self.ny = int(nx), int(ny)
        return _b(self._lib.dymu_planner_init_global_layer(self.h, globalres, localres, nx, ny,
                                                           offset[0], offset[1]))

    def setCostMap(self, cost_map) -> bool:
        a = np.ascontiguousarray(cost_map, dtype=np.float64)
        ny, nx = a.shape
        return _b(self._lib.dymu_planner_set_cost_map(self.h, a, nx, ny))

    def computeCostMap(self, cost_data, slope_values, locomotion_modes, elevation,
                       terrain_map) -> bool:
        lut = np.ascontiguousarray(cost_data, dtype=np.float64)
        sl = np.ascontiguousarray(slope_values, dtype=np.float64)
        modes = (ctypes.c_char_p * len(locomotion_modes))(*[m.encode() for m in locomotion_modes])
        return _b(self._lib.dymu_planner_compute_cost_map(
            self.h, lut, len(lut), sl, len(sl), modes, len(locomotion_modes),
            self._grid(elevation), self._grid(terrain_map)))

    def setGoal(self, w) -> bool:
        return _b(self._lib.dymu_planner_set_goal(self.h, *self._wp(w)))

    def computeTotalCostMap(self, w) -> bool:
        return _b(self._lib.dymu_planner_compute_total_cost_map(self.h, *self._wp(w)))

    def computeEntireTotalCostMap(self) -> bool:
        return _b(self._lib.dymu_planner_compute_entire_total_cost_map(self.h))

    def _matrix(self, fn):
        out = np.empty((self.ny, self.nx))
        _check(fn(self.h, out))
        return out

    def getTotalCostMatrix(self):
        return self._matrix(self._lib.dymu_planner_get_total_cost_matrix)

    def getGlobalCostMatrix(self):
        return self._matrix(self._lib.dymu_planner_get_global_cost_matrix)

    def getHazardDensityMatrix(self):
        return self._matrix(self._lib.dymu_planner_get_hazard_density_matrix)

    def getTrafficabilityMatrix(self):
        return self._matrix(self._lib.dymu_planner_get_trafficability_matrix)

    def totalCostRaw(self):
        return self._matrix(self._lib.dymu_planner_get_total_cost_raw)

    def getTotalCost(self, w) -> float:
        out = ctypes.c_double()
        _check(self._lib.dymu_planner_get_total_cost(self.h, *self._wp(w), ctypes.byref(out)))
        return out.value

    def getPath(self, w, max_wp: int = 1 << 20) -> np.ndarray:
        buf = np.empty(4 * max_wp)
        n = self._lib.dymu_planner_get_path(self.h, *self._wp(w), buf, max_wp)
        if n < 0:
            raise DymuError(n)
        return buf[:4 * min(n, max_wp)].reshape(-1, 4).copy()

    def getLocomotionMode(self, w) -> str:
        buf = ctypes.create_string_buffer(256)
        _check(min(0, self._lib.dymu_planner_get_locomotion_mode(self.h, *self._wp(w), buf, 256)))
        return buf.value.decode()

    def setHazardDensity(self, hd) -> bool:
        return _b(self._lib.dymu_planner_set_hazard_density(self.h, self._grid(hd)))

    def setTrafficability(self, tr) -> bool:
        return _b(self._lib.dymu_planner_set_trafficability(self.h, self._grid(tr)))

    def setHazardDensityWindow(self, i0: int, j0: int, hd) -> bool:
        a = np.ascontiguousarray(hd, dtype=np.float64)
        h, w = a.shape
        return _b(self._lib.dymu_planner_set_hazard_density_window(self.h, i0, j0, w, h, a))

    def setTrafficabilityWindow(self, i0: int, j0: int, tr) -> bool:
        a = np.ascontiguousarray(tr, dtype=np.float64)
        h, w = a.shape
        return _b(self._lib.dymu_planner_set_trafficability_window(self.h, i0, j0, w, h, a))

    def lastBandSize(self) -> int:
        """Narrow-band cells left by the last computeTotalCostMap (0 after a full solve)."""
        return _b_int(self._lib.dymu_planner_last_band_size(self.h))

    def lastSolveKind(self) -> int:
        """0 cold solve, 1 windowed re-propagation, 2 previous map reused."""
        return _b_int(self._lib.dymu_planner_last_solve_kind(self.h))

    def lastEarlyExit(self) -> dict:
        """How the last computeTotalCostMap resolved the reference's pop order at its
        exit value: tied cells, those left OPEN, whether the exact host replay ran
        (degenerate ties only), host milliseconds of the resolution and band replay."""
        o = np.zeros(8)
        _check(self._lib.dymu_planner_last_early_exit_ex(self.h, o.ctypes.data, 8))
        return {"tied": int(o[0]), "open_at_limit": int(o[1]), "exact_replay": bool(o[2]),
                "resolve_ms": float(o[3]), "replay_updates": int(o[4]),
                "band_exact": bool(o[5]), "near_ties": int(o[6]), "replay_threads": int(o[7])}

    def lastStats(self) -> dict:
        st = DymuStats()
        _check(self._lib.dymu_planner_last_stats(self.h, ctypes.byref(st)))
        return st.as_dict()

    # ---- node-level access (src/DyMu.hpp:500-518) ----
    def getGlobalNode(self, i: int, j: int):
        """Snapshot dict of node (i, j), or None (the reference's NULL)."""
        n = DymuGlobalNode()
        if not _b(self._lib.dymu_planner_get_global_node(self.h, i, j, ctypes.byref(n))):
            return None
        return {f: getattr(n, f) for f, _ in DymuGlobalNode._fields_}

    def isSafeNode(self, i: int, j: int) -> bool:
        return _b(self._lib.dymu_planner_is_safe_node(self.h, i, j))

    def isFullyClosedNode(self, i: int, j: int) -> bool:
        return _b(self._lib.dymu_planner_is_fully_closed_node(self.h, i, j))

    def resetTotalCostMap(self):
        _check(self._lib.dymu_planner_reset_total_cost_map(self.h))

    def globalNarrowband(self) -> np.ndarray:
        """global_narrowband (:445) after computeTotalCostMap: (n, 2) array of (i, j)."""
        n = self._lib.dymu_planner_global_narrowband(self.h, None, 0)
        if n < 0:
            _check(int(n))
        ij = np.zeros((max(n, 1), 2), dtype=np.uint32)
        m = self._lib.dymu_planner_global_narrowband(self.h, ij.ctypes.data, n)
        if m < 0:
            _check(int(m))
        return ij[:min(n, m)]

    def minCostGlobalNode(self):
        """minCostGlobalNode (:548-567): ((i, j), total_cost) of the band's lowest
        node, removed from the band list; None on an empty band."""
        ij = np.zeros(2, dtype=np.uint32)
        t = np.zeros(1)
        if not _b(self._lib.dymu_planner_min_cost_global_node(self.h, ij.ctypes.data, t)):
            return None
        return (int(ij[0]), int(ij[1])), float(t[0])

    def resetGlobalNarrowBand(self):
        _check(self._lib.dymu_planner_reset_global_narrow_band(self.h))

    def propagateGlobalNode(self, i: int, j: int):
        """propagateGlobalNode (:500-546) on node (i, j) (host copy of the map)."""
        _check(self._lib.dymu_planner_propagate_global_node(self.h, i, j))

    def setGlobalNodeState(self, i: int, j: int, closed: bool):
        """The public globalNode::state: CLOSED (True) or OPEN."""
        _check(self._lib.dymu_planner_set_global_node_state(self.h, i, j, 1 if closed else 0))

    def nodeStates(self) -> np.ndarray:
        """Every node's state, [ny, nx] uint8 (1 CLOSED, 0 OPEN)."""
        out = np.empty((self.ny, self.nx), dtype=np.uint8)
        _check(self._lib.dymu_planner_get_node_states(self.h, out.ctypes.data))
        return out

    def globalPropagatedNodes(self) -> np.ndarray:
        """global_propagated_nodes (:447): (n, 2) array of (i, j)."""
        n = self._lib.dymu_planner_global_propagated_nodes(self.h, None, 0)
        if n < 0:
            _check(int(n))
        ij = np.zeros((max(n, 1), 2), dtype=np.uint32)
        m = self._lib.dymu_planner_global_propagated_nodes(self.h, ij.ctypes.data, n)
        if m < 0:
            _check(int(m))
        return ij[:min(n, m)]

    # the local layer's per-node steps (L:525-805); nodes are dicts with an "id"
    def _local(self, fn, *args):
        n = DymuLocalNode()
        if not _b(fn(self.h, *args, ctypes.byref(n))):
            return None
        return n.as_dict()

    def getLocalNode(self, x: float, y: float):
        """getLocalNode(Waypoint) (L:177-189; subdivides): dict or None."""
        return self._local(self._lib.dymu_planner_get_local_node, float(x), float(y))

    def localNeighbour(self, node, d: int):
        """node's nb4List[d] (0 (i,j-1), 1 (i-1,j), 2 (i+1,j), 3 (i,j+1)), or None."""
        return self._local(self._lib.dymu_planner_local_neighbour, int(node["id"]), int(d))

    def maxRiskNode(self):
        return self._local(self._lib.dymu_planner_max_risk_node)

    def propagateRisk(self, node):
        _check(self._lib.dymu_planner_propagate_risk(self.h, int(node["id"])))

    def propagateLocalNode(self, node):
        _check(self._lib.dymu_planner_propagate_local_node(self.h, int(node["id"])))

    def setLocalNodeState(self, node, closed: bool):
        _check(self._lib.dymu_planner_set_local_node_state(self.h, int(node["id"]),
                                                           1 if closed else 0))

    def minCostLocalNode(self, Tovertake=None, minC=None, reach=None):
        """minCostLocalNode(Tovertake, minC) (SWEEPING key) or minCostLocalNode(reach)
        (CONSERVATIVE key: deviation + distance to reach)."""
        if reach is not None:
            return self._local(self._lib.dymu_planner_min_cost_local_node_reach, int(reach["id"]))
        return self._local(self._lib.dymu_planner_min_cost_local_node, float(Tovertake or 0.0),
                           float(minC or 0.0))

    def _local_list(self, which: int) -> list:
        n = self._lib.dymu_planner_local_list(self.h, which, None, 0)
        if n < 0:
            _check(int(n))
        arr = (DymuLocalNode * max(n, 1))()
        m = self._lib.dymu_planner_local_list(self.h, which, arr, n)
        if m < 0:
            _check(int(m))
        return [arr[q].as_dict() for q in range(min(n, m))]

    def localNarrowband(self) -> list:
        return self._local_list(0)

    def localExpandableObstacles(self) -> list:
        return self._local_list(1)

    def localPropagatedNodes(self) -> list:
        return self._local_list(2)

    def gradientNode(self, i: int, j: int):
        """gradientNode (:718-772): (dnx, dny)."""
        d = np.zeros(2)
        _check(self._lib.dymu_planner_gradient_node(self.h, i, j, d))
        return float(d[0]), float(d[1])

    def computeLocalWaypointDijkstra(self, w):
        """L:851-869 from the sub-cell at waypoint w: (x, y, z, heading), or None."""
        s = np.array(self._wp(w))
        out = np.zeros(4)
        if not _b(self._lib.dymu_planner_local_waypoint_dijkstra(self.h, s, out)):
            return None
        return tuple(float(v) for v in out)

    def localAgent(self):
        """local_agent's global pose (x, y), or None."""
        xy = np.zeros(2)
        if not _b(self._lib.dymu_planner_local_agent(self.h, xy)):
            return None
        return float(xy[0]), float(xy[1])

    def loadTotalCostMap(self, T) -> bool:
        return _b(self._lib.dymu_planner_load_total_cost_map(self.h, self._grid(T)))

    @property
    def current_path(self) -> np.ndarray:
        n = _b_int(self._lib.dymu_planner_get_current_path(self.h, np.empty(0), 0))
        buf = np.empty(4 * max(n, 1))
        self._lib.dymu_planner_get_current_path(self.h, buf, n)
        return buf[:4 * n].reshape(-1, 4).copy()

    @current_path.setter
    def current_path(self, wps):
        a = np.ascontiguousarray(np.asarray(wps, dtype=np.float64).reshape(-1, 4))
        _check(self._lib.dymu_planner_set_current_path(self.h, a.ctypes.data, len(a)))

    # ---- local layer (src/DyMu_LocalPathRepairing.cpp) ----
    def computeLocalPlanning(self, w, image, res):
        """image: uint8 [height, width] (nonzero = obstacle) or [height, width,
        pixel_size].  Returns (repaired, trajectory [n, 4], local_time_s)."""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, wd = img.shape[:2]
        ps = img.shape[2] if img.ndim == 3 else 1
        cap = max(64, 4 * len(self.current_path) + 4096)
        buf = np.empty(4 * cap)
        n = ctypes.c_int32()
        t = ctypes.c_double()
        r = _b(self._lib.dymu_planner_compute_local_planning(
            self.h, *self._wp(w), img.ctypes.data, wd, h, wd * ps, ps, res, buf, cap,
            ctypes.byref(n), ctypes.byref(t)))
        if not r:
            return False, np.empty((0, 4)), 0.0
        if n.value > cap:
            return True, self.current_path, t.value
        return True, buf[:4 * n.value].reshape(-1, 4).copy(), t.value

    def repairPath(self, w, index: int) -> int:
        rc = self._lib.dymu_planner_repair_path(self.h, *self._wp(w), index)
        if rc < -1:
            raise DymuError(rc)
        return rc

    def evaluatePath(self, starting_index: int) -> bool:
        return _b(self._lib.dymu_planner_evaluate_path(self.h, starting_index))

    def expandRisk(self):
        _check(self._lib.dymu_planner_expand_risk(self.h))

    def setLocalPropagationTimeout(self, seconds: float):
        """computeLocalPropagation's wall-clock limit (reference: 5 s, <= 0: none)."""
        _check(self._lib.dymu_planner_set_local_timeout(self.h, float(seconds)))

    def computeLocalPropagation(self, w_init, w_overtake):
        """The set node's global pose (x, y), or None."""
        s = np.array(self._wp(w_init))
        o = np.array(self._wp(w_overtake))
        xy = np.empty(2)
        if not _b(self._lib.dymu_planner_compute_local_propagation(self.h, s, o, xy)):
            return None
        return float(xy[0]), float(xy[1])

    def resRatio(self) -> int:
        return _b_int(self._lib.dymu_planner_res_ratio(self.h))

    def _window(self, fn, w):
        ls = 21 * self.resRatio()
        out = np.empty((ls, ls))
        _check(fn(self.h, *self._wp(w), out))
        return out

    def getRiskMatrix(self, w):
        return self._window(self._lib.dymu_planner_get_risk_matrix, w)

    def getDeviationMatrix(self, w):
        return self._window(self._lib.dymu_planner_get_deviation_matrix, w)

    def getReconnectingIndex(self) -> int:
        return self._lib.dymu_planner_get_reconnecting_index(self.h)

    def localMapMask(self):
        m = np.zeros((self.ny, self.nx), dtype=np.uint8)
        _b_int(self._lib.dymu_planner_local_map_mask(self.h, m.ctypes.data))
        return m

    def localBlock(self, i: int, j: int):
        """(dev, tc, risk, state, obst) of node (i, j)'s r x r sub-cells, or None."""
        r = self.resRatio()
        dev, tc, risk = (np.empty((r, r)) for _ in range(3))
        st, ob = (np.empty((r, r), dtype=np.uint8) for _ in range(2))
        if not _b(self._lib.dymu_planner_local_block(self.h, i, j, dev.ctypes.data,
                                                    tc.ctypes.data, risk.ctypes.data,
                                                    st.ctypes.data, ob.ctypes.data)):
            return None
        return dev, tc, risk, st, ob

