"""Row-slab sharded solve driven natively (libdymu_dist.so, include/dymu_dist.h).

The exchange loop of dymu.sharded.SlabSolver, moved into C++ on the engine's
stream: K passes (the first merges the rows received after the previous round
into the ghost rows) -> the boundary rows to rank±1 -> every 4th round a
reduction of the queued tile count, read one check late through the engine's
mailbox so the host never drains the device queue.  One loop, three transports:
  "rccl"  grouped ncclSend/ncclRecv over xGMI + ncclAllReduce (one GPU per rank)
  "ipc"   rows pushed into the neighbours' hipIpc-mapped receive rows, counts
          reduced through a /dev/shm board (ranks of one node, may share a GPU)
  "peer"  the rows pushed by the pass kernels themselves into the neighbours'
          peer-mapped receive rows with sequence tags; no host step per round,
          termination from the ranks' posted status on the board
  vdist_solve: every rank in this process (device-to-device copies).

torch.distributed only carries the control plane here (the 128-byte id,
barriers, timing); the data path is the library's own transport.

Reference: computeEntireTotalCostMap's propagation loop
(src/DyMu_GlobalPathPlanning.cpp:443-468), distributed as SURVEY.md s8(e).
"""
from __future__ import annotations

import ctypes
import os

from . import DymuError, DymuStats, _check, lib_path, load_fim

_i32, _u32, _u64, _vp = ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p
ID_BYTES = 128

DIST_SYMBOLS = {
    "dymu_dist_unique_id": (_i32, [ctypes.c_char_p]),
    "dymu_dist_create": (_i32, [ctypes.POINTER(_vp), _vp, _i32, ctypes.c_char_p, _i32, _i32]),
    "dymu_dist_destroy": (_i32, [_vp]),
    "dymu_dist_solve": (_i32, [_vp, _vp, _vp, _u64, _u32, _u32, _u32, _u32, _u32, _vp,
                               ctypes.POINTER(DymuStats)]),
    "dymu_vdist_solve": (_i32, [ctypes.POINTER(_vp), _i32, ctypes.POINTER(_vp),
                                ctypes.POINTER(_vp), _u64, _u32, _u32, _u32, _u32, _u32, _vp,
                                ctypes.POINTER(DymuStats)]),
    "dymu_dist_ipc_unique_id": (_i32, [ctypes.c_char_p]),
    "dymu_dist_create_ipc": (_i32, [ctypes.POINTER(_vp), _vp, _i32, ctypes.c_char_p, _i32, _i32]),
    "dymu_dist_create_peer": (_i32, [ctypes.POINTER(_vp), _vp, _i32, ctypes.c_char_p, _i32, _i32]),
    "dymu_dist_transport": (_i32, [_vp]),
    "dymu_dist_set_timeout": (ctypes.c_double, [ctypes.c_double]),
    "dymu_dist_last_error": (ctypes.c_char_p, [_vp]),
    "dymu_dist_comm_count": (_i32, [_vp, ctypes.POINTER(ctypes.c_int)]),
}

_dl = None


def load_dist() -> ctypes.CDLL:
    global _dl
    if _dl is None:
        load_fim()
        path = lib_path("libdymu_dist.so")
        if not os.path.exists(path):
            raise DymuError(-5, f"dist library missing: {path} (run __graft_entry__.build())")
        lib = ctypes.CDLL(path)
        for name, (res, args) in DIST_SYMBOLS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _dl = lib
    return _dl


TRANSPORTS = ("rccl", "ipc", "peer")


def set_timeout(seconds: float) -> float:
    """Process-wide bound on every host wait on a peer rank (0: DYMU_DIST_TIMEOUT_S /
    300 s again); returns the bound in force."""
    return float(load_dist().dymu_dist_set_timeout(float(seconds)))


def unique_id(transport: str = "rccl") -> bytes:
    """A fresh transport id (call on rank 0, broadcast the bytes): the RCCL
    communicator id, or the shared-memory board's name (IPC and peer transports)."""
    buf = ctypes.create_string_buffer(ID_BYTES)
    lib = load_dist()
    fn = lib.dymu_dist_ipc_unique_id if transport in ("ipc", "peer") else lib.dymu_dist_unique_id
    _check(fn(buf))
    return buf.raw


class DistSolver:
    """One rank of the native sharded solver.  Collective construction."""

    def __init__(self, engine, device: int, uid: bytes, rank: int, world: int,
                 transport: str = "rccl"):
        assert len(uid) == ID_BYTES and transport in TRANSPORTS
        self._lib = load_dist()
        self.eng = engine
        self.rank, self.world = rank, world
        self.transport = transport
        self.h = _vp()
        create = {"ipc": self._lib.dymu_dist_create_ipc,
                  "peer": self._lib.dymu_dist_create_peer}.get(transport, self._lib.dymu_dist_create)
        rc = create(ctypes.byref(self.h), engine.ctx, device, uid, rank, world)
        if rc != 0:
            raise DymuError(rc, f"dymu_dist_create ({transport} transport)")

    def comm_count(self) -> int:
        """Ranks the transport sees (ncclCommCount, or the IPC board's)."""
        n = ctypes.c_int(0)
        rc = self._lib.dymu_dist_comm_count(self.h, ctypes.byref(n))
        if rc != 0:
            raise DymuError(rc, "dymu_dist_comm_count")
        return n.value

    def close(self):
        if self.h:
            self._lib.dymu_dist_destroy(self.h)
            self.h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def solve(self, F_slab: int, T_buf: int, ld: int, nx: int, ny: int, goal_i: int,
              goal_j: int, passes_per_exchange: int = 0, stream: int = 0) -> dict:
        """F_slab: this rank's rows; T_buf: nrows + 2 rows (ghost, owned..., ghost)."""
        st = DymuStats()
        rc = self._lib.dymu_dist_solve(self.h, F_slab, T_buf, ld, nx, ny, goal_i, goal_j,
                                       passes_per_exchange, stream or None, ctypes.byref(st))
        if rc != 0:
            msg = self._lib.dymu_dist_last_error(self.h)
            raise DymuError(rc, msg.decode() if msg else "")
        return st.as_dict()


def vdist_solve(engines, F_slabs, T_bufs, ld: int, nx: int, ny: int, goal_i: int, goal_j: int,
                passes_per_exchange: int = 0, stream: int = 0) -> list:
    """All ranks in one process on one GPU (the C++ loop with copies for RCCL)."""
    lib = load_dist()
    w = len(engines)
    ctxs = (_vp * w)(*[e.ctx for e in engines])
    Fp = (_vp * w)(*F_slabs)
    Tp = (_vp * w)(*T_bufs)
    stats = (DymuStats * w)()
    if not stream:
        stream = load_fim().dymu_get_stream(engines[0].ctx)
    _check(lib.dymu_vdist_solve(ctxs, w, Fp, Tp, ld, nx, ny, goal_i, goal_j,
                                passes_per_exchange, stream, stats))
    return [s.as_dict() for s in stats]
