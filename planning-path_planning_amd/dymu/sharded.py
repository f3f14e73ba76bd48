"""Row-slab sharded total-cost propagation over torch.distributed.

One process per GPU.  Rank r owns rows [row0, row0+nrows) of the global
grid (dymu.slab_rows) in a torch tensor of nrows+2 rows: row 0 and row
nrows+1 are ghost rows (the neighbours' boundary rows, read-only halo for the
kernels).  The solve alternates

    K local FIM passes  ->  exchange boundary rows with rank-1 / rank+1
    (batched P2P send/recv; RCCL over xGMI on GPU, gloo in the CPU tests)
    ->  min-merge received rows into the ghost rows and queue the tiles under
    improved columns

and every few exchanges all-reduces the number of queued tiles; 0 on every
rank means the global fixed point is reached.  Because values only decrease
and each rank relaxes the reference's own update (:500-546) against halo
values that are valid upper bounds, the result is the single-GPU fixed point
(SURVEY s8(e)).

`engine` is a dymu.Engine (or, in CPU tests, an object with the same dom_*
methods).  No collective touches the interior data: only two boundary rows per
rank per exchange plus one 4-byte all-reduce every `check_every` exchanges.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class SlabSolver:
    def __init__(self, engine, nx: int, ny: int, rank: int, world: int, row0: int, nrows: int,
                 device, group=None, passes_per_exchange: int = 4, check_every: int = 4):
        self.eng = engine
        self.nx, self.ny = nx, ny
        self.rank, self.world = rank, world
        self.row0, self.nrows = row0, nrows
        self.group = group
        self.K = passes_per_exchange
        self.check_every = check_every
        self.device = device
        self.lo = rank > 0
        self.hi = rank < world - 1
        self.recv_lo = torch.empty(nx, dtype=torch.float64, device=device)
        self.recv_hi = torch.empty(nx, dtype=torch.float64, device=device)
        self.pending = torch.zeros(1, dtype=torch.int32, device=device)
        self.exchanges = 0
        # gloo cannot move device tensors point-to-point: stage rows on the host
        # (used to rehearse N ranks on one GPU; RCCL ('nccl') moves them directly)
        self.host_stage = device.type == "cuda" and dist.get_backend(group) != "nccl"
        if self.host_stage:
            self.h_send = [torch.empty(nx, dtype=torch.float64) for _ in range(2)]
            self.h_recv = [torch.empty(nx, dtype=torch.float64) for _ in range(2)]
            self.h_pending = torch.zeros(1, dtype=torch.int32)

    def _stream(self) -> int:
        if self.device.type == "cuda":
            h = torch.cuda.current_stream(self.device).cuda_stream
            # 0 would mean "the engine's own stream" to the C-ABI, which is not
            # ordered with torch's collectives: solve() always runs on a real stream
            assert h != 0, "SlabSolver needs a non-default torch stream"
            return h
        return 0

    def _exchange(self, T_buf: torch.Tensor):
        if self.host_stage:
            return self._exchange_host(T_buf)
        ops = []
        if self.lo:
            ops.append(dist.P2POp(dist.isend, T_buf[1], self.rank - 1, group=self.group))
            ops.append(dist.P2POp(dist.irecv, self.recv_lo, self.rank - 1, group=self.group))
        if self.hi:
            ops.append(dist.P2POp(dist.isend, T_buf[self.nrows], self.rank + 1, group=self.group))
            ops.append(dist.P2POp(dist.irecv, self.recv_hi, self.rank + 1, group=self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()

    def _exchange_host(self, T_buf: torch.Tensor):
        torch.cuda.current_stream(self.device).synchronize()
        ops = []
        if self.lo:
            self.h_send[0].copy_(T_buf[1])
            ops.append(dist.P2POp(dist.isend, self.h_send[0], self.rank - 1, group=self.group))
            ops.append(dist.P2POp(dist.irecv, self.h_recv[0], self.rank - 1, group=self.group))
        if self.hi:
            self.h_send[1].copy_(T_buf[self.nrows])
            ops.append(dist.P2POp(dist.isend, self.h_send[1], self.rank + 1, group=self.group))
            ops.append(dist.P2POp(dist.irecv, self.h_recv[1], self.rank + 1, group=self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        if self.lo:
            self.recv_lo.copy_(self.h_recv[0])
        if self.hi:
            self.recv_hi.copy_(self.h_recv[1])

    def _all_reduce_pending(self) -> int:
        if self.host_stage:
            self.h_pending.copy_(self.pending)
            dist.all_reduce(self.h_pending, group=self.group)
            return int(self.h_pending.item())
        dist.all_reduce(self.pending, group=self.group)
        return int(self.pending.item())

    def solve(self, F: torch.Tensor, T_buf: torch.Tensor, goal_i: int, goal_j: int,
              max_exchanges: int = 1 << 30) -> dict:
        """F: [nrows, nx] slab; T_buf: [nrows+2, nx] (ghost rows 0 and nrows+1)."""
        if self.device.type == "cuda":
            if not hasattr(self, "_torch_stream"):
                self._torch_stream = torch.cuda.Stream(self.device)
            self._torch_stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self._torch_stream):
                out = self._solve(F, T_buf, goal_i, goal_j, max_exchanges)
            torch.cuda.current_stream(self.device).wait_stream(self._torch_stream)
            return out
        return self._solve(F, T_buf, goal_i, goal_j, max_exchanges)

    def _solve(self, F, T_buf, goal_i, goal_j, max_exchanges):
        assert F.shape == (self.nrows, self.nx) and T_buf.shape == (self.nrows + 2, self.nx)
        st = self._stream()
        gl = goal_j - self.row0 if self.row0 <= goal_j < self.row0 + self.nrows else -1
        ld = self.nx
        tptr = T_buf.data_ptr() + 8 * ld  # owned row 0
        self.eng.dom_begin(F.data_ptr(), tptr, self.nx, self.nrows, ld, self.lo, self.hi,
                           goal_i if gl >= 0 else 0, gl, st)
        # the first P2P of an NCCL group must not be a partial one
        self._all_reduce_pending()
        self.exchanges = 0
        converged = False
        while self.exchanges < max_exchanges:
            self.eng.dom_run(self.K, st)
            self._exchange(T_buf)
            self.eng.dom_merge_ghosts(self.recv_lo.data_ptr() if self.lo else 0,
                                      self.recv_hi.data_ptr() if self.hi else 0,
                                      self.pending.data_ptr(), st)
            self.exchanges += 1
            if self.exchanges % self.check_every == 0:
                if self._all_reduce_pending() == 0:
                    converged = True
                    break
        stats = self.eng.dom_finish(st)
        stats["rounds"] = self.exchanges
        if not converged:  # every rank stops at the same exchange count: all raise
            raise RuntimeError(f"SlabSolver: no global fixed point after {self.exchanges} "
                               f"exchanges (max_exchanges={max_exchanges})")
        return stats
