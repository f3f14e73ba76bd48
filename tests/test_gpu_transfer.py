"""Host <-> device transfers of the early exit (VERDICT r5 "do this" 1).

Round 5's computeTotalCostMap once wrote T = 0 into cell (0, 0): dymu_scatter staged
its indices and values in stream-ordered pool memory (hipMallocAsync), and on this stack
a kernel reading such memory beyond its first 4 KiB page sees an earlier allocation's
bytes, whatever the copy (tools/copy_order_probe.hip, profiles/r06/copy_order_probe.jsonl).
dymu_scatter / dymu_find_equal now hand their data to the kernels in pinned host memory,
and no product source allocates from a stream-ordered pool.

The GPU test runs scatter / find_equal on one context right after a windowed
re-propagation and an early exit, at the probe's sizes (one page and far beyond), and
checks every cell of the map afterwards."""
import os
import re

import numpy as np
import pytest

from test_gpu_solver import assert_parity

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_stream_ordered_allocations_in_product():
    """No product source calls the stream-ordered allocator (its mapping is not coherent
    between the copy paths and the kernels here)."""
    csrc = os.path.join(ROOT, "planning-path_planning_amd", "csrc")
    pat = re.compile(r"\bhip(MallocAsync|FreeAsync|MallocFromPoolAsync|MemPoolCreate)\s*\(")
    hits = []
    for name in sorted(os.listdir(csrc)):
        with open(os.path.join(csrc, name), encoding="utf-8") as f:
            for k, line in enumerate(f, 1):
                if pat.search(line.split("//")[0]):
                    hits.append(f"{name}:{k}")
    assert not hits, hits


@pytest.mark.gpu
def test_scatter_find_equal_after_window_and_early_exit(dymu, oracle):
    N, g, s = 512, (256, 256), (102, 128)
    eng = dymu.Engine()
    dF = dT = None
    try:
        dF, dT = eng.alloc(8 * N * N), eng.alloc(8 * N * N)
        F0 = oracle.synth_speed(N, N, seed=1, obst_frac=0.0, obst_seed=3, goal=g)
        eng.h2d(dF, F0)
        eng.solve_device(dF, dT, N, N, N, *g)
        # a windowed re-propagation (speed raised in a box) on the same context
        F1 = F0.copy()
        F1[100:140, 60:120] *= 1.5
        eng.h2d(dF, F1)
        eng.update_window_device(dF, dT, N, N, N, g[0], g[1], 60, 100, 60, 40, False)
        T = np.empty((N, N))
        eng.d2h(T, dT)
        Tref, _ = oracle.fmm(F1, g)
        assert_parity(T, Tref)
        # then an early exit
        tc, _ = eng.solve_until_device(dF, dT, N, N, N, g[0], g[1], *s)
        assert np.isfinite(tc)
        eng.d2h(T, dT)
        cur = T.ravel().copy()
        rng = np.random.default_rng(5)
        for n in (150, 1328, 4096, 65536):  # within one page, and far beyond it
            idx = rng.choice(np.arange(1, N * N), size=n, replace=False).astype(np.uint64)
            vals = rng.uniform(1e3, 2e3, n)
            eng.scatter(dT, N, N, idx, vals)
            cur[idx] = vals
            eng.d2h(T, dT)
            assert np.array_equal(T.ravel(), cur), f"scatter of {n} cells"
            # plant one value at those cells and find exactly them
            v = 7777.25
            eng.scatter(dT, N, N, idx, np.full(n, v))
            cnt, got = eng.find_equal(dT, N, N, N, v, n)
            assert cnt == n
            assert np.array_equal(np.sort(got), np.sort(idx))
            cnt_small, got_small = eng.find_equal(dT, N, N, N, v, 16)
            assert cnt_small == n and len(got_small) == 16
            assert np.isin(got_small, idx).all()
            eng.scatter(dT, N, N, idx, vals)
        eng.d2h(T, dT)
        assert np.array_equal(T.ravel(), cur)
        assert T[0, 0] == cur[0]  # the cell round 5 saw overwritten
    finally:
        for p in (dF, dT):
            if p:
                eng.free(p)
        eng.close()
