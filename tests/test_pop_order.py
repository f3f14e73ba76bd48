"""The reference FMM's pop / insertion order rebuilt from the total costs alone
(planning-path_planning_amd/csrc/pop_order.hpp), against the order the oracle's
FMM actually followed (oracle_fmm_order: each node's band-insertion sequence, the
linear scan's tie rule of src/DyMu_GlobalPathPlanning.cpp:551-568).  This is what
lets the planner's early exit (:364-408) decide ties at its exit value and list
global_narrowband in the reference's order without replaying the FMM.  CPU only:
the header is compiled into a small test library with g++."""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "planning-path_planning_amd", "csrc")
U64 = np.uint64(np.iinfo(np.uint64).max)


@pytest.fixture(scope="module")
def po(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("needs g++")
    out = str(tmp_path_factory.mktemp("po") / "libpo.so")
    subprocess.run(["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-I" + CSRC,
                    os.path.join(ROOT, "tests", "pop_order", "pop_order_check.cpp"), "-o", out],
                   check=True)
    lib = ctypes.CDLL(out)
    dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
    up = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
    bp = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
    u32, u64 = ctypes.c_uint32, ctypes.c_uint64
    lib.po_ins_sort.argtypes = [dp, u32, u32, u64, up, u64]
    lib.po_ins_sort.restype = ctypes.c_int
    lib.po_pop_before.argtypes = [dp, u32, u32, u64, up, up, u64, bp]
    lib.po_pop_before.restype = ctypes.c_int
    return lib


def _maps(oracle):
    """(name, F, goal): constant speed (every mirror image ties), two-valued speed
    (many exact ties off the axes), random U(1,5) with obstacles, a non-square grid."""
    rng = np.random.default_rng(7)
    two = np.where(rng.random((80, 80)) < 0.5, 1.0, 2.0)
    F = oracle.synth_speed(120, 120, seed=11, obst_frac=0.05, obst_seed=12, goal=(40, 70))
    rect = np.ones((37, 90))
    rect[10:20, 30] = np.inf
    return [("const96", np.ones((96, 96)), (48, 48)), ("const_edge", np.ones((64, 64)), (0, 5)),
            ("two_valued", two, (40, 40)), ("random", F, (40, 70)), ("rect", rect, (70, 3))]


@pytest.mark.parametrize("k", range(5))
def test_insertion_order_full_solve(po, oracle, k):
    """Every reached node sorted by the rebuilt insertion order equals the oracle's
    global_propagated_nodes order (bit-exact oracle values)."""
    name, F, g = _maps(oracle)[k]
    ny, nx = F.shape
    T, _, _, seq = oracle.fmm_order(F, g)
    reached = np.flatnonzero(seq.ravel() != U64).astype(np.uint64)
    want = reached[np.argsort(seq.ravel()[reached], kind="stable")]
    cells = reached.copy()
    deg = po.po_ins_sort(np.ascontiguousarray(T), nx, ny, g[1] * nx + g[0], cells, cells.size)
    assert deg == 0, name
    assert np.array_equal(cells, want), name


@pytest.mark.parametrize("k", range(5))
def test_pop_order_ties(po, oracle, k):
    """pop(x) < pop(y) for every pair of nodes of exactly equal total cost (the
    ties the linear scan breaks by band order), against (T, seq) of the oracle."""
    name, F, g = _maps(oracle)[k]
    ny, nx = F.shape
    T, _, _, seq = oracle.fmm_order(F, g)
    t, s = T.ravel(), seq.ravel()
    fin = np.flatnonzero(np.isfinite(t))
    order = fin[np.lexsort((s[fin], t[fin]))]
    same = t[order[1:]] == t[order[:-1]]
    x = order[:-1][same].astype(np.uint64)
    y = order[1:][same].astype(np.uint64)
    if name.startswith("const") or name == "two_valued":
        assert x.size > 10, name  # the maps are meant to tie
    out = np.zeros(x.size, dtype=np.uint8)
    assert po.po_pop_before(np.ascontiguousarray(T), nx, ny, g[1] * nx + g[0], x, y, x.size,
                            out) == 0
    assert out.all(), name
    assert po.po_pop_before(np.ascontiguousarray(T), nx, ny, g[1] * nx + g[0], y, x, y.size,
                            out) == 0
    assert not out.any(), name


@pytest.mark.parametrize("N,g,s", [(160, (80, 80), (20, 140)), (96, (48, 48), (48, 20)),
                                   (96, (30, 30), (60, 60))])
def test_early_exit_band_order(po, oracle, N, g, s):
    """At the early exit (:390-398) on constant speed: the band (reached, not CLOSED)
    in rebuilt insertion order equals the reference's band vector, and the cells of
    exactly the exit value the reference had not closed are exactly those popped
    after the last of the start and its nb4."""
    F = np.ones((N, N))
    T, rc, closed, seq = oracle.fmm_order(F, g, start=s)
    t, sq, cl = T.ravel(), seq.ravel(), closed.ravel()
    band = np.flatnonzero((cl == 0) & np.isfinite(t)).astype(np.uint64)
    want = band[np.argsort(sq[band], kind="stable")]
    cells = band.copy()
    assert po.po_ins_sort(np.ascontiguousarray(T), N, N, g[1] * N + g[0], cells, cells.size) == 0
    assert np.array_equal(cells, want)
    sk = s[1] * N + s[0]
    probes = np.array([sk, sk - N, sk - 1, sk + 1, sk + N], dtype=np.uint64)
    tstar = t[probes].max()
    eq = np.flatnonzero(t == tstar).astype(np.uint64)
    cand = probes[t[probes] == tstar]
    last = cand[np.argmax(sq[cand])]
    others = eq[eq != last]
    after = np.zeros(others.size, dtype=np.uint8)
    po.po_pop_before(np.ascontiguousarray(T), N, N, g[1] * N + g[0],
                     np.full(others.size, last, dtype=np.uint64), others, others.size, after)
    assert np.array_equal(after.astype(bool), cl[others] == 0)
