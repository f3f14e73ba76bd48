"""bench.py's whole-map parity block (oracle_parity): the headline map against the
oracle FMM's map of the same grid -- identical +inf mask, <= 1e-12 relative."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _maps(n=2500, seed=0):
    rng = np.random.default_rng(seed)
    To = rng.uniform(0, 5e4, (n, n))
    To[rng.random((n, n)) < 0.02] = np.inf
    return To.copy(), To


def test_identical_maps_pass():
    Tg, To = _maps()
    p = bench.oracle_parity(Tg, To)
    assert p["ok"] and p["max_rel"] == 0.0 and p["mismatched_cells"] == 0
    assert p["finite_cells"] == int(np.isfinite(To).sum())


def test_ulp_differences_pass_and_larger_fail():
    Tg, To = _maps(seed=1)
    Tg[5, 7] = np.nextafter(To[5, 7], np.inf) if np.isfinite(To[5, 7]) else Tg[5, 7]
    assert bench.oracle_parity(Tg, To)["ok"]
    j = np.argwhere(np.isfinite(To) & (To > 1))[0]
    Tg[j[0], j[1]] = To[j[0], j[1]] * (1 + 1e-10)
    p = bench.oracle_parity(Tg, To)
    assert not p["ok"] and 5e-11 < p["max_rel"] < 2e-10


def test_mask_mismatch_fails():
    Tg, To = _maps(seed=2)
    j = np.argwhere(np.isfinite(To))[0]
    Tg[j[0], j[1]] = np.inf
    p = bench.oracle_parity(Tg, To)
    assert not p["ok"] and p["mismatched_cells"] == 1
