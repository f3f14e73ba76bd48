"""Sparse passes (k_fim_sparse): many kernel-5 passes in one launch on
the workgroups of one XCD, with a workgroup barrier between passes instead of a kernel
boundary.  They run the dense kernel's passes (same body, same buffers, same rotation),
so every map must meet the same oracle bounds as the dense path:
  - every pass sparse (DYMU_SPARSE_MAX huge): open grids, the maze, obstacles;
  - the sparse -> dense switch mid-solve (a small threshold on an open grid);
  - windowed updates and the early exit (the probe posts) through sparse passes;
  - the launch count falls by the passes per launch.
The threshold is read from the environment when an Engine is created."""
import os

import numpy as np
import pytest

from test_gpu_maze import maze_speed, signed_dev, solve_device
from test_gpu_solver import assert_parity

pytestmark = pytest.mark.gpu


@pytest.fixture
def sparse_env():
    """set DYMU_SPARSE_* for the Engines created inside the test, restore after"""
    keys = ("DYMU_SPARSE_MAX", "DYMU_SPARSE_PASSES", "DYMU_SPARSE_WG")
    old = {k: os.environ.get(k) for k in keys}

    def set_(**kw):
        for k in keys:
            os.environ.pop(k, None)
        for k, v in kw.items():
            os.environ["DYMU_SPARSE_" + k.upper()] = str(v)

    yield set_
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.mark.parametrize("N", [257, 1024])
def test_all_passes_sparse_open_grid(dymu, oracle, sparse_env, N):
    g = (N // 3, N // 2)
    F = oracle.synth_speed(N, N, seed=5, obst_frac=0.02, obst_seed=7, goal=g)
    Tref, _ = oracle.fmm(F, g)
    sparse_env(max=10 ** 9)
    T, st = solve_device(dymu, F, g)
    assert_parity(T, Tref)
    assert st["kernel"] == 5
    assert st["launches"] * 4 < st["passes"]  # 16 passes per launch (less the last)


def test_all_passes_sparse_maze(dymu, oracle, sparse_env):
    F, g = maze_speed(oracle, 2048)
    Tref, _ = oracle.fmm(F, g)
    sparse_env(max=10 ** 9, passes=64)
    T, st = solve_device(dymu, F, g)
    assert_parity(T, Tref)
    up, dn = signed_dev(T, Tref)
    assert dn <= 1e-13
    sparse_env(max=0)
    T0, st0 = solve_device(dymu, F, g)
    assert st["launches"] * 16 < st0["launches"]  # one launch per 64 passes vs one per pass
    assert abs(st["passes"] - st0["passes"]) <= 0.05 * st0["passes"]  # the same passes


def test_sparse_then_dense(dymu, oracle, sparse_env):
    """an open grid whose list outgrows a threshold of 64 tiles: sparse launches at
    first, single dense launches after; the map is the oracle's"""
    N = 2048
    g = (N // 2, N // 2)
    F = oracle.synth_speed(N, N, seed=11, obst_frac=0.02, obst_seed=3, goal=g)
    Tref, _ = oracle.fmm(F, g)
    sparse_env(max=64, passes=8)
    T, st = solve_device(dymu, F, g)
    assert_parity(T, Tref)
    sparse_env(max=0)
    _, st0 = solve_device(dymu, F, g)
    assert st["launches"] < st0["launches"]  # some passes ran sparse


@pytest.mark.parametrize("wg", [8, 32])
def test_sparse_workgroup_counts(dymu, oracle, sparse_env, wg):
    N = 1024
    g = (7, N - 9)
    F = oracle.synth_speed(N, N, seed=3, obst_frac=0.05, obst_seed=9, goal=g)
    Tref, _ = oracle.fmm(F, g)
    sparse_env(max=10 ** 9, wg=wg)
    T, _ = solve_device(dymu, F, g)
    assert_parity(T, Tref)
