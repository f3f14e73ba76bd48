"""Shared pytest fixtures.

* ``oracle`` -- ctypes handle on oracle/build/liboracle.so (CPU restatement;
  test infrastructure only).
* ``dymu``   -- the product's Python binding (planning-path_planning_amd/dymu).
GPU tests are marked ``@pytest.mark.gpu`` and call the HIP path through the
C-ABI; everything else runs on CPU.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "planning-path_planning_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


def _ensure_built(target_dir, target):
    path = os.path.join(target_dir, target)
    if not os.path.exists(path):
        subprocess.run(["make", "-s"], cwd=target_dir, check=True)
    return path


@pytest.fixture(scope="session")
def oracle():
    import oracle_ffi
    return oracle_ffi.load()


@pytest.fixture(scope="session")
def dymu():
    import dymu as _d
    return _d


@pytest.fixture(scope="session")
def engine(dymu):
    eng = dymu.Engine()
    yield eng
    eng.close()


# pass kernels under test: 3 = plain block FIM, 4 = priority passes with a small
# per-pass target so that deferral happens even on test-sized grids
KERNELS = {"fim": dict(kernel=3), "prio": dict(kernel=4, prio_target=64),
           "prio16": dict(kernel=5, prio_target=16)}


@pytest.fixture(scope="session", params=sorted(KERNELS))
def kengine(request, dymu):
    eng = dymu.Engine(**KERNELS[request.param])
    yield eng
    eng.close()
