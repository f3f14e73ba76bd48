"""CPU tests of the drop-in boundary: both C-ABI libraries load and export
every function include/*.h declares; without a GPU the engine refuses loudly
(DYMU_ERR_NO_DEVICE) instead of falling back to anything."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dymu_[a-z0-9_]+)\s*\(", src)))


def test_fim_exports_every_declared_symbol(dymu):
    lib = dymu.load_fim()
    names = declared("dymu_fim.h")
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) <= set(dymu.FIM_SYMBOLS), set(names) - set(dymu.FIM_SYMBOLS)


def test_planner_exports_every_declared_symbol(dymu):
    lib = dymu.load_planner()
    names = declared("dymu_planner.h")
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) <= set(dymu.PLANNER_SYMBOLS), set(names) - set(dymu.PLANNER_SYMBOLS)


def test_dist_exports_every_declared_symbol(dymu):
    from dymu import dist

    lib = dist.load_dist()
    names = [n for n in declared("dymu_dist.h")]
    assert len(names) >= 6
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) <= set(dist.DIST_SYMBOLS), set(names) - set(dist.DIST_SYMBOLS)


def test_dist_rejects_bad_arguments(dymu):
    """Argument checks run before any device or RCCL call."""
    from dymu import dist

    lib = dist.load_dist()
    h = ctypes.c_void_p()
    assert lib.dymu_dist_create(ctypes.byref(h), None, 0, b"\0" * 128, 0, 1) == -1
    assert lib.dymu_dist_solve(None, None, None, 0, 8, 8, 0, 0, 0, None, None) == -1
    assert lib.dymu_vdist_solve(None, 2, None, None, 8, 8, 8, 0, 0, 0, None, None) == -1


def test_abi_version_and_strerror(dymu):
    lib = dymu.load_fim()
    assert lib.dymu_abi_version() == 5
    assert lib.dymu_strerror(-4) == b"pass cap reached before convergence"


def _no_gpu(dymu):
    return dymu.device_count() == 0


def test_engine_refuses_without_device(dymu):
    if not _no_gpu(dymu):
        pytest.skip("a GPU is visible")
    with pytest.raises(dymu.DymuError) as e:
        dymu.Engine()
    assert e.value.status == -5


def test_planner_solve_refuses_without_device(dymu):
    if not _no_gpu(dymu):
        pytest.skip("a GPU is visible")
    p = dymu.Planner()
    assert p.initGlobalLayer(1.0, 0.5, 16, 16)
    assert p.setCostMap(np.ones((16, 16)))
    assert p.setGoal((8, 8))
    with pytest.raises(dymu.DymuError) as e:
        p.computeEntireTotalCostMap()
    assert e.value.status == -5


def test_headers_compile_as_c_and_cpp(tmp_path):
    """The C-ABI headers are plain C; DyMu.hpp builds without Rock."""
    c = tmp_path / "t.c"
    c.write_text('#include "dymu_fim.h"\n#include "dymu_planner.h"\n#include "dymu_dist.h"\n'
                 'int main(void){return 0;}\n')
    cc = tmp_path / "t.cpp"
    cc.write_text('#include "DyMu.hpp"\nint main(){PathPlanning_lib::DyMuPathPlanner p(1,1,1,'
                  'PathPlanning_lib::CONSERVATIVE);return 0;}\n')
    inc = os.path.join(ROOT, "include")
    import subprocess
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", inc, "-c", str(c), "-o",
                    str(tmp_path / "t.o")], check=True)
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-I", inc, "-c", str(cc), "-o",
                    str(tmp_path / "t2.o")], check=True)
