"""bench.py --gpus N means N ranks (VERDICT r1 "do this" 2, ADVICE r1 bench.py:157).

* Without a launcher, `bench.py --gpus 2` spawns 2 rank processes itself
  (torch.distributed.run), and the JSON line reports what the communicator saw
  (`ranks_seen`) and every rank's slab; exercised on CPU with --fake-cpu
  (gloo, numpy stand-in engine), whose gathered map must equal the oracle FMM.
* A launcher world that disagrees with --gpus fails before anything runs."""
import glob
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(kw)
    return env


def test_bench_gpus2_spawns_two_ranks(oracle, tmp_path):
    n = 96
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--fake-cpu", "--size", str(n), "--steps", "1", "--warmup", "0",
                          "--obst", "0.05"],
                         env=_env(DYMU_BENCH_DUMP=str(tmp_path)), cwd=ROOT, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2
    assert rec["config"]["ranks_seen"] == 2
    slabs = rec["config"]["slabs"]
    assert [s[0] for s in slabs] == [0, 1]
    assert slabs[0][1] == 0 and slabs[0][1] + slabs[0][2] == slabs[1][1]
    assert slabs[1][1] + slabs[1][2] == n
    # the run's own check of its stitched map (bench_sharded.self_check)
    par = rec["parity"]
    assert par["ok"] and par["residual"] <= 1e-12 and par["sum_rel"] <= 1e-12
    assert par["finite_cells"] == par["finite_cells_single"] and par["ghost_max_abs_diff"] == 0
    T = np.empty((n, n))
    files = glob.glob(str(tmp_path / "T_rank*_row*.npy"))
    assert len(files) == 2
    for f in files:
        row0 = int(f.rsplit("_row", 1)[1].split(".")[0])
        part = np.load(f)
        T[row0:row0 + part.shape[0]] = part
    g = (n // 2, n // 2)
    F = oracle.synth_speed(n, n, seed=1, obst_frac=0.05, obst_seed=3, goal=g)
    Tref, _ = oracle.fmm(F, g)
    fin = np.isfinite(Tref)
    assert np.array_equal(np.isfinite(T), fin)
    assert (np.abs(T[fin] - Tref[fin]) / np.maximum(1, Tref[fin])).max() <= 1e-12


def test_bench_world_mismatch_fails():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--fake-cpu", "--size", "64"],
                         env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"), cwd=ROOT,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode != 0
    assert "WORLD_SIZE=3" in out.stderr


@pytest.mark.gpu
def test_bench_gpus2_one_gpu_transport_choice_self_check():
    """The multi-GPU bench path end to end on the one GPU of a test box: `bench.py
    --gpus 2` spawns two ranks (torch.distributed.run), both on device 0, and --
    before the timed region -- times every candidate transport x passes per round:
    IPC (RCCL refuses two ranks on one GPU; on a node with a GPU per rank the
    candidate is RCCL) against the GPU-initiated peer transport.  The line carries
    both candidates' times and the choice, and the run's self-check (slab residual,
    ghost rows, sum / count vs a single-GPU solve) must pass -- the code the
    driver's N-GPU run executes."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--size", "2048", "--steps", "2", "--warmup", "1", "--cpu-sample", "0"],
                         env=_env(DYMU_DIST_TIMEOUT_S="60"), cwd=ROOT, capture_output=True,
                         text=True, timeout=280)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["n_gpus"] == 2 and rec["config"]["ranks_seen"] == 2
    par = rec["parity"]
    assert par["ok"] and par["ghost_max_abs_diff"] == 0 and par["mismatched_cells"] == 0
    assert par["finite_cells"] == par["finite_cells_single"] > 0.9 * 2048 * 2048
    # every candidate timed, the fastest (transport, K) kept (bench_sharded.K_CANDIDATES)
    tune = rec["config"]["k_autotune_ms"]
    assert sorted(tune) == ["ipc", "peer"]
    for tr in tune:
        assert sorted(int(k) for k in tune[tr]) == [2, 4, 8] and min(tune[tr].values()) > 0
    best = min(((tr, int(k)) for tr in tune for k in tune[tr]),
               key=lambda c: tune[c[0]][str(c[1])])
    assert (rec["config"]["transport"], rec["config"]["passes_per_exchange"]) == best


@pytest.mark.gpu
def test_bench_gpus2_candidate_failure_dropped_with_reason():
    """A candidate transport that fails while the bench times the candidates (here
    forced on rank 1 by DYMU_BENCH_FAIL_CANDIDATE) is dropped on every rank with its
    reason, under the tuning's short wait bound, and the line still prints with the
    other transport and a passing self-check (VERDICT r4 "do this" 4)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--size", "1024", "--steps", "1", "--warmup", "1", "--cpu-sample", "0"],
                         env=_env(DYMU_DIST_TIMEOUT_S="60", DYMU_BENCH_FAIL_CANDIDATE="peer:1"),
                         cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    cfg = rec["config"]
    assert cfg["transport"] == "ipc" and rec["parity"]["ok"]
    assert "peer" in cfg["transports_dropped"] and "timing" in cfg["transports_dropped"]["peer"]
    assert sorted(cfg["k_autotune_ms"]) == ["ipc"]


@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["ipc", "peer"])
def test_bench_gpus2_fixed_transport_self_check(exchange):
    """`--exchange ipc|peer` runs that transport only, with its self-check."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--exchange", exchange, "--size", "1024", "--steps", "2", "--warmup",
                          "1", "--cpu-sample", "0", "--passes-per-exchange", "4"],
                         env=_env(DYMU_DIST_TIMEOUT_S="60"), cwd=ROOT, capture_output=True,
                         text=True, timeout=280)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["config"]["transport"] == exchange and rec["parity"]["ok"]
    assert rec["config"]["passes_per_exchange"] == 4


@pytest.mark.gpu
def test_bench_single_gpu_oracle_parity():
    """The single-GPU bench line checks its whole map against the cpu_baseline's
    oracle FMM map of the same grid (bench.oracle_parity) and carries the block."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--size", "1024",
                          "--cpu-sample", "1024", "--cpu-linear-size", "256", "--steps", "2",
                          "--warmup", "1", "--no-variants", "--no-planner"],
                         env=_env(), cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    par = rec["parity"]
    assert par["ok"] and par["mismatched_cells"] == 0 and par["max_rel"] <= 1e-12
    assert par["finite_cells"] > 0.9 * 1024 * 1024
    assert rec["cpu_baseline"]["sample"].startswith("1024x1024")
