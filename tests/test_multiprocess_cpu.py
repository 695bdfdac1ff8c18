"""Real multi-process runs over torch.distributed/gloo (world_size 2 and 4).

The same SPMD code that runs one rank per MI355X over RCCL, here with CPU
tensors: decomposition invariance against the global NumPy golden model, the
T_eff reference protocol, collectives, and the ring P2P smoke test
(scripts/rocmaware_test_selectdevice.jl)."""
import os

import numpy as np
import pytest

import golden
from helpers import run_procs


@pytest.mark.parametrize("variant,world,dims", [("perf_hide", 2, (2, 1)), ("kp", 2, (1, 2)),
                                                ("perf", 4, (2, 2)), ("ap", 4, (4, 1))])
def test_gloo_decomposition_invariance(tmp_path, variant, world, dims):
    nx, ny, nt = 40, 36, 30
    run_procs(world, "mp_targets:diffusion", str(tmp_path), variant, nx, ny, nt, dims)
    Tv = np.load(tmp_path / "Tv.npy")
    nxg, nyg, transport, teff, timed = open(tmp_path / "meta.txt").read().split()
    assert transport == "gloo" and int(timed) == nt - 10 and float(teff) > 0
    G = golden.run(int(nxg), int(nyg), nt)
    assert np.array_equal(Tv, G[1:-1, 1:-1])


@pytest.mark.parametrize("world,dims", [(2, (2, 1)), (4, (2, 2))])
def test_user_example_matches_golden(tmp_path, world, dims):
    """examples/diffusion_2D_user.py (the user's own loop over the IGG API,
    stencil_step + update_halo_ per step) on gloo ranks == the golden model."""
    nx, ny, nt = 40, 36, 30
    run_procs(world, "mp_targets:user_example", str(tmp_path), nx, ny, nt, dims)
    nxg, nyg = dims[0] * (nx - 2) + 2, dims[1] * (ny - 2) + 2
    G0 = golden.initial_torch(nxg, nyg)
    assert np.array_equal(np.load(tmp_path / "T0.npy"), G0[1:-1, 1:-1])
    assert np.array_equal(np.load(tmp_path / "T.npy"), golden.run(nxg, nyg, nt, T0=G0)[1:-1, 1:-1])


def test_ring_sendrecv(tmp_path):
    run_procs(3, "mp_targets:ring", str(tmp_path))
    for r in range(3):
        v = np.load(tmp_path / f"ring{r}.npy")
        assert np.all(v == (r - 1) % 3)


def test_collectives_and_timers(tmp_path):
    run_procs(2, "mp_targets:collectives", str(tmp_path))
    for r in range(2):
        s, mx, t, n, d0, d1, d2 = np.load(tmp_path / f"coll{r}.npy")
        assert s == 3 and mx == 1 and t >= 0 and n == 2 and (d0, d1, d2) == (2, 1, 1)


@pytest.mark.parametrize("variant,K", [("perf_hide", 3), ("perf", 4)])
def test_gloo_temporal_blocking_tiles(tmp_path, variant, K):
    """2 processes over gloo, K steps per pass with width-K halos (overlap
    2K): every tile equals its window of the global golden model."""
    import torch

    from rocm_mpi_amd import ops

    nx, ny, nt = 40, 31, 23
    run_procs(2, "mp_targets:diffusion_tiles", str(tmp_path), variant, nx, ny, nt, (2, 1), K)
    metas = [open(tmp_path / f"meta{r}.txt").read().split() for r in range(2)]
    nxg, nyg = int(metas[0][2]), int(metas[0][3])
    assert (nxg, nyg) == (2 * (nx - 2 * K) + 2 * K, ny) and metas[0][6] == "gloo"
    T0 = torch.empty((nyg, nxg), dtype=torch.float64)
    ops.init_random_(T0, ops.TileGeometry(0, 0, nxg, nyg, 1.0, 1.0), seed=1234)
    G = golden.run(nxg, nyg, nt, T0=T0.numpy())
    for r in range(2):
        cx, cy, ol = int(metas[r][0]), int(metas[r][1]), int(metas[r][4])
        T = np.load(tmp_path / f"tile{r}.npy")
        gx0, gy0 = cx * (nx - ol), cy * (ny - ol)
        assert np.array_equal(T, G[gy0:gy0 + ny, gx0:gx0 + nx])


@pytest.mark.parametrize("world,extra", [(2, ["--temporal", "4", "--dims", "2,1"]),
                                         (4, ["--temporal", "16", "--dims", "2,2"]),
                                         (8, ["--temporal", "16", "--dims", "4,2"])])
def test_bench_driver_contract_multirank(tmp_path, world, extra):
    """bench.py's multi-rank path (the driver runs it under torch.distributed.run
    at N = 2, 4, 8) on the CPU twins over gloo: rank 0 prints ONE JSON line with
    the contract's keys, n_gpus == WORLD_SIZE, value == N x per-rank T_eff,
    weak scaling (same local tile), the global grid of a dims decomposition, and
    exit status 0 on every rank (teardown through comm.shutdown_distributed)."""
    import json
    import subprocess
    import sys

    from helpers import free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    nx = 72
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.join(root, "bench.py"),
           "--gpus", str(world), "--steps", "20", "--warmup", "3", "--device", "cpu",
           "--nx", str(nx), "--single-step-steps", "4", *extra]
    K = int(extra[1])
    # the N = 1 record of this tile class, as the driver's N = 1 run of the
    # same sweep leaves it (bench.py save_n1): e_box is then defined. The
    # in-run attribution (e_gpu included) must not need it:
    # the 4-rank case runs without any cache file.
    import bench

    cache = tmp_path / "n1.json"
    n1_ms = 1.0 if world != 4 else None
    if n1_ms:
        cache.write_text(json.dumps({"key": bench._n1_key(nx, nx, 20, 3, K, True, "perf_hide"),
                                     "ms_per_step": n1_ms, "pci_bus_id": "cpu"}))
    env = dict(os.environ, OMP_NUM_THREADS="1", RMA_DIAG=f"bench_n1_cache={cache}")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path),
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["n_gpus"] == world and d["steps"] == 20 and d["warmup"] == 3
    assert d["scaling"] == "weak" and d["higher_is_better"] is True
    c = d["config"]
    assert c["local_grid"] == [nx, nx]
    dims = [int(v) for v in extra[3].split(",")]
    assert c["global_grid"] == [dims[0] * (nx - 2 * K) + 2 * K, dims[1] * (nx - 2 * K) + 2 * K]
    assert abs(d["value"] - world * c["teff_per_gpu_GBps"]) <= 1e-6 * d["value"] + 0.005 * world + 0.01
    assert c["full_field_check"]["ok"] and c["full_field_check"]["nonfinite"] == 0
    # self-validation of a multi-rank point
    assert c["ranks"] == world and c["transport"] == "gloo"
    assert sum(c["passes_timed"]) == 20 and max(c["passes_timed"]) <= K
    assert c["fast_math"] is True  # the timed passes, not the canonical side run after them
    # per-rank own (pre-barrier) times: the job time is the slowest rank's
    assert c["teff_per_gpu_GBps"] <= c["teff_per_gpu_min_GBps"] * (1 + 1e-9) + 0.02
    assert c["teff_per_gpu_min_GBps"] <= c["teff_per_gpu_max_GBps"]
    pt = c["pass_timing"]
    assert pt["passes"] == len(c["passes_timed"])
    for k in ("frame_ms", "halo_ms", "interior_ms", "pass_ms", "exposed_halo_ms"):
        assert pt[k] >= 0
    assert pt["halo_ms"] > 0 and pt["overlap_fraction"] is not None
    assert 0 < c["weak_scaling_eff_same_run"] and c["solo_ms_per_step"] > 0
    # every rank's detail
    rd = c["ranks_detail"]
    assert [r["rank"] for r in rd] == list(range(world))
    assert sorted(tuple(r["coords"]) for r in rd) == sorted(
        (x, y) for x in range(dims[0]) for y in range(dims[1]))
    assert len({r["pci_bus_id"] for r in rd}) == world
    for r in rd:
        assert r["ms_per_step"] > 0 and r["solo_ms_per_step"] > 0
        assert r["ms_per_step"] <= d["ms_per_step"] * (1 + 1e-6) + 1e-6
        assert r["pass_timing"]["passes"] == len(c["passes_timed"])
        assert r["pass_timing"]["halo_ms"] > 0
    assert min(r["teff_GBps"] for r in rd) == c["teff_per_gpu_min_GBps"]
    assert max(r["teff_GBps"] for r in rd) == c["teff_per_gpu_max_GBps"]
    assert rd[c["slowest_rank"]]["ms_per_step"] == max(r["ms_per_step"] for r in rd)
    # preflight ring + tiny halo check before the tile, then the in-run checks
    assert c["preflight"]["ring_ok"] is True
    assert c["preflight"]["halo"]["tiles_mismatched"] == 0
    assert c["rccl_halo_bitwise_ok"] is True
    hc = c["halo_check"]
    assert hc["tiles_mismatched"] == 0 and hc["transport"] == "gloo"
    assert hc["global_grid"] == [dims[0] * (130 - 2 * K) + 2 * K, dims[1] * (130 - 2 * K) + 2 * K]
    dc = c["drift_check"]
    assert dc["steps"] == 23 and 0 <= c["fast_math_drift_max"] <= dc["bound"]
    # the timed field itself: three full-width row windows vs the CPU twin
    wc = c["headline_window_check"]
    assert wc["windows"] == 3 and wc["bitwise"] is True and wc["steps"] == 23
    assert wc["full_width"] is True and wc["boxes"] == 3
    # E(N) attribution: value is the aggregate
    assert d["value_kind"] == "aggregate"
    assert abs(d["teff_per_gpu"] - c["teff_per_gpu_GBps"]) <= 0.01
    ea = c["e_attribution"]
    for k in ("e_halo", "e_coef", "e_gpu", "e_product", "weak_scaling_eff_same_run_iso",
              "fastest_solo_iso_ms_per_step"):
        assert ea[k] is not None and ea[k] > 0, k
    assert abs(ea["e_halo"] - c["weak_scaling_eff_same_run"]) <= 1e-4
    assert abs(ea["e_halo"] * ea["e_coef"] - ea["weak_scaling_eff_same_run_iso"]) <= 1e-5
    t_it = d["ms_per_step"]
    fast = ea["fastest_solo_iso_ms_per_step"]
    assert fast == min(r["solo_iso_ms_per_step"] for r in rd)
    slow = max(r["solo_iso_ms_per_step"] for r in rd)
    assert 0 < ea["e_gpu"] <= 1 + 1e-9
    assert abs(ea["e_gpu"] - fast / slow) <= 1e-4 * ea["e_gpu"]
    assert abs(ea["e_product"] - ea["e_halo"] * ea["e_coef"] * ea["e_gpu"]) <= 1e-5
    # the product is the in-run efficiency up to the barrier time in the job's
    # solo_iso (max over ranks incl. the closing barrier) vs the slowest own time
    assert abs(ea["e_product"] - fast / t_it * c["solo_iso_ms_per_step"] / slow) <= 1e-3 * max(
        1.0, ea["e_product"])
    if n1_ms:
        assert abs(ea["e_box"] - n1_ms / fast) <= 1e-4 * ea["e_box"]
        assert abs(ea["e_product_vs_n1"] - ea["e_box"] * ea["e_product"]) <= 1e-5
    else:
        assert ea["e_box"] is None and ea["e_product_vs_n1"] is None
    if dims[0] == dims[1]:  # dx == dy: the isotropic re-time IS the solo time
        assert ea["e_coef"] == 1.0 and c["solo_iso_ms_per_step"] == c["solo_ms_per_step"]
    for r in rd:
        assert r["solo_iso_ms_per_step"] > 0 and r["e_halo"] > 0 and r["e_coef"] > 0
        assert abs(r["e_gpu"] - fast / r["solo_iso_ms_per_step"]) <= 1e-4 * r["e_gpu"]
        if n1_ms:
            assert abs(r["e_gpu_vs_n1"] - n1_ms / r["solo_iso_ms_per_step"]) <= 1e-4 * r["e_gpu_vs_n1"]
    assert c["rccl_nranks"] is None and c["preflight"]["ring_transport"] == "gloo"


def test_bench_window_check_detects_a_wrong_cell(tmp_path):
    """The headline window check compares the timed field itself: one
    perturbed cell in the last rank's snapshot fails the run (exit 4) with
    headline_window_check.bitwise false."""
    import json
    import subprocess
    import sys

    from helpers import free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "12", "--warmup", "2",
           "--device", "cpu", "--nx", "64", "--temporal", "4", "--dims", "2,1",
           "--single-step-steps", "0", "--check", "0", "--drift-steps", "0"]
    env = dict(os.environ, OMP_NUM_THREADS="1",
               RMA_DIAG=f"bench_window_corrupt,bench_n1_cache={tmp_path / 'none.json'}")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path),
                       env=env)
    assert r.returncode != 0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout + r.stderr[-2000:]
    d = json.loads(lines[0])
    wc = d["config"]["headline_window_check"]
    assert wc["bitwise"] is False and "1: window rows" in wc["error"]
    assert d["config"]["e_attribution"]["e_box"] is None  # no N = 1 record cached
    assert d["config"]["e_attribution"]["e_gpu"] is not None  # in-run: needs no record


def test_bench_halo_check_detects_a_wrong_tile(tmp_path):
    """The in-run check compares every gathered tile bitwise with the 1-rank
    run: one perturbed cell on the last rank makes the run fail (exit 4) with
    rccl_halo_bitwise_ok false."""
    import json
    import subprocess
    import sys

    from helpers import free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "8", "--warmup", "2",
           "--device", "cpu", "--nx", "64", "--single-step-steps", "0", "--temporal", "4",
           "--solo-steps", "0"]
    env = dict(os.environ, OMP_NUM_THREADS="1", RMA_DIAG="bench_check_corrupt")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path),
                       env=env)
    assert r.returncode != 0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout + r.stderr[-2000:]
    c = json.loads(lines[0])["config"]
    assert c["rccl_halo_bitwise_ok"] is False and c["halo_check"]["tiles_mismatched"] == 1


@pytest.mark.parametrize("where,tmo", [("after", 60), ("before", 8)])
def test_bench_check_exception_fails_every_rank(tmp_path, where, tmo):
    """A check that raises on one rank fails the run on EVERY rank (VERDICT r2
    next 1b): 'after' the check grid ran, the ranks agree through a bounded
    status exchange; 'before' it, the peers block in the halo exchange and the
    check-phase watchdog (3 x --check-timeout) ends them. Either way rank 0
    prints the record with rccl_halo_bitwise_ok false and the error."""
    import json
    import subprocess
    import sys
    import time

    from helpers import free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rcdir = tmp_path / "rc"
    rcdir.mkdir()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "8", "--warmup", "2",
           "--device", "cpu", "--nx", "64", "--single-step-steps", "0", "--temporal", "4",
           "--solo-steps", "0", "--drift-steps", "0", "--check-timeout", str(tmo)]
    env = dict(os.environ, OMP_NUM_THREADS="1",
               RMA_DIAG=f"bench_check_raise={where},bench_rc_dir={rcdir}")
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path),
                       env=env)
    assert r.returncode != 0
    assert time.time() - t0 < 3 * tmo + 60
    rcs = {p.name: int(p.read_text()) for p in rcdir.iterdir() if p.name.startswith("rc")}
    assert set(rcs) == {"rc0", "rc1"} and all(v != 0 for v in rcs.values()), rcs
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout + r.stderr[-2000:]
    d = json.loads(lines[0])
    assert "error" in d
    c = d["config"]
    if where == "after":
        assert c["rccl_halo_bitwise_ok"] is False
        assert "injected" in c["halo_check"]["error"] and "rank(s) 1" in d["error"]
    else:
        assert "watchdog" in d["error"]


def test_bench_preflight_runs_before_the_tile(tmp_path):
    """One CPU rank: the preflight ring + tiny halo check and the drift bound
    are in the record, the halo check is off by default without a GPU."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "30",
                        "--warmup", "3", "--device", "cpu", "--nx", "80", "--temporal", "6",
                        "--single-step-steps", "0"], capture_output=True, text=True,
                       timeout=300, cwd=str(tmp_path), env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    c = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])["config"]
    assert c["preflight"]["ring_ok"] is True and c["preflight"]["halo"]["tiles_mismatched"] == 0
    assert c["halo_check"] is None and c["rccl_halo_bitwise_ok"] is None
    assert c["weak_scaling_eff_same_run"] is None  # no neighbour: solo is the run
    assert c["drift_check"]["steps"] == 33 and c["fast_math_drift_max"] <= 1e-14
    assert c["ranks_detail"][0]["rank"] == 0


def test_node_local_rank_from_hostnames(tmp_path):
    """4 ranks on 2 fake nodes (hostname exchange, no LOCAL_RANK): local ranks
    restart at 0 on every node — the reference's smoke test instead took the
    local rank modulo the GLOBAL size (rocmaware_test_selectdevice.jl:12-13)."""
    run_procs(4, "mp_targets:node_local", str(tmp_path), 2)
    got = [np.load(tmp_path / f"local{r}.npy").tolist() for r in range(4)]
    assert got == [[0, 2, 0, 2], [1, 2, 1, 2], [0, 2, 0, 2], [1, 2, 1, 2]]


def test_slurm_style_environment(tmp_path):
    """Ranks that only see SLURM_PROCID / SLURM_NTASKS / SLURM_LOCALID (srun)
    bootstrap the grid: world from SLURM, node-local ranks from the hostname
    exchange, rendezvous on the default loopback address."""
    run_procs(2, "mp_targets:slurm_env", str(tmp_path))
    got = [np.load(tmp_path / f"slurm{r}.npy").tolist() for r in range(2)]
    assert got == [[0, 2, 0, 2, 1.0], [1, 2, 1, 2, 1.0]]
