"""Direct-store halos: the pipelined K-step kernels store
the cells that are a neighbour's halo straight into the neighbour's output
field (csrc/kernels/stencil_pipe.h, DirectStores; executor set_direct), so a
pass has no pack / send / receive / unpack. Pass counts in device words order
the ranks: pass n waits until every neighbour's frame of pass n - 1 is done.

Every case is bitwise equal to the exchange path / the 1-rank run of the same
global grid (reference semantics: update_halo! in the time loop,
scripts/diffusion_2D_perf_hide.jl:94-101, scripts/diffusion_2D_perf.jl:51)."""
import numpy as np
import pytest
import torch

from helpers import run_loopback
from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
from rocm_mpi_amd.parallel import implicit_grid as gg

pytestmark = pytest.mark.gpu


def run_self(n, K, nt, periods, direct, variant="perf_hide", ny=None):
    ny = ny or n
    gg.init_global_grid(n, ny, 1, periodx=periods[0], periody=periods[1], quiet=True,
                        overlaps=(2 * K, 2 * K, 2), halowidths=(K, K, 1))
    m = Diffusion2D(DiffusionConfig(variant=variant, nx=n, ny=ny, nt=nt, init="random",
                                    quiet=True, periods=(*periods, 0), temporal=K, fast_math=True,
                                    halo_direct=direct))
    try:
        m.step(nt)
        f = m.field.cpu().numpy().copy()
        info = (m.executor.direct, m.executor.direct_passes, m.executor.passes_done)
    finally:
        m.close()
        gg.finalize_global_grid()
    return f, info


@pytest.mark.parametrize("periods", [(1, 1), (1, 0), (0, 1)])
@pytest.mark.parametrize("K,n,nt", [(24, 1028, 61), (8, 516, 37), (20, 2052, 45)])
def test_direct_self_periodic_equals_exchange(periods, K, n, nt):
    """One rank, periodic: the kernel stores its own periodic images (one
    launch per pass, no exchange) == local self copies after each pass. A
    single rank stores only on passes of one wave of tasks (beyond, its local
    copies cost less than the direct-store kernel's row loop): every pass of
    the small tiles, some of the 2052^2 K=20 plan's."""
    a, (da, dp, npass) = run_self(n, K, nt, periods, True)
    b, (db, _, _) = run_self(n, K, nt, periods, False)
    assert da and not db and npass >= 2 and 1 <= dp <= npass
    if n <= 1028:
        assert dp == npass
    assert np.array_equal(a, b)


def test_direct_self_perf_variant():
    a, (da, _, _) = run_self(1028, 16, 40, (1, 1), True, variant="perf")
    b, _ = run_self(1028, 16, 40, (1, 1), False, variant="perf")
    assert da and np.array_equal(a, b)


def spmd(rank, hub, nx, ny, nt, dims, periods, K, direct):
    gg.init_global_grid(nx, ny, 1, dimx=dims[0], dimy=dims[1], periodx=periods[0],
                        periody=periods[1], overlaps=(2 * K, 2 * K, 2), halowidths=(K, K, 1),
                        quiet=True, loopback=(hub, rank))
    m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=nx, ny=ny, nt=nt, init="random",
                                    quiet=True, dims=dims, periods=(*periods, 0), temporal=K,
                                    fast_math=True, halo_direct=direct))
    try:
        plan = list(m.executor.plan(nt))
        geos = {k: m.executor.geometry(k) for k in set(plan)}

        def fusable(g):  # aligned frames around a non-empty interior
            x0, x1, y0, y1 = g["interior"]
            return g["aligned"] and x1 > x0 and y1 > y0 and any(
                r[1] > r[0] and r[3] > r[2] for r in g["frame"])

        # direct mode fuses only with other ranks and more than one wave of
        # tasks (one-wave tiles: one launch per pass)
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        want = sum(1 for k in plan if fusable(geos[k]) and geos[k]["tasks"] > 2 * cus)
        m.step(nt)
        m.synchronize()
        out = (m.g.coords, m.field.cpu().numpy().copy(), m.g.nxyz_g,
               (m.executor.direct, m.executor.direct_passes, m.executor.fused_passes, want))
    finally:
        m.close()
        gg.finalize_global_grid()
    return out


@pytest.mark.parametrize("dims,periods,K,nx,ny,nt,fused", [
    ((2, 2), (0, 0), 24, 1028, 900, 53, "auto"),
    ((2, 2), (1, 1), 24, 1100, 3500, 49, "1"),
    ((2, 1), (1, 0), 24, 3000, 5000, 49, "1"),
    ((2, 2), (1, 0), 8, 516, 400, 29, "0"),
    ((2, 1), (0, 1), 16, 1028, 600, 41, "auto"),
    ((1, 2), (0, 0), 20, 1100, 3000, 47, "1"),
    ((3, 1), (1, 0), 12, 516, 300, 33, "0"),
])
def test_direct_loopback_ranks_equal_one_rank(dims, periods, K, nx, ny, nt, fused, monkeypatch):
    """Rank threads of one process (loopback) storing into each other's
    fields: every tile == its window of the 1-rank run, bitwise, with
    one-launch, fused and split passes; every pass ran in direct mode."""
    P = dims[0] * dims[1]
    monkeypatch.setenv("RMA_EXEC_FUSED", fused)
    res = run_loopback(P, spmd, nx, ny, nt, dims, periods, K, True, timeout=240)
    nxg, nyg, _ = res[0][2]
    ol = 2 * K
    # the 1-rank run of the same global grid (periodic: the tile of the
    # global interior plus its overlap)
    n1x = nxg + ol if periods[0] else nxg
    n1y = nyg + ol if periods[1] else nyg
    monkeypatch.setenv("RMA_EXEC_FUSED", "0")
    one = run_loopback(1, spmd, n1x, n1y, nt, (1, 1), periods, K, False, timeout=240)[0][1]
    for coords, T, _, (direct, dpasses, _, _) in res:
        assert direct and dpasses >= 2, (coords, dpasses)
        gx0, gy0 = coords[0] * (nx - ol), coords[1] * (ny - ol)
        assert np.array_equal(T, one[gy0:gy0 + ny, gx0:gx0 + nx]), coords
    # RMA_EXEC_FUSED=1: every pass with aligned frames and more than one wave
    # of tasks ran fused (frame tasks first, counts raised at their flag);
    # one-wave tiles ran one launch per pass; 0: never fused
    if fused == "1":
        assert all(r[3][2] == r[3][3] for r in res), [r[3] for r in res]
        assert nx * ny < 10**7 or all(r[3][2] > 0 for r in res)  # the big case fuses
    if fused == "0":
        assert all(r[3][2] == 0 for r in res), [r[3] for r in res]


def test_direct_refuses_canonical_passes():
    """halo_direct needs the fast-math pipelined passes (the only kernels
    with direct-store variants)."""
    gg.init_global_grid(516, 516, 1, periodx=1, periody=1, quiet=True, overlaps=(16, 16, 2),
                        halowidths=(8, 8, 1))
    try:
        with pytest.raises(ValueError, match="fast-math"):
            Diffusion2D(DiffusionConfig(variant="perf_hide", nx=516, ny=516, nt=8, quiet=True,
                                        periods=(1, 1, 0), temporal=8, fast_math=False,
                                        halo_direct=True))
    finally:
        gg.finalize_global_grid()


@pytest.mark.parametrize("dims,periods,K,nx,ny,nt", [
    ((2, 2), (0, 0), 8, 260, 200, 29),
    ((2, 2), (1, 1), 24, 1100, 1200, 53),
    ((2, 1), (1, 0), 16, 516, 300, 35),
])
def test_direct_ipc_processes_equal_the_exchange(tmp_path, dims, periods, K, nx, ny, nt):
    """Separate processes sharing cuda:0: every rank's kernels store its
    neighbours' halos straight into their fields, mapped once through HIP IPC
    (IpcMap: T, T2 and the pass-count words of each peer). Every tile ==
    the same processes' run with the IPC halo exchange, bitwise; every pass ran
    direct and each peer's allocations were opened once."""
    from helpers import run_procs

    P = dims[0] * dims[1]
    env = {"RMA_TRANSPORT": "ipc", "RMA_IPC_MAILBOX_MB": "2"}
    out = {}
    for direct in (1, 0):
        d = tmp_path / f"d{direct}"
        d.mkdir()
        run_procs(P, "mp_targets:direct_tiles", str(d), nx, ny, nt, dims, periods, K, direct,
                  env=env, timeout=240)
        out[direct] = [(open(d / f"meta{r}.txt").read().split(), np.load(d / f"tile{r}.npy"))
                       for r in range(P)]
    for (ma, a), (mb, b) in zip(out[1], out[0]):
        assert ma[:3] == mb[:3] and ma[2] == "ipc"
        on, dpasses, npass, maps = map(int, ma[3:])
        assert on == 1 and dpasses == npass >= 2 and maps >= 1, ma
        assert int(mb[3]) == 0
        assert np.array_equal(a, b), ma[:2]


def test_entry_point_runs_direct_halos():
    """The reference-named perf_hide entry point with --halo-direct on a
    periodic single-rank grid: runs, reports, and its field equals the same
    run without direct stores (checkpointed tiles compared bitwise)."""
    import json
    import os
    import subprocess
    import sys
    import tempfile

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for direct in (True, False):
            ck = os.path.join(td, f"ck{int(direct)}")
            cmd = [sys.executable, "-m", "rocm_mpi_amd.apps.diffusion_2D_perf_hide", "--nx", "1028",
                   "--ny", "1028", "--nt", "60", "--temporal", "24", "--periods", "1,1",
                   "--no-vis", "--json", "--quiet", "--checkpoint", ck]
            if direct:
                cmd.append("--halo-direct")
            r = subprocess.run(cmd, capture_output=True, text=True, cwd=root, timeout=240,
                               env=dict(os.environ, RMA_AUTOBUILD="0"))
            assert r.returncode == 0, r.stderr[-3000:]
            rec = json.loads(r.stdout.strip().splitlines()[-1])
            assert rec["nt"] == 60
            out[direct] = np.load(os.path.join(ck, "rank0.npy"), allow_pickle=False)
    assert np.array_equal(out[True], out[False])
