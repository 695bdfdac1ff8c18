"""Decomposition invariance on CPU.

P logical ranks (loopback threads) run the distributed problem; the gathered
interior must equal the NumPy golden model of the GLOBAL grid bitwise, for
every variant and several process grids. Includes the reference's own
oracle: 4 ranks x 128^2 (2x2), 1000 steps -> max T = 0.397865
(docs/Temp_4_252_252.png).
"""
import numpy as np
import pytest
import torch

import golden
from helpers import run_loopback
from rocm_mpi_amd import ops
from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
from rocm_mpi_amd.parallel import implicit_grid as gg


def spmd(rank, hub, variant, nx, ny, nt, dims, periods=(0, 0, 0), init="gaussian", bw=(4, 2),
         init_on="host"):
    gg.init_global_grid(nx, ny, 1, dimx=dims[0], dimy=dims[1], periodx=periods[0],
                        periody=periods[1], quiet=True, loopback=(hub, rank),
                        select_device=False)
    m = Diffusion2D(DiffusionConfig(variant=variant, nx=nx, ny=ny, nt=nt, init=init,
                                    init_on=init_on, b_width=bw, quiet=True, dims=dims,
                                    periods=periods))
    m.step(nt)
    Tv = m.gather_interior()
    out = (Tv.numpy().copy() if Tv is not None else None, m.g.nxyz_g)
    gg.finalize_global_grid()
    return out


@pytest.mark.parametrize("variant", ["ap", "kp", "perf", "perf_hide"])
@pytest.mark.parametrize("P,dims", [(1, (1, 1)), (2, (2, 1)), (2, (1, 2)), (4, (2, 2)),
                                    (8, (4, 2)), (3, (3, 1))])
def test_decomposed_equals_golden(variant, P, dims):
    nx, ny, nt = 34, 30, 40
    res = run_loopback(P, spmd, variant, nx, ny, nt, dims)
    Tv, (nxg, nyg, _) = res[0]
    G = golden.run(nxg, nyg, nt)
    assert Tv.shape == (nyg - 2, nxg - 2)
    assert np.array_equal(Tv, G[1:-1, 1:-1])


def test_reference_oracle_4_ranks_1000_steps():
    """The reference README run: 4 MI50, 2x2 x 128^2, 1000 steps, max ~0.39."""
    res = run_loopback(4, spmd, "perf", 128, 128, 1000, (2, 2))
    Tv, (nxg, nyg, _) = res[0]
    assert (nxg, nyg) == (254, 254) and Tv.shape == (252, 252)  # Temp_4_252_252
    assert float(Tv.max()) == pytest.approx(0.397865, abs=5e-7)
    assert float(Tv.sum()) == pytest.approx(2026.758, abs=5e-3)
    G = golden.run(254, 254, 1000)
    assert np.array_equal(Tv, G[1:-1, 1:-1])


def test_perf_hide_equals_perf_with_random_init():
    a = run_loopback(4, spmd, "perf_hide", 70, 50, 25, (2, 2), init="random", bw=(3, 2))[0][0]
    b = run_loopback(4, spmd, "perf", 70, 50, 25, (2, 2), init="random")[0][0]
    c = run_loopback(1, spmd, "perf", 2 * 70 - 2, 2 * 50 - 2, 25, (1, 1), init="random")[0][0]
    assert np.array_equal(a, b) and np.array_equal(b, c)


def test_periodic_decomposition_invariance():
    # periodic in x: 2 ranks (nx=20) vs 1 rank (nx=38) on the same 36-cell periodic grid
    a = run_loopback(2, spmd, "perf", 20, 16, 30, (2, 1), periods=(1, 0, 0), init="random")[0]
    b = run_loopback(1, spmd, "perf", 2 * (20 - 2) + 2, 16, 30, (1, 1), periods=(1, 0, 0),
                     init="random")[0]
    assert a[1][0] == b[1][0] == 36
    # periodic global grid of 36 cells: the first local cell is a ghost, so the
    # gathered interiors cover global 0..35 in both runs
    ta, tb = a[0], b[0]
    assert ta.shape == tb.shape == (14, 36)
    np.testing.assert_array_equal(ta, tb)


def spmd_tiles(rank, hub, variant, nx, ny, nt, dims, temporal, periods=(0, 0, 0)):
    """Every rank returns (coords, full local field incl. halo, global sizes)."""
    ol = 2 * temporal
    gg.init_global_grid(nx, ny, 1, dimx=dims[0], dimy=dims[1], periodx=periods[0],
                        periody=periods[1], overlaps=(ol, ol, 2),
                        halowidths=(temporal, temporal, 1), quiet=True, loopback=(hub, rank),
                        select_device=False)
    m = Diffusion2D(DiffusionConfig(variant=variant, nx=nx, ny=ny, nt=nt, init="random",
                                    quiet=True, dims=dims, periods=periods, temporal=temporal,
                                    b_width=(1, 1)))
    m.step(nt)
    out = (m.g.coords, m.field.numpy().copy(), m.g.nxyz_g, m.g.overlaps)
    gg.finalize_global_grid()
    return out


@pytest.mark.parametrize("variant", ["perf", "perf_hide"])
@pytest.mark.parametrize("P,dims", [(1, (1, 1)), (2, (2, 1)), (3, (1, 3)), (4, (2, 2))])
@pytest.mark.parametrize("nt,K", [(20, 2), (13, 2), (23, 3), (26, 4)])
def test_temporal_blocking_equals_golden(variant, P, dims, nt, K):
    """K steps per pass + width-K halos on an overlap-2K grid: every local
    tile (halo included) equals its window of the global golden model, also
    when nt is not a multiple of K."""
    nx, ny = 37, 30
    res = run_loopback(P, spmd_tiles, variant, nx, ny, nt, dims, K)
    nxg, nyg, _ = res[0][2]
    assert (nxg, nyg) == (dims[0] * (nx - 2 * K) + 2 * K, dims[1] * (ny - 2 * K) + 2 * K)
    T0 = torch.empty((nyg, nxg), dtype=torch.float64)  # the global random field
    ops.init_random_(T0, ops.TileGeometry(0, 0, nxg, nyg, 1.0, 1.0), seed=1234)
    G = golden.run(nxg, nyg, nt, T0=T0.numpy())
    for coords, T, _, ol in res:
        gx0, gy0 = coords[0] * (nx - ol[0]), coords[1] * (ny - ol[1])
        assert np.array_equal(T, G[gy0:gy0 + ny, gx0:gx0 + nx])
