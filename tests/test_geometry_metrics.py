"""Implicit-global-grid geometry, T_eff metric and reference output format."""
import math

import pytest
import torch

import rocm_mpi_amd as rma
from rocm_mpi_amd.parallel import geometry as geo
from rocm_mpi_amd.utils import metrics


def test_nx_g_formula():
    assert geo.n_global(128, 2, 2, 0) == 254  # docs/Temp_4_252_252.png: (254-2) = 252
    assert geo.n_global(128, 2, 2, 1) == 252
    assert geo.n_global(12288, 1, 2, 0) == 12288


def test_single_rank_grid_and_x_g():
    me, dims, nprocs, coords, comm = rma.init_global_grid(10, 8, 1, quiet=True,
                                                          select_device=False)
    assert (me, tuple(dims), nprocs, tuple(coords)) == (0, (1, 1, 1), 1, (0, 0, 0))
    assert rma.nx_g() == 10 and rma.ny_g() == 8 and rma.nz_g() == 1
    T = torch.zeros(8, 10)
    assert rma.x_g(3, 0.5, T) == 1.5
    Vx = torch.zeros(8, 11)  # staggered in x: x0 = -dx/2
    assert rma.x_g(0, 0.5, Vx) == -0.25
    rma.tic()
    assert rma.toc() >= 0


def test_periodic_x_g_wraps():
    rma.init_global_grid(10, 8, 1, periodx=1, quiet=True, select_device=False)
    assert rma.nx_g() == 8
    T = torch.zeros(8, 10)
    d = 1.0
    assert rma.x_g(0, d, T) == 7.0  # first cell is a ghost of the last
    assert rma.x_g(1, d, T) == 0.0
    assert rma.x_g(9, d, T) == 0.0


def test_teff_formula_and_line():
    # 12288^2 fp64, 990 timed steps in 10 s -> A_eff = 3*12288^2*8/1e9
    a = metrics.a_eff_gb(12288, 12288)
    assert a == pytest.approx(3 * 12288 ** 2 * 8 / 1e9)
    t = metrics.t_eff(12288, 12288, 10.0, 990)
    assert t == pytest.approx(a / (10.0 / 990))
    line = metrics.reference_line(1000, 10.0, 1234.5678)
    assert line == "Executed 1000 steps in = 1.000e+01 sec (@ T_eff = 1230.00 GB/s) "
    assert metrics.round_sig(0.0012345, 3) == 0.00123
    assert math.isnan(metrics.t_eff(4, 4, 1.0, 0))
    assert metrics.weak_scaling_efficiency(95.0, 100.0) == pytest.approx(0.95)


def test_grid_validation():
    with pytest.raises(ValueError):
        rma.init_global_grid(3, 8, 1, quiet=True, select_device=False, overlaps=(4, 2, 2))
    with pytest.raises(ValueError):
        rma.init_global_grid(8, 8, 1, dimz=2, quiet=True, select_device=False)
