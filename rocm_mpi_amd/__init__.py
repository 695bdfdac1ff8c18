"""rocm_mpi_amd — MI355X-native distributed 2D-diffusion stencil framework.

Same capabilities as williamfgc/ROCm-MPI (its diffusion variants, T_eff
metric, ROCm-aware P2P smoke test) and the ImplicitGlobalGrid API it relies
on, re-designed for MI355X: hand-written gfx950 HIP kernels, GPU-direct RCCL
halo exchange over xGMI with comm/compute overlap, one process per GPU.

Public API (ImplicitGlobalGrid names, torch tensors, 0-based indices)::

    me, dims, nprocs, coords, comm = init_global_grid(nx, ny, 1)
    update_halo_(T); gather_(T_nh, T_v); nx_g(); x_g(ix, dx, T); tic(); toc()
    finalize_global_grid()
"""
import os as _os

# RCCL / HIP IPC between the processes of a node need the dmabuf IPC mode on
# this driver (hipIpcGetMemHandle fails with "invalid argument" otherwise;
# scripts/setenv.sh). The HSA runtime reads it when it initialises, so it is
# set on import, before any GPU call, for every entry path (torchrun -m
# rocm_mpi_amd.apps.*, user scripts) and not only through setenv.sh / bench.py.
_os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

from .parallel import (CartTopology, dims_create, finalize_global_grid, gather, gather_,
                       global_grid, grid_is_initialized, init_global_grid, me, nx_g, ny_g, nz_g,
                       tic, toc, update_halo, update_halo_, x_g, y_g, z_g)

__version__ = "0.1.0"

__all__ = [
    "CartTopology", "dims_create", "finalize_global_grid", "gather", "gather_", "global_grid",
    "grid_is_initialized", "init_global_grid", "me", "nx_g", "ny_g", "nz_g", "tic", "toc",
    "update_halo", "update_halo_", "x_g", "y_g", "z_g", "__version__",
]
