"""Domain decomposition: topology, implicit global grid, halo exchange, comm."""
from .comm import (Communicator, LoopbackComm, LoopbackHub, P2P, RcclComm, SelfComm,
                   TorchDistComm)
from .implicit_grid import (GlobalGrid, finalize_global_grid, global_grid, grid_is_initialized,
                          init_global_grid, me, nx_g, ny_g, nz_g, tic, toc, x_g, y_g, z_g)
from .halo import gather, gather_, update_halo, update_halo_
from .topology import CartTopology, dims_create

__all__ = [
    "Communicator", "LoopbackComm", "LoopbackHub", "P2P", "RcclComm", "SelfComm",
    "TorchDistComm", "GlobalGrid", "finalize_global_grid", "global_grid", "grid_is_initialized",
    "init_global_grid", "me", "nx_g", "ny_g", "nz_g", "tic", "toc", "x_g", "y_g", "z_g",
    "gather", "gather_", "update_halo", "update_halo_", "CartTopology", "dims_create",
]
