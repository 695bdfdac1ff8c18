"""Implicit global grid: the ImplicitGlobalGrid.jl API used by the reference.

Call sites in the reference (all five diffusion scripts, e.g.
``scripts/diffusion_2D_ap.jl``): ``init_global_grid(nx,ny,1)`` (:17),
``nx_g()/ny_g()`` (:19), ``x_g/y_g`` (:28), ``update_halo!(T)`` (:42),
``gather!(T_nh,T_v)`` (:46), ``finalize_global_grid()`` (:48), ``tic()/toc()``
(``diffusion_2D_perf.jl:48,53``). SURVEY.md C14-C19.

Python naming: ``update_halo_`` / ``gather_`` (trailing underscore = in-place,
torch style) with ``update_halo`` / ``gather`` aliases. Local indices are
0-based (IGG's ``ix`` = ours + 1). Fields are torch tensors laid out
``(ny, nx)`` / ``(nz, ny, nx)`` with x fastest, i.e. the same memory as the
Julia column-major ``A[ix,iy,iz]``.

State is per process (like IGG) with a thread-local override so several
logical ranks can live in one process (loopback transport).
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass, field
from typing import Sequence

import torch

from ..config import diag_flag
from . import comm as C
from . import geometry as geo
from .topology import CartTopology, dims_create

_global: "GlobalGrid | None" = None
_tls = threading.local()


@dataclass
class GlobalGrid:
    nxyz: tuple  # local (nx, ny, nz), halo included
    nxyz_g: tuple  # global sizes
    dims: tuple
    overlaps: tuple
    halowidths: tuple
    periods: tuple
    nprocs: int
    me: int
    coords: tuple
    neighbors: tuple  # ((xlo,xhi),(ylo,yhi),(zlo,zhi)), -1 = none
    disp: int
    reorder: int
    comm: C.Communicator
    device: torch.device
    transport: str
    quiet: bool = False
    local_rank: int = 0
    local_size: int = 1
    owns_dist: bool = False
    halo: object = None  # native HaloExchanger (GPU transports)
    topo: object = None
    t0: float | None = None
    extra: dict = field(default_factory=dict)

    # convenience -----------------------------------------------------------
    @property
    def nx(self):
        return self.nxyz[0]

    @property
    def ny(self):
        return self.nxyz[1]

    @property
    def nz(self):
        return self.nxyz[2]

    def describe(self) -> str:
        g = self.nxyz_g
        d = self.dims
        return (f"Global grid: {g[0]}x{g[1]}x{g[2]} (nprocs: {self.nprocs}, "
                f"dims: {d[0]}x{d[1]}x{d[2]}, transport: {self.transport})")


def _set_grid(g: GlobalGrid | None, thread_local: bool) -> None:
    global _global
    if thread_local:
        _tls.grid = g
    else:
        _global = g


def global_grid() -> GlobalGrid:
    g = getattr(_tls, "grid", None) or _global
    if g is None:
        raise RuntimeError("no global grid: call init_global_grid() first")
    return g


def grid_is_initialized() -> bool:
    return (getattr(_tls, "grid", None) or _global) is not None


def _choose_transport(transport: str, size: int, device: torch.device,
                      local_size: int | None = None) -> str:
    t = os.environ.get("RMA_TRANSPORT", transport)
    legacy = os.environ.get("IGG_ROCMAWARE_MPI")
    if t == "auto" and legacy is not None and device.type == "cuda" and size > 1:
        t = "rccl" if legacy.strip() == "1" else "staged"
    if t == "auto":
        if size == 1:
            return "self"
        return "rccl" if device.type == "cuda" else "gloo"
    if t not in ("rccl", "ipc", "staged", "gloo", "loopback", "self"):
        raise ValueError(f"unknown transport {t!r}")
    if t in ("rccl", "ipc") and device.type != "cuda":
        raise ValueError(f"transport {t!r} needs a GPU device")
    if t == "ipc" and size == 1:
        return "self"
    if t == "ipc" and local_size is not None and local_size != size:
        raise ValueError(f"transport 'ipc' connects the processes of ONE node; {size} ranks "
                         f"span nodes ({local_size} on this one): use rccl")
    return t


def init_global_grid(nx: int, ny: int, nz: int = 1, *, dimx: int = 0, dimy: int = 0,
                     dimz: int = 0, periodx: int = 0, periody: int = 0, periodz: int = 0,
                     overlaps: Sequence[int] = (2, 2, 2), halowidths: Sequence[int] | None = None,
                     disp: int = 1, reorder: int = 1, transport: str = "auto",
                     device: str | torch.device | None = None, select_device: bool = True,
                     quiet: bool = False, init_dist: bool = True,
                     loopback: tuple | None = None,
                     timeout_s: float = C.DEFAULT_TIMEOUT_S,
                     self_via_transport: bool = False):
    """Create the implicit global grid and return ``(me, dims, nprocs, coords, comm)``.

    Mirrors ``ImplicitGlobalGrid.init_global_grid``: MPI-style
    ``Dims_create`` (``nz==1`` forces ``dimz=1``), a row-major Cartesian
    topology (open by default), neighbours by ``Cart_shift``, node-local device
    selection, and the halo transport. ``loopback=(hub, rank)`` creates one
    logical rank of an in-process group (tests); its grid is thread-local and,
    on a GPU, its halo runs through the native engine over the device loopback
    transport (the production code path with RCCL swapped for D2D copies).
    ``self_via_transport`` routes periodic self-neighbours through the P2P
    transport (exercises RCCL send/recv on a single GPU).
    """
    nxyz = (int(nx), int(ny), int(nz))
    if min(nxyz) < 1:
        raise ValueError(f"local sizes must be >= 1, got {nxyz}")
    overlaps = tuple(int(o) for o in overlaps)
    if halowidths is None:
        halowidths = tuple(max(1, o // 2) for o in overlaps)
    halowidths = tuple(int(h) for h in halowidths)
    periods = (int(periodx), int(periody), int(periodz))
    dims_in = [int(dimx), int(dimy), int(dimz)]
    for d in range(3):
        if nxyz[d] == 1:
            if dims_in[d] > 1 or periods[d]:
                raise ValueError(f"dimension {d} has local size 1: it cannot be split or periodic")
            dims_in[d] = 1
        elif overlaps[d] < 2 * halowidths[d] or halowidths[d] < 1:
            raise ValueError(f"dim {d}: overlap {overlaps[d]} must be >= 2*halowidth {halowidths[d]}")
        elif nxyz[d] < overlaps[d] + halowidths[d]:
            raise ValueError(f"dim {d}: local size {nxyz[d]} < overlap+halowidth")

    thread_local = loopback is not None
    owns_dist = False
    if loopback is not None:
        hub, rank = loopback
        comm_rank, comm_size = rank, hub.size
    else:
        comm_rank, comm_size, _ = C.env_world()
        if comm_size > 1 and init_dist and not torch.distributed.is_initialized():
            C.init_distributed(timeout_s=timeout_s)
            owns_dist = True
        if torch.distributed.is_initialized():
            comm_rank = torch.distributed.get_rank()
            comm_size = torch.distributed.get_world_size()

    # device selection (one GPU per process, node-local rank)
    if loopback is not None:
        local_rank, local_size = comm_rank, comm_size
    else:
        local_rank, local_size = C.node_local_rank(comm_rank, comm_size)
    if device is not None:
        dev = torch.device(device)
        if dev.type == "cuda":
            if dev.index is None:
                dev = torch.device("cuda", local_rank % max(1, C.visible_devices()))
            torch.cuda.set_device(dev)
    elif select_device and torch.cuda.is_available():
        dev = C.select_device(local_rank)
    else:
        dev = torch.device("cpu")

    tname = ("loopback" if loopback is not None
             else _choose_transport(transport, comm_size, dev, local_size))
    if loopback is not None:
        comm: C.Communicator = C.LoopbackComm(hub, comm_rank)
    elif tname == "self":
        comm = C.SelfComm()
    elif tname == "rccl":
        if local_size == comm_size and "NCCL_SOCKET_IFNAME" not in os.environ:
            # single node: RCCL only bootstraps over sockets (data moves over
            # xGMI); pin the bootstrap to loopback so odd container interfaces
            # cannot stall ncclCommInitRank
            os.environ["NCCL_SOCKET_IFNAME"] = "lo"
        try:
            comm = C.RcclComm(dev, timeout_s=timeout_s)
        except RuntimeError as e:
            # RCCL is the perf path: a failed init is fatal unless the caller
            # opted into the host-staged validation transport
            # (RMA_DIAG=rccl_fallback; bench.py never does: a scaling point must
            # not silently run staged)
            if (not diag_flag("rccl_fallback")
                    or os.environ.get("RMA_RCCL_STRICT", "0") == "1"
                    or not torch.distributed.is_initialized()):
                raise
            import warnings

            warnings.warn(f"RCCL communicator init failed ({e}); falling back to the host-staged "
                          "transport (RMA_DIAG=rccl_fallback)", RuntimeWarning, stacklevel=2)
            tname = "staged"
            comm = C.TorchDistComm(staged=True)
    elif tname == "ipc":
        comm = None  # needs the topology's peers: built below
    else:
        comm = C.TorchDistComm(staged=(tname == "staged"))

    dims = tuple(dims_create(comm_size, dims_in))
    topo = CartTopology(comm_size, dims, periods)
    me = comm_rank
    coords = tuple(topo.coords(me))
    neighbors = tuple(tuple(p) for p in topo.neighbors(me))
    if tname == "ipc":
        peers = [p for nb in neighbors for p in nb] + list(topo.diagonals(me))
        comm = C.IpcComm(dev, peers, timeout_s=timeout_s)
    nxyz_g = tuple(geo.n_global(nxyz[d], dims[d], overlaps[d], periods[d]) if nxyz[d] > 1 else 1
                   for d in range(3))

    halo = None
    extra = {}
    if dev.type == "cuda" and tname in ("rccl", "ipc", "self", "loopback"):
        from .._native import native

        if tname == "loopback":
            ncomm = native().LoopbackEndpoint(hub.native_hub(), me)
            extra["endpoint"] = ncomm
            # each logical rank drives its own stream (threads share the default one)
            stream = torch.cuda.Stream(dev)
            extra["stream"] = stream
            torch.cuda.set_stream(stream)
        else:
            ncomm = comm.native if isinstance(comm, (C.RcclComm, C.IpcComm)) else None
        halo = native().HaloExchanger(ncomm, me, [list(p) for p in neighbors])
        if self_via_transport:
            halo.set_self_via_transport(True)
        # diagonal ranks: the executor's exact exchange with x AND y
        # neighbours is then one group (corner blocks to the diagonals)
        halo.set_diagonals(list(topo.diagonals(me)))

    g = GlobalGrid(nxyz=nxyz, nxyz_g=nxyz_g, dims=dims, overlaps=overlaps, halowidths=halowidths,
                   periods=periods, nprocs=comm_size, me=me, coords=coords, neighbors=neighbors,
                   disp=disp, reorder=reorder, comm=comm, device=dev, transport=tname,
                   quiet=quiet, local_rank=local_rank, local_size=local_size, owns_dist=owns_dist,
                   halo=halo, topo=topo, extra=extra)
    _set_grid(g, thread_local)
    if not quiet and me == 0:
        print(g.describe(), flush=True)
    return me, dims, comm_size, coords, comm


def finalize_global_grid(finalize_dist: bool = True) -> None:
    """Release the grid (halo buffers, communicator); IGG ``finalize_global_grid``."""
    g = global_grid()
    try:
        g.comm.finalize()
    finally:
        g.halo = None
        if getattr(_tls, "grid", None) is g:
            _tls.grid = None
        else:
            _set_grid(None, False)
        if g.owns_dist and finalize_dist:
            C.shutdown_distributed()


# ---------------------------------------------------------------------------
# geometry accessors (IGG names)
# ---------------------------------------------------------------------------
def nx_g() -> int:
    return global_grid().nxyz_g[0]


def ny_g() -> int:
    return global_grid().nxyz_g[1]


def nz_g() -> int:
    return global_grid().nxyz_g[2]


def _size_along(A, d: int) -> int:
    if isinstance(A, int):
        return A
    shape = tuple(A.shape)
    return shape[len(shape) - 1 - d] if d < len(shape) else 1


def _coord(ix, d: int, dd: float, A) -> float:
    g = global_grid()
    return geo.coord(ix, dd, g.coords[d], g.nxyz[d], _size_along(A, d), g.overlaps[d],
                     g.nxyz_g[d], g.periods[d])


def x_g(ix, dx: float, A) -> float:
    """Global x of 0-based local index ix of array A (IGG ``x_g(ix+1,dx,A)``)."""
    return _coord(ix, 0, dx, A)


def y_g(iy, dy: float, A) -> float:
    return _coord(iy, 1, dy, A)


def z_g(iz, dz: float, A) -> float:
    return _coord(iz, 2, dz, A)


def me() -> int:
    return global_grid().me


# ---------------------------------------------------------------------------
# collective timers (IGG tic/toc): barrier + wall clock
# ---------------------------------------------------------------------------
def tic() -> None:
    g = global_grid()
    g.comm.barrier()
    g.t0 = time.perf_counter()


def toc() -> float:
    g = global_grid()
    if g.t0 is None:
        raise RuntimeError("toc() without tic()")
    g.comm.barrier()
    return time.perf_counter() - g.t0
