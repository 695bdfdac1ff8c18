"""``update_halo_`` and ``gather_`` (ImplicitGlobalGrid update_halo! / gather!).

``update_halo_(*arrays)`` — reference call sites ``diffusion_2D_ap.jl:42``,
``diffusion_2D_kp.jl:91``, ``diffusion_2D_perf.jl:51``; semantics SURVEY.md
C18. GPU fields on the ``rccl``/``self`` transports go through the native
:class:`HaloExchanger` (pack kernels + one RCCL group per dimension on the
current stream, zero-copy for contiguous planes, no host synchronisation).
Every other case (CPU tensors, host-staged, loopback) runs the same plane
algebra in Python over the communicator's tagged P2P groups.

``gather_(A, A_global, root)`` — reference call sites ``ap.jl:46``,
``kp.jl:95``, ``perf.jl:61``; every rank's block lands in ``A_global`` at its
Cartesian coordinates (no overlap removal: callers strip the halo first, as
the reference does with ``T_nh .= Array(T[2:end-1,2:end-1])``).
"""
from __future__ import annotations

import os

import torch

from ..config import diag_flag
from . import comm as C
from .implicit_grid import GlobalGrid, global_grid


def _sizes(A: torch.Tensor) -> tuple[int, int, int]:
    s = tuple(A.shape)
    if not 1 <= len(s) <= 3:
        raise ValueError(f"halo fields must be 1-, 2- or 3-D, got shape {s}")
    r = s[::-1] + (1,) * (3 - len(s))
    return r[0], r[1], r[2]


def field_overlaps(g: GlobalGrid, A: torch.Tensor) -> tuple[int, int, int]:
    """Overlap of array A per dim: ol + (size(A) - n) (staggered arrays)."""
    sz = _sizes(A)
    out = []
    for d in range(3):
        if sz[d] == 1:
            out.append(g.overlaps[d])
            continue
        diff = sz[d] - g.nxyz[d]
        if abs(diff) > 1 and g.dims[d] > 1:
            raise ValueError(f"array size {sz[d]} along dim {d} is incompatible with the local "
                             f"grid size {g.nxyz[d]} (staggering of at most +-1 supported)")
        out.append(g.overlaps[d] + diff)
    return tuple(out)


def has_halo(g: GlobalGrid, A: torch.Tensor, d: int) -> bool:
    """True when A exchanges planes along d (IGG skips dims where the array's
    overlap cannot hold two halo planes, e.g. size n-1 with overlap 2)."""
    n = _sizes(A)[d]
    ol = field_overlaps(g, A)[d]
    hw = g.halowidths[d]
    return n > 1 and ol >= 2 * hw and n >= ol + hw


def _check_has_some_halo(g: GlobalGrid, arrays) -> None:
    for i, A in enumerate(arrays):
        if not any(has_halo(g, A, d) for d in range(3)):
            raise ValueError(f"field {i} (shape {tuple(A.shape)}) has no halo in any dimension")


def _active_dims(g: GlobalGrid) -> list[int]:
    return [d for d in range(3) if g.neighbors[d][0] >= 0 or g.neighbors[d][1] >= 0]


def update_halo_(*arrays: torch.Tensor, dims=(0, 1, 2)) -> None:
    """Update the halo of every array (in place), dimension by dimension."""
    if not arrays:
        return
    g = global_grid()
    dev = arrays[0].device
    for A in arrays:
        if A.device != dev:
            raise ValueError("all arrays of one update_halo_ call must be on one device")
        if not A.is_contiguous():
            raise ValueError("halo fields must be contiguous")
    mask = 0
    for d in dims:
        mask |= 1 << d
    _check_has_some_halo(g, arrays)
    if dev.type == "cuda" and g.halo is not None:
        fields = []
        for A in arrays:
            sz = _sizes(A)
            ol = field_overlaps(g, A)
            fields.append((A.data_ptr(), list(sz), A.element_size(), list(ol),
                           list(g.halowidths)))
        stream = torch.cuda.current_stream(dev).cuda_stream
        # x AND y neighbours, 2D fields: one group with the corner blocks sent to
        # the diagonal ranks (bitwise the same halos as the per-dimension groups;
        # csrc/runtime/halo_plan.cpp plan_exchange_merged, RMA_DIAG no_halo_merged: off)
        nb = g.neighbors
        if (mask & 3) == 3 and all(f[1][2] == 1 for f in fields) and g.halo.has_diagonals \
                and max(nb[0]) >= 0 and max(nb[1]) >= 0 \
                and not diag_flag("no_halo_merged"):
            g.halo.exchange_merged(fields, stream)
        else:
            g.halo.exchange(fields, stream, mask)
        return
    _update_halo_python(g, arrays, mask)


update_halo = update_halo_


def _plane(A: torch.Tensor, d: int, start: int, width: int) -> torch.Tensor:
    return A.narrow(A.dim() - 1 - d, start, width)


def _update_halo_python(g: GlobalGrid, arrays, mask: int) -> None:
    for d in _active_dims(g):
        if not (mask >> d & 1):
            continue
        hw = g.halowidths[d]
        sends, recvs, unpack = [], [], []
        for i, A in enumerate(arrays):
            if not has_halo(g, A, d):
                continue
            n = _sizes(A)[d]
            ol = field_overlaps(g, A)[d]
            send_p = [_plane(A, d, ol - hw, hw), _plane(A, d, n - ol, hw)]
            recv_p = [_plane(A, d, 0, hw), _plane(A, d, n - hw, hw)]
            s_ops, r_ops = [None, None], [None, None]
            for s in (0, 1):
                p = g.neighbors[d][s]
                if p < 0:
                    continue
                if p == g.me:
                    recv_p[s].copy_(send_p[1 - s])
                    continue
                buf = torch.empty(recv_p[s].shape, dtype=A.dtype, device=A.device)
                s_ops[s] = C.P2P("send", send_p[s].contiguous(), p, tag=2 * i + s)
                r_ops[s] = C.P2P("recv", buf, p, tag=2 * i + (1 - s))
                unpack.append((recv_p[s], buf))
            # order matters for order-matched transports (RCCL): sends lo,hi; recvs hi,lo
            sends += [o for o in s_ops if o is not None]
            recvs += [o for o in r_ops[::-1] if o is not None]
        if sends or recvs:
            g.comm.exchange(sends + recvs)
            for dst, buf in unpack:
                dst.copy_(buf)


def gather_(A: torch.Tensor, A_global: torch.Tensor | None = None, root: int = 0):
    """Gather every rank's ``A`` into ``A_global`` on ``root`` (returned there;
    None elsewhere). ``A_global`` defaults to a new CPU tensor of shape
    ``dims .* size(A)``."""
    g = global_grid()
    sz = _sizes(A)
    shape_g = tuple(g.dims[d] * sz[d] for d in range(3))
    parts = g.comm.gather(A.contiguous(), root)
    if g.me != root:
        return None
    nd = A.dim()
    want = shape_g[:nd][::-1]
    if A_global is None:
        A_global = torch.empty(want, dtype=A.dtype)
    if tuple(A_global.shape) != want:
        raise ValueError(f"A_global has shape {tuple(A_global.shape)}, expected {want}")
    for r, part in enumerate(parts):
        c = g.topo.coords(r)
        idx = []
        for d in reversed(range(nd)):
            idx.append(slice(c[d] * sz[d], (c[d] + 1) * sz[d]))
        A_global[tuple(idx)] = part.to(A_global.device)
    return A_global


gather = gather_
