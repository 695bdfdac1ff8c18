"""Halo pack/unpack primitive (K7/K8 of SURVEY.md §2.3) on torch tensors.

``copy_plane(dst, src)`` copies one (possibly strided) plane view into another
with the native ``copy2d`` kernel: both views must be 2-D with a unit-stride
inner dimension (the shapes the halo engine produces: an x-plane of a
row-major field is a column, i.e. rows of length hw at stride nx).
``copy_planes([(dst, src), ...])`` runs up to ``copy2d_batch_max()`` such
copies of one dtype in ONE launch (the halo engine batches all packs of a
dimension, then all its unpacks, the same way).
"""
from __future__ import annotations

import torch

from .._native import native
from .stencil import stream_handle


def _check(dst: torch.Tensor, src: torch.Tensor) -> None:
    if dst.shape != src.shape or dst.dim() != 2:
        raise ValueError("copy_plane needs two 2-D views of equal shape")
    if dst.dtype != src.dtype or dst.device != src.device:
        raise ValueError("dtype/device mismatch")
    if dst.stride(1) != 1 or src.stride(1) != 1:
        raise ValueError("inner dimension must be unit-stride")


def copy_planes(pairs) -> None:
    """Batched ``copy_plane``: every (dst, src) pair in one kernel launch."""
    pairs = list(pairs)
    if not pairs:
        return
    d0 = pairs[0][0]
    if len(pairs) > native().copy2d_batch_max():
        raise ValueError(f"at most {native().copy2d_batch_max()} copies per batch")
    descs = []
    for dst, src in pairs:
        _check(dst, src)
        if dst.dtype != d0.dtype or dst.device != d0.device:
            raise ValueError("one dtype and device per batch")
        descs.append((dst.data_ptr(), dst.stride(0), src.data_ptr(), src.stride(0), dst.shape[0],
                      dst.shape[1]))
    native().copy2d_batch(descs, d0.element_size(), stream_handle(d0), d0.is_cuda)


def copy_plane(dst: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    _check(dst, src)
    es = dst.element_size()
    native().copy2d(dst.data_ptr(), dst.stride(0), src.data_ptr(), src.stride(0), dst.shape[0],
                    dst.shape[1], es, stream_handle(dst), dst.is_cuda)
    return dst
