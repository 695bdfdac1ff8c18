"""Hand-written HIP/CDNA4 kernels (gfx950) exposed on torch tensors."""
from .stencil import (KERNELS, Rect, StencilCoef, StencilTuning, TileGeometry, check_field,
                      fill_, flux, hide_rects, kp_views, init_gaussian_, init_random_, interior_rect, reduce,
                      residual, stencil2_step, stencil_step, stencilk_step, stencil_torch, stream_handle, strip_cells, update,
                      validate_rects)
from .halo_ops import copy_plane

__all__ = [
    "KERNELS", "Rect", "StencilCoef", "StencilTuning", "TileGeometry", "check_field", "fill_",
    "flux", "hide_rects", "kp_views", "init_gaussian_", "init_random_", "interior_rect", "reduce", "residual",
    "stencil2_step", "stencil_step", "stencilk_step", "stencil_torch", "stream_handle", "strip_cells", "update", "validate_rects",
    "copy_plane",
]
