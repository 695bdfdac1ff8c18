"""Hand-written HIP/CDNA4 kernels (gfx950) exposed on torch tensors."""
from .stencil import (FAST5, KERNELS, KSTEP_CORE, LAB_KERNELS, PIPE, PIPE_MAX_K, Rect, StencilCoef, StencilTuning,
                      TileGeometry, check_field, fast5_constants, fast5_ok, field_stats, fill_, flux,
                      fma_exact, hide_rects, init_gaussian_, init_random_, interior_rect,
                      kernel_id, kernel_name, kp_views, reduce, residual, stencil2_step, stencil5_torch, stencil_step,
                      stencil_torch, stencilk_step, stream_handle, strip_cells, update,
                      validate_rects)
from .halo_ops import copy_plane, copy_planes

__all__ = [
    "FAST5", "KERNELS", "KSTEP_CORE", "LAB_KERNELS", "PIPE", "PIPE_MAX_K", "Rect", "StencilCoef", "StencilTuning",
    "TileGeometry", "check_field", "fast5_constants", "fast5_ok", "field_stats", "fill_", "flux", "fma_exact",
    "hide_rects", "init_gaussian_", "init_random_", "interior_rect", "kernel_id", "kernel_name", "kp_views", "reduce",
    "residual", "stencil2_step", "stencil5_torch", "stencil_step", "stencil_torch",
    "stencilk_step", "stream_handle", "strip_cells", "update", "validate_rects", "copy_plane", "copy_planes",
]
