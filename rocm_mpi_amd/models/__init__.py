"""Model family: the 2D diffusion variants of the reference (ap, kp, perf, perf_hide)."""
from .diffusion import VARIANTS, Diffusion2D, DiffusionConfig

__all__ = ["VARIANTS", "Diffusion2D", "DiffusionConfig"]
