"""Headless heatmap output (the reference's Plots/GR ``heatmap`` + ``png``).

Reference: ``gr(); ENV["GKSwstype"]="nul"`` then
``heatmap(transpose(T_v)); png("../output/Temp_<variant>_<nprocs>_<nxg>_<nyg>.png")``
(scripts/diffusion_2D_ap.jl:30,47; kp.jl:96; perf.jl:62; perf_hide.jl:116).
Plots is not available here, so this module writes the PNG itself (zlib +
struct): the field is mapped through the ``inferno`` colour map (Plots'
heatmap default) with y increasing upwards, plus a colour bar strip.
"""
from __future__ import annotations

import os
import struct
import zlib

import numpy as np

# inferno control points (matplotlib/Plots) at t = 0, 0.125, ..., 1
_INFERNO = np.array([
    [0.001462, 0.000466, 0.013866], [0.087411, 0.044556, 0.224813],
    [0.258234, 0.038571, 0.406485], [0.416331, 0.090203, 0.432943],
    [0.578304, 0.148039, 0.404411], [0.735683, 0.215906, 0.330245],
    [0.865006, 0.316822, 0.226055], [0.954506, 0.468744, 0.099874],
    [0.987622, 0.64532, 0.039886], [0.964394, 0.843848, 0.273391],
    [0.988362, 0.998364, 0.644924]])


def colormap(v: np.ndarray) -> np.ndarray:
    """Map values in [0,1] to uint8 RGB via piecewise-linear inferno."""
    v = np.clip(np.nan_to_num(v, nan=0.0), 0.0, 1.0) * (len(_INFERNO) - 1)
    i0 = np.floor(v).astype(np.int64).clip(0, len(_INFERNO) - 2)
    f = (v - i0)[..., None]
    rgb = _INFERNO[i0] * (1 - f) + _INFERNO[i0 + 1] * f
    return (rgb * 255 + 0.5).astype(np.uint8)


def write_png(path: str, rgb: np.ndarray) -> None:
    h, w, _ = rgb.shape
    raw = b"".join(b"\x00" + rgb[r].tobytes() for r in range(h))

    def chunk(tag: bytes, data: bytes) -> bytes:
        return (struct.pack(">I", len(data)) + tag + data
                + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF))

    png = (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
           + chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))
    with open(path, "wb") as f:
        f.write(png)


def heatmap_png(field, path: str, max_pixels: int = 1024, colorbar: bool = True) -> dict:
    """Write ``field`` (2D, rows = y, cols = x) as a heatmap PNG. Large fields
    are subsampled to at most ``max_pixels`` per side. Returns min/max."""
    a = np.asarray(field.cpu().numpy() if hasattr(field, "cpu") else field, dtype=np.float64)
    if a.ndim != 2:
        raise ValueError("heatmap needs a 2D field")
    sy = max(1, -(-a.shape[0] // max_pixels))
    sx = max(1, -(-a.shape[1] // max_pixels))
    a = a[::sy, ::sx]
    lo, hi = float(np.nanmin(a)), float(np.nanmax(a))
    span = hi - lo if hi > lo else 1.0
    img = colormap((a - lo) / span)[::-1]  # y up
    if colorbar:
        h = img.shape[0]
        bar = colormap(np.linspace(1.0, 0.0, h))[:, None, :].repeat(max(4, img.shape[1] // 24), 1)
        gap = np.full((h, 4, 3), 255, np.uint8)
        img = np.concatenate([img, gap, bar], axis=1)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    write_png(path, np.ascontiguousarray(img))
    return {"min": lo, "max": hi, "path": path}


def output_name(variant: str, nprocs: int, nxg: int, nyg: int, outdir: str = "output") -> str:
    return os.path.join(outdir, f"Temp_{variant}_{nprocs}_{nxg}_{nyg}.png")
