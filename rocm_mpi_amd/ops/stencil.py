"""Tensor-level entry points of the hand-written HIP kernels.

Each op validates shapes, dtype, contiguity and device on the host BEFORE any
launch (a bad shape must never reach a kernel), then dispatches:

* CUDA (ROCm) tensors -> the gfx950 kernels in ``rocm_mpi_amd._C`` on the
  current torch stream; the extension is mandatory (loud failure otherwise);
* CPU tensors -> the bit-identical C++ twins in the same extension, or a pure
  torch formulation when the extension is absent (CPU-only environments).

Reference kernels: K4 fused step ``scripts/diffusion_2D_perf.jl:3-13``; K5
split step ``scripts/diffusion_2D_perf_hide.jl:15-29``; K1-K3
``scripts/diffusion_2D_kp.jl:16-54``; initial condition
``scripts/diffusion_2D_ap.jl:28``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, NamedTuple, Sequence

import torch

from .._native import has_native, native

Rect = tuple  # (x0, x1, y0, y1), half-open, 0-based cell indices

# Kernel ids (StencilTuning.kernel names). The core library (librma_core.so)
# holds what the executor and the ops run by default:
#   one-step:  "march" (0, the fused one-step kernel; "lds", 1, the LDS-tiled
#              baseline, is in the lab library: 3.90 vs 6.20 TB/s, SUMMARY_r1);
#   K-step:    "lds_dpp" (3: canonical, K = 2, 3, 4, 6, 8; LDS 1/Cp ring + DPP),
#              "pipe" (9: the stage-pipelined fast-math kernel, ANY K in 1..24,
#              csrc/kernels/stencil_pipe.h), "pipec" (10: the same pipeline with the
#              canonical arithmetic, bitwise equal to K one-step updates), "piper"
#              (12: "pipe" with the factor rows in registers instead of the LDS
#              ring and an LDS-DMA prefetch, K = 10..24, the executor's fast
#              kernel from K = 14; from K = 10 on tiles of >= 65536 rows).
# LAB_KERNELS live in librma_lab.so (csrc/lab: superseded / experimental kernels kept as
# test oracles and for sweeps), loaded on first use: K-step "march"/"lds"/"dpp" (0/1/2:
# canonical variants of kernel 3), "fast" (4: reassociated, not bitwise), "fast5" (5: the
# 5-point sum with one folded per-cell factor, the GPU oracle of "pipe"), "fast5p2/p4/p8"
# (6/7/8: fixed-K pipelined fast5), "pipeb" (11: pipe with ds_bpermute lane moves), and
# the pipelined kernels' non-default stage splits, two-column blocks and 5 cells per lane,
# "pipe_diag1" (13: a diagnosis, WRONG results: one factor-ring read per stage and row),
# and "piper6" / "piper7" (14 / 15: register factors with the split fast-math form for
# dx != dy, T2 = fma(g, fma(ry, fma(-2,c,U+D), fma(-2,c,L+R)), c); CPU twin: FAST6), and
# "piper_u3" (16: piper with the round-3 unroll by 3, an A/B of the core's unroll by 6),
# "piper_iso" (17: piper for ry == 1 exactly, the y-sum FMA by 1 as an add; bitwise = piper),
# "piper_diag_s0" (18: a diagnosis, WRONG results: stage 0 runs one level fewer),
# "piper_w1" (19: piper at one wave per SIMD, unrolled by 6 also at K = 21..24),
# "piper_mask" (20: piper whose lanes outside a level's valid cone skip it; bitwise = piper)
# and its control "piper_mask_ctl" (21: the same asm arithmetic under the full EXEC),
# "piper_nosb" (22: piper without the sched_barriers inside a level; bitwise = piper),
# "piper_rot" (23: piper with the stage -> wave map rotated by 2 in odd blocks),
# "piper_diag_hb" (24: a diagnosis, WRONG results: the row barrier every other row only),
# "piper_u6s" (25: piper unrolled by 6 also at K = 21..24, spilling),
# "piper_sp" / "piper_sp2" (26 / 27: levels software-pipelined, with / without a
# sched_barrier per level; bitwise = piper), "piper_prio" (28: the rotated stage map
# plus s_setprio for stage-0 waves) and its control "piper_prio_nr" (29: the
# priority without the rotation); bitwise = piper.
FAST5 = ("fast5", "fast5p2", "fast5p4", "fast5p8", "pipe", "pipeb", "piper", "piper_u3",
         "piper_iso", "piper_diag_s0", "piper_w1", "piper_mask", "piper_mask_ctl", "piper_nosb",
         "piper_rot", "piper_diag_hb", "piper_u6s",
         "piper_sp", "piper_sp2", "piper_prio", "piper_prio_nr")
FAST6 = ("piper6", "piper7")
PIPE = ("pipe", "pipec", "pipeb", "piper", "pipe_diag1", "piper6", "piper7", "piper_u3",
        "piper_iso", "piper_diag_s0", "piper_w1", "piper_mask", "piper_mask_ctl", "piper_nosb",
         "piper_rot", "piper_diag_hb", "piper_u6s",
         "piper_sp", "piper_sp2", "piper_prio", "piper_prio_nr")
PIPE_MAX_K = 24
KERNELS = {"march": 0, "lds_dpp": 3, "pipe": 9, "pipec": 10, "piper": 12}
LAB_KERNELS = {"lds": 1, "dpp": 2, "fast": 4, "fast5": 5, "fast5p2": 6, "fast5p4": 7, "fast5p8": 8,
               "pipeb": 11, "pipe_diag1": 13, "piper6": 14, "piper7": 15,
               "piper_u3": 16, "piper_iso": 17, "piper_diag_s0": 18, "piper_w1": 19,
               "piper_mask": 20, "piper_mask_ctl": 21, "piper_nosb": 22, "piper_rot": 23,
               "piper_diag_hb": 24, "piper_u6s": 25, "piper_sp": 26, "piper_sp2": 27,
               "piper_prio": 28, "piper_prio_nr": 29}
KSTEP_CORE = ("lds_dpp", "pipe", "pipec", "piper")


def kernel_id(name: str) -> int:
    """Numeric id of a kernel name (core or lab)."""
    if name in KERNELS:
        return KERNELS[name]
    if name in LAB_KERNELS:
        return LAB_KERNELS[name]
    raise ValueError(f"unknown kernel {name!r}: one of {sorted(KERNELS) + sorted(LAB_KERNELS)}")


def kernel_name(kid: int) -> str:
    """Name of a numeric kernel id (core or lab table). The executor's own
    choices include lab-named ids: its K = 24 kernel is "piper_nosb" (22),
    instantiated in the core as well (csrc/kernels/stencil_pipe_r24.hip)."""
    for table in (KERNELS, LAB_KERNELS):
        for k, v in table.items():
            if v == kid:
                return k
    raise ValueError(f"unknown kernel id {kid}")


def _kstep_needs_lab(K: int, tn: "StencilTuning") -> bool:
    """Does this K-step launch run a librma_lab.so kernel?"""
    if tn.kernel == "piper_nosb" and K == 24 and tn.cols != 2 and not tn.stages:
        return False  # the executor's K = 24 kernel, in the core (stencil_pipe_r24.hip)
    if tn.kernel not in KSTEP_CORE or tn.cols == 2 or (tn.kernel == "pipe" and tn.vec == 5):
        return True
    if tn.kernel in PIPE and tn.stages and has_native():
        return tn.stages != native().pipe_default_stages(K)
    return False


class StencilCoef(NamedTuple):
    """Coefficients of the canonical update (see csrc/include/rma/common.h)."""

    mlam: float  # -lam
    rdx: float  # 1/dx
    rdy: float  # 1/dy
    dt: float

    @classmethod
    def from_physics(cls, lam: float, dx: float, dy: float, dt: float) -> "StencilCoef":
        return cls(-lam, 1.0 / dx, 1.0 / dy, dt)


@dataclass
class StencilTuning:
    """Knobs of the march kernel (defaults = the fastest measured on MI355X,
    profiles/sweep_16k.md): rows per wave-task, rows whose loads are issued
    together, non-temporal bitmask (1: T2 stores, 2: 1/Cp loads), cells per
    lane (2 or 4; the fast5 ``pipe`` kernel also 5 at K = 16..20 when nx % 5 == 0, a
    lab-library experiment, see ``native().pipe_vec``), and the kernel family ("march"
    or the "lds" baseline).
    Bit 2 of the non-temporal mask also streams T loads (implies bits 0-1)."""

    chunk_rows: int = 4
    nontemporal: int = 3
    kernel: str = "march"
    unroll: int = 4
    vec: int = 2
    xcd_remap: int = -1  # -1: chosen by tile width (see csrc/kernels/stencil.hip)
    stages: int = 0  # pipe / pipec: waves per strip (0: native pipe_default_stages)
    cols: int = 0  # pipe: column waves per stage (0: native pipe_default_cols; 2 needs vec=4)


@dataclass
class TileGeometry:
    """Placement of a local tile in the implicit global grid (IGG x_g/y_g)."""

    gx0: int
    gy0: int
    nxg: int
    nyg: int
    dx: float
    dy: float
    xoff: float = 0.0
    yoff: float = 0.0
    periodx: int = 0
    periody: int = 0

    def as_tuple(self):
        return (int(self.gx0), int(self.gy0), int(self.nxg), int(self.nyg), float(self.dx),
                float(self.dy), float(self.xoff), float(self.yoff), int(self.periodx),
                int(self.periody))


def stream_handle(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream if t.is_cuda else 0


def _ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


def check_field(name: str, t: torch.Tensor, shape=None, device=None) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor, got {type(t).__name__}")
    if t.dtype != torch.float64:
        raise TypeError(f"{name} must be float64 (reference fields are Float64), got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")
    if device is not None and t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")


def _use_native_cpu() -> bool:
    return has_native()


def interior_rect(nx: int, ny: int) -> Rect:
    return (1, nx - 1, 1, ny - 1)


def validate_rects(rects: Sequence[Rect], nx: int, ny: int) -> list[Rect]:
    out = []
    if len(rects) > 8:
        raise ValueError("at most 8 rects per launch")
    for r in rects:
        x0, x1, y0, y1 = (int(v) for v in r)
        if x1 <= x0 or y1 <= y0:
            continue
        if x0 < 1 or y0 < 1 or x1 > nx - 1 or y1 > ny - 1:
            raise ValueError(f"rect {r} outside the interior [1,{nx - 1})x[1,{ny - 1})")
        out.append((x0, x1, y0, y1))
    return out


# --------------------------------------------------------------------------
# fused / split stencil
# --------------------------------------------------------------------------
def stencil_torch(T2: torch.Tensor, T: torch.Tensor, iCp: torch.Tensor, c: StencilCoef,
                  rects: Iterable[Rect]) -> None:
    """Pure-torch twin of the fused kernel (same operation order, bitwise)."""
    for x0, x1, y0, y1 in rects:
        cu = T[y0:y1, x0:x1]
        xr = T[y0:y1, x0 + 1:x1 + 1]
        xl = T[y0:y1, x0 - 1:x1 - 1]
        dn = T[y0 + 1:y1 + 1, x0:x1]
        up = T[y0 - 1:y1 - 1, x0:x1]
        qxR = (c.mlam * (xr - cu)) * c.rdx
        qxL = (c.mlam * (cu - xl)) * c.rdx
        qyU = (c.mlam * (dn - cu)) * c.rdy
        qyD = (c.mlam * (cu - up)) * c.rdy
        d = iCp[y0:y1, x0:x1] * ((-(qxR - qxL)) * c.rdx - (qyU - qyD) * c.rdy)
        T2[y0:y1, x0:x1] = cu + c.dt * d


def stencil_step(T2: torch.Tensor, T: torch.Tensor, iCp: torch.Tensor, coef: StencilCoef,
                 rects: Sequence[Rect] | None = None, tuning: StencilTuning | None = None) -> None:
    """T2[r] = T[r] + dt*iCp*(div q)[r] for every rect r (default: the interior)."""
    check_field("T", T)
    ny, nx = T.shape
    check_field("T2", T2, (ny, nx), T.device)
    check_field("iCp", iCp, (ny, nx), T.device)
    if T2.data_ptr() == T.data_ptr():
        raise ValueError("T2 must not alias T (double buffering)")
    rects = validate_rects(rects if rects is not None else [interior_rect(nx, ny)], nx, ny)
    if not rects:
        return
    tn = tuning or StencilTuning()
    if T.is_cuda:
        if tn.kernel != "march":  # the LDS-tiled one-step kernel lives in librma_lab.so
            from .._native import load_lab

            load_lab()
        native().stencil_rects(_ptr(T2), _ptr(T), _ptr(iCp), nx, ny, rects, tuple(coef),
                               tn.chunk_rows, int(tn.nontemporal), kernel_id(tn.kernel),
                               stream_handle(T), True, tn.unroll, tn.vec, tn.xcd_remap)
    elif _use_native_cpu():
        native().stencil_rects(_ptr(T2), _ptr(T), _ptr(iCp), nx, ny, rects, tuple(coef),
                               64, 0, 0, 0, False)
    else:
        stencil_torch(T2, T, iCp, coef, rects)


def stencil2_step(T2: torch.Tensor, T: torch.Tensor, iCp: torch.Tensor, coef: StencilCoef,
                  rects: Sequence[Rect] | None = None, tuning: StencilTuning | None = None) -> None:
    """Two time steps in one pass (temporal blocking, csrc/kernels/stencil_tb.hip):
    T2[r] = f(f(T))[r] for every rect r, where the intermediate step is f(T) on
    the interior and T on the boundary/halo cells. Bitwise equal to two
    ``stencil_step`` calls. Default tuning: 8-row chunks, unroll 2."""
    check_field("T", T)
    ny, nx = T.shape
    check_field("T2", T2, (ny, nx), T.device)
    check_field("iCp", iCp, (ny, nx), T.device)
    if T2.data_ptr() == T.data_ptr():
        raise ValueError("T2 must not alias T (double buffering)")
    rects = validate_rects(rects if rects is not None else [interior_rect(nx, ny)], nx, ny)
    if not rects:
        return
    tn = tuning or StencilTuning(chunk_rows=8, unroll=2)
    if T.is_cuda:
        native().stencil2_rects(_ptr(T2), _ptr(T), _ptr(iCp), nx, ny, rects, tuple(coef),
                                tn.chunk_rows, int(tn.nontemporal), stream_handle(T), True,
                                tn.unroll, tn.xcd_remap)
    elif _use_native_cpu():
        native().stencil2_rects(_ptr(T2), _ptr(T), _ptr(iCp), nx, ny, rects, tuple(coef),
                                8, 0, 0, False)
    else:
        S1 = T.clone()
        stencil_torch(S1, T, iCp, coef, [interior_rect(nx, ny)])
        stencil_torch(T2, S1, iCp, coef, rects)


def stencilk_step(K: int, T2: torch.Tensor, T: torch.Tensor, iCp: torch.Tensor,
                  coef: StencilCoef, rects: Sequence[Rect] | None = None,
                  tuning: StencilTuning | None = None) -> None:
    """K time steps in one pass (csrc/kernels/stencil_kstep.hip, stencil_pipe.h; lab kernels: csrc/lab):
    T2[r] = f^K(T)[r], the intermediate levels being f on the interior and T
    on boundary/halo cells. Kernels: K = 2, 3, 4, 6, 8 for march/lds/dpp/lds_dpp/
    fast/fast5 (12, 16 also fast5 and the fast5p* variants); ANY K in 1..24 for
    pipe (fast5 arithmetic) and pipec (canonical). Canonical kernels are bitwise
    equal to K ``stencil_step`` calls; the fast5 family to the fast5 CPU twin
    (``kernel`` picks the CPU twin's arithmetic too). Default tuning: the native
    executor's (chunk by tile height, LDS 1/Cp ring, DPP)."""
    K = int(K)
    kname = tuning.kernel if tuning is not None else "lds_dpp"
    if kname in PIPE:
        if not 1 <= K <= PIPE_MAX_K:
            raise ValueError(f"K must be in 1..{PIPE_MAX_K} for the pipelined kernels, got {K}")
    elif K not in (2, 3, 4, 6, 8, 12, 16):
        raise ValueError(f"K must be 2, 3, 4, 6, 8, 12 or 16 (any K: kernel 'pipe'/'pipec'), "
                         f"got {K}")
    check_field("T", T)
    if K > 8 and T.is_cuda and kname not in FAST5 + PIPE:
        raise ValueError("12 or 16 steps per pass need a fast5 or pipelined kernel on the GPU")
    ny, nx = T.shape
    check_field("T2", T2, (ny, nx), T.device)
    check_field("iCp", iCp, (ny, nx), T.device)
    if T2.data_ptr() == T.data_ptr():
        raise ValueError("T2 must not alias T (double buffering)")
    rects = validate_rects(rects if rects is not None else [interior_rect(nx, ny)], nx, ny)
    if not rects:
        return
    if tuning is None:  # the executor's measured defaults (default_tune_k)
        ch = native().default_chunk_k(K, ny) if has_native() else 16
        tuning = StencilTuning(chunk_rows=ch, kernel="lds_dpp", xcd_remap=1)
    tn = tuning
    if tn.kernel in FAST5 + FAST6 and not fast5_ok(coef):
        raise ValueError("kernel 'fast5' folds dy^-2/dx^-2 into one factor: needs lam != 0 "
                         f"and finite coefficients, got {tuple(coef)}")
    if T.is_cuda:
        if _kstep_needs_lab(K, tn):
            from .._native import load_lab

            load_lab()
        native().stencilk_rects(K, _ptr(T2), _ptr(T), _ptr(iCp), nx, ny, rects, tuple(coef),
                                tn.chunk_rows, int(tn.nontemporal), stream_handle(T), True,
                                tn.xcd_remap, tn.vec, kernel_id(tn.kernel), int(tn.stages),
                                int(tn.cols))
    elif _use_native_cpu():
        native().stencilk_rects(K, _ptr(T2), _ptr(T), _ptr(iCp), nx, ny, rects, tuple(coef),
                                16, 0, 0, False, -1, 2, kernel_id(tn.kernel), 0)
    elif tn.kernel in FAST5:
        a = T.clone()
        for _ in range(K - 1):
            b = a.clone()
            stencil5_torch(b, a, iCp, coef, [interior_rect(nx, ny)])
            a = b
        stencil5_torch(T2, a, iCp, coef, rects)
    else:
        a = T.clone()
        for _ in range(K - 1):
            b = a.clone()
            stencil_torch(b, a, iCp, coef, [interior_rect(nx, ny)])
            a = b
        stencil_torch(T2, a, iCp, coef, rects)


def fast5_constants(coef: StencilCoef) -> tuple[float, float, float]:
    """(ry, -2(1+ry), dt*lam/dx^2) of the fast5 arithmetic, computed in the
    same order as the kernels (csrc/kernels/stencil_pipe.h)."""
    ax = (-coef.mlam) * coef.rdx * coef.rdx
    ay = (-coef.mlam) * coef.rdy * coef.rdy
    ry = ay / ax
    return ry, -2.0 * (1.0 + ry), coef.dt * ax


def stencil5_torch(T2: torch.Tensor, T: torch.Tensor, iCp: torch.Tensor, c: StencilCoef,
                   rects: Iterable[Rect]) -> None:
    """Torch twin of ONE fast5 step (CPU without the extension). torch has no
    fused multiply-add for float64 tensors: each fma is emulated with
    fma_exact (error-free product and sum, see its caveats)."""
    ry, mkc, gs = fast5_constants(c)
    for x0, x1, y0, y1 in rects:
        cu = T[y0:y1, x0:x1]
        sx = T[y0:y1, x0 + 1:x1 + 1] + T[y0:y1, x0 - 1:x1 - 1]
        sy = T[y0 - 1:y1 - 1, x0:x1] + T[y0 + 1:y1 + 1, x0:x1]
        t = fma_exact(torch.full_like(cu, mkc), cu, sx)
        t = fma_exact(torch.full_like(cu, ry), sy, t)
        g = gs * iCp[y0:y1, x0:x1]
        T2[y0:y1, x0:x1] = fma_exact(g, t, cu)


def _two_prod(a: torch.Tensor, b: torch.Tensor):
    p = a * b
    split = 134217729.0  # 2^27 + 1
    ca, cb = split * a, split * b
    ah = ca - (ca - a)
    al = a - ah
    bh = cb - (cb - b)
    bl = b - bh
    e = ((ah * bh - p) + ah * bl + al * bh) + al * bl
    return p, e


def fma_exact(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor) -> torch.Tensor:
    """Emulated fma(a, b, c) for float64 tensors (the no-extension CPU fallback
    of the fast5 twin only): a*b = p + e exactly (Dekker two_prod) and p + c =
    s + err exactly (two_sum); the result s + (err + e) rounds twice, so it is
    NOT always the correctly rounded fma: it differs when err + e is inexact
    (near-ties after cancellation) and the Veltkamp split overflows for |a| or
    |b| above ~2^996. On the fields the tests use it matches std::fma bitwise
    (tests/test_fast5_cpu.py); the GPU kernels and the native CPU twins use a
    real fma."""
    p, e = _two_prod(a, b)
    s = p + c  # two_sum(p, c)
    bp = s - p
    err = (p - (s - bp)) + (c - bp)
    return s + (err + e)


def fast5_ok(coef: StencilCoef) -> bool:
    """Mirror of rma::fast5_ok: kernel 5 divides by lam/dx^2."""
    import math

    ax = (-coef.mlam) * coef.rdx * coef.rdx
    ay = (-coef.mlam) * coef.rdy * coef.rdy
    return (ax != 0.0 and math.isfinite(ax) and math.isfinite(ay) and math.isfinite(ay / ax)
            and math.isfinite(coef.dt * ax))


def strip_cells(nx: int, vec: int = 2) -> int:
    """x-width of one wave-strip of the march kernel (perf_hide frame rounding)."""
    if has_native():
        return native().stencil_strip_cells(nx, vec)
    if nx % 2:
        return 64
    return 256 if vec == 4 and nx % 4 == 0 else 128


def hide_rects(nx: int, ny: int, bwx: int, bwy: int,
               vec: int = 2) -> tuple[list[Rect], Rect | None]:
    """Frame rects and interior rect of the boundary/interior split.

    The frame holds the send planes (x = 1, nx-2; y = 1, ny-2): width 1 is
    enough. The reference uses b_width=(32,4) (perf_hide.jl:42) because its
    masks run on whole thread blocks; thin x-frames here run in the kernel's
    column mode. Mirrors DiffusionExecutor. ``vec`` is accepted for API
    stability (the split no longer depends on the strip width).
    """
    if bwx < 1 or bwy < 1:
        raise ValueError("b_width must be >= 1 so the send planes are computed first")
    xi0, xi1 = 1 + bwx, nx - 1 - bwx
    yi0, yi1 = 1 + bwy, ny - 1 - bwy
    full = interior_rect(nx, ny)
    if xi0 >= xi1 or yi0 >= yi1:
        return [full], None
    frame = [(1, nx - 1, 1, yi0), (1, nx - 1, yi1, ny - 1), (1, xi0, yi0, yi1),
             (xi1, nx - 1, yi0, yi1)]
    return frame, (xi0, xi1, yi0, yi1)


# --------------------------------------------------------------------------
# kp kernels: QX, QY, D are (ny, nx) buffers indexed like T (csrc/kernels/kp.hip)
# --------------------------------------------------------------------------
def kp_views(QX: torch.Tensor, QY: torch.Tensor, D: torch.Tensor):
    """The reference-shaped arrays qx (ny-2, nx-1), qy (ny-1, nx-2), dTdt
    (ny-2, nx-2) of kp.jl:72-74 as views of the T-indexed buffers."""
    return QX[1:-1, :-1], QY[:-1, 1:-1], D[1:-1, 1:-1]


def _kp_native(t: torch.Tensor) -> bool:
    return t.is_cuda or _use_native_cpu()


def flux(QX, QY, T, mlam: float, rdx: float, rdy: float) -> None:
    check_field("T", T)
    ny, nx = T.shape
    check_field("QX", QX, (ny, nx), T.device)
    check_field("QY", QY, (ny, nx), T.device)
    if _kp_native(T):
        native().flux(_ptr(QX), _ptr(QY), _ptr(T), nx, ny, mlam, rdx, rdy, stream_handle(T),
                      T.is_cuda)
    else:
        QX[1:-1, :-1] = (mlam * (T[1:-1, 1:] - T[1:-1, :-1])) * rdx
        QY[:-1, 1:-1] = (mlam * (T[1:, 1:-1] - T[:-1, 1:-1])) * rdy


def residual(D, QX, QY, iCp, rdx: float, rdy: float) -> None:
    check_field("iCp", iCp)
    ny, nx = iCp.shape
    for name, a in (("D", D), ("QX", QX), ("QY", QY)):
        check_field(name, a, (ny, nx), iCp.device)
    if _kp_native(iCp):
        native().residual(_ptr(D), _ptr(QX), _ptr(QY), _ptr(iCp), nx, ny, rdx, rdy,
                          stream_handle(iCp), iCp.is_cuda)
    else:
        ddx = (QX[1:-1, 1:-1] - QX[1:-1, :-2]) * rdx
        ddy = (QY[1:-1, 1:-1] - QY[:-2, 1:-1]) * rdy
        D[1:-1, 1:-1] = iCp[1:-1, 1:-1] * (-(ddx + ddy))


def update(T, D, dt: float) -> None:
    check_field("T", T)
    ny, nx = T.shape
    check_field("D", D, (ny, nx), T.device)
    if _kp_native(T):
        native().update(_ptr(T), _ptr(D), nx, ny, dt, stream_handle(T), T.is_cuda)
    else:
        T[1:-1, 1:-1] = T[1:-1, 1:-1] + dt * D[1:-1, 1:-1]


# --------------------------------------------------------------------------
# initial conditions
# --------------------------------------------------------------------------
def init_gaussian_(T: torch.Tensor, geom: TileGeometry, lx: float, ly: float) -> torch.Tensor:
    """T = exp(-(x_g+dx/2-lx/2)^2 - (y_g+dy/2-ly/2)^2) evaluated on the device."""
    check_field("T", T)
    ny, nx = T.shape
    if T.is_cuda or _use_native_cpu():
        native().init_gaussian(_ptr(T), nx, ny, geom.as_tuple(), lx, ly, stream_handle(T),
                               T.is_cuda)
    else:
        from ..parallel.geometry import coords_1d

        x = coords_1d(geom.gx0, nx, geom.dx, geom.xoff, geom.nxg, geom.periodx)
        y = coords_1d(geom.gy0, ny, geom.dy, geom.yoff, geom.nyg, geom.periody)
        a = (x + geom.dx / 2) - lx / 2
        b = (y + geom.dy / 2) - ly / 2
        T.copy_(torch.exp(-(a * a)[None, :] - (b * b)[:, None]))
    return T


def init_random_(A: torch.Tensor, geom: TileGeometry, seed: int = 0, lo: float = 0.0,
                 hi: float = 1.0) -> torch.Tensor:
    """Counter-based uniform field keyed by the global cell index."""
    check_field("A", A)
    ny, nx = A.shape
    native().init_random(_ptr(A), nx, ny, geom.as_tuple(), int(seed) & (2**64 - 1), lo, hi,
                         stream_handle(A), A.is_cuda)
    return A


def fill_(A: torch.Tensor, value: float) -> torch.Tensor:
    if A.is_cuda and A.dtype == torch.float64 and A.is_contiguous():
        native().fill(_ptr(A), A.numel(), float(value), stream_handle(A))
    else:
        A.fill_(value)
    return A


# --------------------------------------------------------------------------
# reductions
# --------------------------------------------------------------------------
_RED = {"sum": 0, "max": 1, "min": 2, "maxabs": 3, "nonfinite": 4}
_ws_cache: dict = {}


def reduce(A: torch.Tensor, op: str = "sum") -> torch.Tensor:
    """Device reduction of a float64 field -> 0-d float64 tensor (same device)."""
    if op not in _RED:
        raise ValueError(f"op must be one of {sorted(_RED)}")
    if not (A.dtype == torch.float64 and A.is_contiguous()):
        A = A.contiguous().to(torch.float64)
    if A.is_cuda:
        key = A.device
        ws = _ws_cache.get(key)
        if ws is None:
            ws = torch.empty(native().reduce_workspace_doubles() + 1, dtype=torch.float64,
                             device=A.device)
            _ws_cache[key] = ws
        out = torch.empty((), dtype=torch.float64, device=A.device)
        native().reduce_gpu(_ptr(A), A.numel(), _RED[op], _ptr(out), _ptr(ws), stream_handle(A))
        return out
    if _use_native_cpu():
        return torch.tensor(native().reduce_cpu(_ptr(A), A.numel(), _RED[op]), dtype=torch.float64)
    f = {"sum": torch.sum, "max": torch.max, "min": torch.min,
         "maxabs": lambda a: a.abs().max(), "nonfinite": lambda a: (~torch.isfinite(a)).sum()}[op]
    return f(A).to(torch.float64)


def field_stats(A: torch.Tensor) -> tuple[float, float, float]:
    """(non-finite cell count, min, max of the finite cells) of a float64 field
    in ONE pass (native kernel on the GPU and its CPU twin): the full-field
    check of a timed run. Synchronises the field's stream (returns floats)."""
    if not (A.dtype == torch.float64 and A.is_contiguous()):
        raise TypeError("field_stats expects a contiguous float64 tensor")
    if A.is_cuda:
        key = ("stats", A.device)
        ws = _ws_cache.get(key)
        if ws is None:
            ws = torch.empty(native().field_stats_workspace_doubles(), dtype=torch.float64,
                             device=A.device)
            _ws_cache[key] = ws
        out = torch.empty(3, dtype=torch.float64, device=A.device)
        native().field_stats_gpu(_ptr(A), A.numel(), _ptr(out), _ptr(ws), stream_handle(A))
        bad, lo, hi = out.tolist()
        return bad, lo, hi
    if _use_native_cpu():
        return tuple(native().field_stats_cpu(_ptr(A), A.numel()))
    fin = torch.isfinite(A)
    v = A[fin]
    return (float((~fin).sum()), float(v.min()) if v.numel() else float("inf"),
            float(v.max()) if v.numel() else float("-inf"))

