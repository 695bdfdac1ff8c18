"""NumPy float64 golden model of the reference problem on the GLOBAL grid.

Independent of the package: same physics as scripts/diffusion_2D_ap.jl:11-43
with ImplicitGlobalGrid's global geometry (nx_g = dims*(nx-2)+2, x_g = global
index * dx), using the canonical operation order (multiply by 1/dx and by
1/Cp) so that decomposed runs of the package must match it bitwise.
"""
import numpy as np


def params(nxg, nyg, lx=10.0, ly=10.0, lam=1.0, Cp0=1.0):
    dx, dy = lx / nxg, ly / nyg
    dt = min(dx * dx, dy * dy) * Cp0 / lam / 4.1
    return dx, dy, dt


def initial(nxg, nyg, lx=10.0, ly=10.0):
    dx, dy, _ = params(nxg, nyg, lx, ly)
    x = np.arange(nxg, dtype=np.float64) * dx
    y = np.arange(nyg, dtype=np.float64) * dy
    a = (x + dx / 2) - lx / 2
    b = (y + dy / 2) - ly / 2
    return np.exp(-(a * a)[None, :] - (b * b)[:, None])  # shape (nyg, nxg)


def initial_torch(nxg, nyg, lx=10.0, ly=10.0):
    """initial() with torch's exp: the same doubles up to exp's last-ulp rounding,
    which differs between exp implementations (NumPy's and torch's vector paths
    differ on some CPUs): the oracle for code that evaluates the initial
    condition with torch."""
    import torch

    dx, dy, _ = params(nxg, nyg, lx, ly)
    x = torch.arange(nxg, dtype=torch.float64) * dx
    y = torch.arange(nyg, dtype=torch.float64) * dy
    a = (x + dx / 2) - lx / 2
    b = (y + dy / 2) - ly / 2
    return torch.exp(-(a * a)[None, :] - (b * b)[:, None]).numpy()


def step(T, iCp, mlam, rdx, rdy, dt):
    cu = T[1:-1, 1:-1]
    qxR = (mlam * (T[1:-1, 2:] - cu)) * rdx
    qxL = (mlam * (cu - T[1:-1, :-2])) * rdx
    qyU = (mlam * (T[2:, 1:-1] - cu)) * rdy
    qyD = (mlam * (cu - T[:-2, 1:-1])) * rdy
    out = T.copy()
    out[1:-1, 1:-1] = cu + dt * (iCp[1:-1, 1:-1] * ((-(qxR - qxL)) * rdx - (qyU - qyD) * rdy))
    return out


def run(nxg, nyg, nt, lx=10.0, ly=10.0, lam=1.0, Cp0=1.0, T0=None):
    dx, dy, dt = params(nxg, nyg, lx, ly, lam, Cp0)
    T = initial(nxg, nyg, lx, ly) if T0 is None else np.array(T0, dtype=np.float64)
    iCp = np.full_like(T, 1.0 / Cp0)
    for _ in range(nt):
        T = step(T, iCp, -lam, 1.0 / dx, 1.0 / dy, dt)
    return T


# ---------------------------------------------------------------------------
# fast5 arithmetic (csrc/kernels/stencil_pipe.h, csrc/lab/stencil_kstep_lab.hip kernel 5): the
# 5-point sum with one folded per-cell factor,
#   T2 = fma(g, fma(ry, U+D, fma(-2(1+ry), c, R+L)), c),  g = dt*lam/dx^2 * iCp,
# evaluated with EXACT rational fused multiply-adds (fractions.Fraction; int /
# int true division in CPython is correctly rounded, so float(Fraction) is the
# round-to-nearest-even of the exact value, i.e. what v_fma_f64 / std::fma
# return). Independent of the package: slow, for small grids only.
# ---------------------------------------------------------------------------
def fma(a: float, b: float, c: float) -> float:
    from fractions import Fraction

    return float(Fraction(a) * Fraction(b) + Fraction(c))


def fast5_constants(mlam, rdx, rdy, dt):
    ax = (-mlam) * rdx * rdx
    ay = (-mlam) * rdy * rdy
    ry = ay / ax
    return ry, -2.0 * (1.0 + ry), dt * ax


def step5(T, iCp, mlam, rdx, rdy, dt):
    ry, mkc, gs = fast5_constants(mlam, rdx, rdy, dt)
    ny, nx = T.shape
    out = T.copy()
    for y in range(1, ny - 1):
        for x in range(1, nx - 1):
            c = float(T[y, x])
            sx = float(T[y, x + 1]) + float(T[y, x - 1])
            sy = float(T[y - 1, x]) + float(T[y + 1, x])
            t = fma(mkc, c, sx)
            t = fma(ry, sy, t)
            out[y, x] = fma(gs * float(iCp[y, x]), t, c)
    return out


def run5(T0, iCp, nt, mlam, rdx, rdy, dt):
    T = np.array(T0, dtype=np.float64)
    for _ in range(nt):
        T = step5(T, iCp, mlam, rdx, rdy, dt)
    return T
