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
