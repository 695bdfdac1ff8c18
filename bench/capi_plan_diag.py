"""Diagnosis: C ABI executor, periodic single rank, eager runs split into
different run() calls (different pass decompositions) vs one-step runs."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from test_capi_gpu import ck, coef4, grid, lib  # noqa: E402

L = lib()
s = torch.cuda.current_stream().cuda_stream


def run(nx, ny, K, mode, fast, seq, periods, halo_first):
    g = grid(L, nx, ny, K, periods=periods)
    T = torch.rand(ny, nx, dtype=torch.float64, generator=torch.Generator().manual_seed(3)).cuda()
    if halo_first:
        ck(L, L.rma_update_halo(g, 1, (ctypes.c_void_p * 1)(T.data_ptr()),
                                (ctypes.c_int64 * 3)(nx, ny, 1), (ctypes.c_int * 1)(8),
                                ctypes.c_void_p(s)))
    T2 = T.clone()
    iCp = torch.ones_like(T)
    ex = ctypes.c_void_p()
    ck(L, L.rma_executor_create_g(g, mode, ctypes.c_void_p(T.data_ptr()),
                                  ctypes.c_void_p(T2.data_ptr()), ctypes.c_void_p(iCp.data_ptr()),
                                  ctypes.c_int64(nx), ctypes.c_int64(ny), coef4(L, g, nx, ny),
                                  ctypes.c_int64(1), ctypes.c_int64(1), K, fast, 0, None,
                                  None, None, ctypes.byref(ex)))
    for n in seq:
        ck(L, L.rma_executor_run(ex, ctypes.c_int64(n), ctypes.c_void_p(s)))
    par = L.rma_executor_parity(ex)
    torch.cuda.synchronize()
    out = (T2 if par else T).cpu().numpy()
    ck(L, L.rma_executor_destroy(ex))
    ck(L, L.rma_finalize_global_grid(g))
    return out


for nx, ny in [(514, 300)]:
    for periods in [(1, 1, 0), (0, 0, 0), (1, 0, 0), (0, 1, 0)]:
        for mode in (0, 1):
          for hf in (False, True):
            for fast in (0, 1):
                K = 8
                ref = run(nx, ny, K, mode, fast, [1] * 16, periods, hf)
                for seq in ([16], [8, 8], [7, 7, 2], [6, 6, 4], [5, 5, 6], [4] * 4, [2] * 8,
                            [3, 3, 3, 3, 4], [8, 4, 4]):
                    o = run(nx, ny, K, mode, fast, seq, periods, hf)
                    d = np.abs(o - ref)
                    w = np.argwhere(d > 0)
                    print(periods, "halo_first", hf, "mode", mode, "fast", fast, seq, "maxdiff", float(d.max()),
                          "ndiff", len(w),
                          "rows", (int(w[:, 0].min()), int(w[:, 0].max())) if len(w) else None,
                          "cols", (int(w[:, 1].min()), int(w[:, 1].max())) if len(w) else None,
                          flush=True)
