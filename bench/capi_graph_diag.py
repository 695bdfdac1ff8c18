"""Diagnosis: C ABI executor, periodic single rank, graph replay vs eager."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import golden  # noqa: E402
from test_capi_gpu import ck, coef4, grid, lib  # noqa: E402

L = lib()
nx, ny = 514, 300
s = torch.cuda.current_stream().cuda_stream


def run(K, nt, graph_steps, init):
    g = grid(L, nx, ny, K, periods=(1, 1, 0))
    if init == "gauss":
        T = torch.from_numpy(golden.initial(nx, ny)).cuda()
    else:
        T = torch.rand(ny, nx, dtype=torch.float64, generator=torch.Generator().manual_seed(3)).cuda()
    T2 = T.clone()
    iCp = torch.ones_like(T)
    ex = ctypes.c_void_p()
    ck(L, L.rma_executor_create_g(g, 1, ctypes.c_void_p(T.data_ptr()),
                                  ctypes.c_void_p(T2.data_ptr()), ctypes.c_void_p(iCp.data_ptr()),
                                  ctypes.c_int64(nx), ctypes.c_int64(ny), coef4(L, g, nx, ny),
                                  ctypes.c_int64(1), ctypes.c_int64(1), K, 0, graph_steps, None,
                                  None, None, ctypes.byref(ex)))
    ck(L, L.rma_executor_run(ex, ctypes.c_int64(nt), ctypes.c_void_p(s)))
    par = L.rma_executor_parity(ex)
    torch.cuda.synchronize()
    out = (T2 if par else T).cpu().numpy()
    ck(L, L.rma_executor_destroy(ex))
    ck(L, L.rma_finalize_global_grid(g))
    return out, par


for K, nt, gs in [(8, 43, 10), (8, 40, 10), (8, 10, 10), (8, 20, 10), (4, 43, 10), (6, 43, 10),
                  (2, 43, 10), (8, 43, 8)]:
    for init in ("gauss", "rand"):
        a, pa = run(K, nt, 0, init)
        b, pb = run(K, nt, gs, init)
        d = np.abs(a - b)
        where = np.argwhere(d > 0)
        print(K, nt, gs, init, "parity", pa, pb, "maxdiff", float(d.max()), "ndiff", len(where),
              "rows", (where[:, 0].min(), where[:, 0].max()) if len(where) else None,
              "cols", (where[:, 1].min(), where[:, 1].max()) if len(where) else None, flush=True)
