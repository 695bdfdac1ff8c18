"""A/B of the block -> task order of the pipelined passes at the 288 GB tile:
xcd_remap=1 (each XCD a contiguous 1/8 of the tasks) vs 0 (dispatch order)."""
import json
import math
import statistics
import sys

import torch

sys.path.insert(0, ".")
from rocm_mpi_amd import ops  # noqa: E402
from rocm_mpi_amd._native import native  # noqa: E402

free, _ = torch.cuda.mem_get_info()
n = int(math.isqrt(int(0.80 * free / 24))) // 256 * 256
T = torch.empty((n, n), dtype=torch.float64, device="cuda")
ops.init_random_(T, ops.TileGeometry(0, 0, n, n, 1.0, 1.0), seed=1)
T2 = T.clone()
iCp = torch.empty_like(T)
ops.fill_(iCp, 1.0)
dx = 10.0 / n
coef = ops.StencilCoef.from_physics(1.0, dx, dx, dx * dx / 4.1)
rect = [ops.interior_rect(n, n)]
res = {}
for K in (20, 24):
    ch = native().fast_kernel_k(K, n, tuple(coef))[2]
    for remap in (1, 0, 1, 0):
        tn = ops.StencilTuning(chunk_rows=ch, kernel="pipe", vec=4, xcd_remap=remap)
        ops.stencilk_step(K, T2, T, iCp, coef, rect, tn)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.stencilk_step(K, T2, T, iCp, coef, rect, tn)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        res.setdefault(f"K{K}_remap{remap}", []).append(round(statistics.median(ts), 3))
print(json.dumps({"tile": n, "ms_per_pass": res}))
