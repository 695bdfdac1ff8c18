#!/usr/bin/env python
"""Fixed workload for rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE per kernel).

Runs the march stencil, the LDS stencil, the kp kernels and the copy/triad
roofline probes a few times each on an N x N fp64 tile (far beyond the 256 MiB
Infinity Cache), so per-dispatch HBM bytes can be compared with the T_eff
model (24 B/cell). See scripts/profile.sh.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rocm_mpi_amd import ops  # noqa: E402
from rocm_mpi_amd._native import native  # noqa: E402

n = int(os.environ.get("RMA_PROBE_N", "16384"))
reps = int(os.environ.get("RMA_PROBE_REPS", "3"))
f = dict(dtype=torch.float64, device="cuda")
T = torch.empty((n, n), **f)
ops.init_random_(T, ops.TileGeometry(0, 0, n, n, 1.0, 1.0), seed=1)
T2 = torch.empty_like(T)
iCp = torch.empty_like(T)
ops.fill_(iCp, 1.0)
c = ops.StencilCoef(-1.0, 1.0, 1.0, 0.2)
s = torch.cuda.current_stream().cuda_stream
nat = native()
which = os.environ.get("RMA_PROBE_SET", "all")
if which == "fast":  # fast-math K-step kernels at the executor's tuning (bench default)
    K = int(os.environ.get("RMA_PROBE_K", "8"))
    ch = nat.default_chunk_k(K, n)
    for kern in os.environ.get("RMA_PROBE_KERNELS", "fast,fast5").split(","):
        vec = 4 if kern in ("fast5p2", "fast5p4", "fast5p8") else 2
        for _ in range(reps):
            ops.stencilk_step(K, T2, T, iCp, c, tuning=ops.StencilTuning(chunk_rows=ch, xcd_remap=1,
                                                                        kernel=kern, vec=vec))
    torch.cuda.synchronize()
    print(f"probe done n={n} reps={reps} set={which} K={K} chunk={ch}")
    sys.exit(0)
if which == "piper":  # the executor's register-factor kernel alone (scheduler A/B counters)
    K = int(os.environ.get("RMA_PROBE_K", "20"))
    ch = nat.pipe_chunk_rows(K, n, False) or nat.default_chunk_k(K, n)
    rect = [ops.interior_rect(n, n)]
    for _ in range(reps):
        ops.stencilk_step(K, T2, T, iCp, c, rect,
                          ops.StencilTuning(chunk_rows=ch, xcd_remap=1, kernel="piper", vec=4))
    torch.cuda.synchronize()
    print(f"probe done n={n} reps={reps} set={which} K={K} chunk={ch}")
    sys.exit(0)
if which == "cols":  # piper with 1 vs 2 column waves per stage
    from rocm_mpi_amd._native import load_lab

    load_lab()
    K = int(os.environ.get("RMA_PROBE_K", "20"))
    ch = nat.pipe_chunk_rows(K, n, False) or nat.default_chunk_k(K, n)
    rect = [ops.interior_rect(n, n)]
    for kern, cols in (("piper", 1), ("piper", 2), ("piper_rot", 2)):
        for _ in range(reps):
            ops.stencilk_step(K, T2, T, iCp, c, rect,
                              ops.StencilTuning(chunk_rows=ch, xcd_remap=1, kernel=kern, vec=4,
                                                cols=cols))
    torch.cuda.synchronize()
    print(f"probe done n={n} reps={reps} set={which} K={K} chunk={ch}")
    sys.exit(0)
if which in ("all", "tbk"):  # multi-step kernels (temporal blocking)
    for K, ch in ((2, 16), (3, 128), (4, 128), (6, 128), (8, 128)):
        for _ in range(reps):
            ops.stencilk_step(K, T2, T, iCp, c, tuning=ops.StencilTuning(chunk_rows=ch,
                                                                        xcd_remap=1))
    for _ in range(reps):
        ops.stencil2_step(T2, T, iCp, c)
    if which == "tbk":
        for _ in range(reps):
            ops.stencil_step(T2, T, iCp, c)
        torch.cuda.synchronize()
        print(f"probe done n={n} reps={reps} set={which}")
        sys.exit(0)
for _ in range(reps):
    ops.stencil_step(T2, T, iCp, c)
for _ in range(reps):
    ops.stencil_step(T2, T, iCp, c, tuning=ops.StencilTuning(kernel="lds"))
for _ in range(reps):
    nat.stream_copy(T2.data_ptr(), T.data_ptr(), n * n, s, 1)
for _ in range(reps):
    nat.stream_triad(T2.data_ptr(), T.data_ptr(), iCp.data_ptr(), 0.5, n * n, s, 1)
torch.cuda.synchronize()
print(f"probe done n={n} reps={reps}")
