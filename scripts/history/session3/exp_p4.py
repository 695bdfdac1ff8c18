"""A/B of fast5p4 experiment bits (RMA_EXP_P) at K=16, interleaved in one process.

The RMA_EXP_P hook (stage rotation = 2, stage-0 s_setprio = 4) lived in a scratch
build of csrc/kernels/stencil_tbk.hip only; results in profiles/pmc_fast5_r1.md."""
import os, sys, statistics, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
from rocm_mpi_amd import ops

n = int(os.environ.get("N", "101376")); K = int(os.environ.get("K", "16"))
variants = os.environ.get("VARIANTS", "0,2,4,6").split(",")
kern = os.environ.get("KERN", "fast5p4"); vec = int(os.environ.get("VEC", "4"))
chunk = int(os.environ.get("CHUNK", "1024")); rounds = int(os.environ.get("ROUNDS", "3"))
dev = torch.device("cuda", 0)
T = torch.empty((n, n), dtype=torch.float64, device=dev)
ops.init_random_(T, ops.TileGeometry(0, 0, n, n, 1.0, 1.0), seed=1)
iCp = torch.ones_like(T)
T2 = torch.zeros_like(T)
c = ops.StencilCoef(-1.0, 1.0, 1.0, 0.24) if hasattr(ops, "StencilCoef") else None
tn = ops.StencilTuning(chunk_rows=chunk, xcd_remap=1, kernel=kern, vec=vec)
ev = lambda: torch.cuda.Event(enable_timing=True)
res = {v: [] for v in variants}
ref = None
for r in range(rounds):
    for v in variants:
        if "=" in v:  # NAME=VALUE: an environment switch of a scratch build
            name, val = v.split("=", 1)
            os.environ[name] = val
        else:
            os.environ["RMA_EXP_P"] = v
        ops.stencilk_step(K, T2, T, iCp, c, tuning=tn)
        torch.cuda.synchronize()
        if r == 0:
            s = float(T2[:: n // 97, :: n // 89].sum())
            if ref is None: ref = s
            print(f"variant {v} checksum {s!r} same={s == ref}", flush=True)
        a, b = ev(), ev()
        a.record()
        for _ in range(2):
            ops.stencilk_step(K, T2, T, iCp, c, tuning=tn)
        b.record(); torch.cuda.synchronize()
        res[v].append(a.elapsed_time(b) / 2)
    print("round", r, {v: round(res[v][-1], 3) for v in variants}, flush=True)
out = {v: {"median_ms": statistics.median(x), "best_ms": min(x),
           "teff_TBps": K * 24 * n * n / 1e12 / (statistics.median(x) / 1e3)} for v, x in res.items()}
print(json.dumps({"n": n, "K": K, "kernel": kern, "vec": vec, "chunk": chunk, "results": out}))
