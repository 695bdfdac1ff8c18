#!/usr/bin/env python
"""Kernel-level tuning sweep + same-box HBM roofline (one process, interleaved).

Times every stencil variant (march: chunk_rows x unroll x nontemporal; the
LDS-tiled kernel) on an N x N fp64 tile and the streaming probes (copy = 1R1W,
triad = 2R1W, the stencil's byte mix) in interleaved rounds (§5.4 rule 24 of
the CDNA guide: A/B in one process, report median and min). Prints one JSON
document; the bytes model is the reference's T_eff (24 B/cell).

    python bench/stencil_sweep.py --n 16384 --rounds 5 --iters 20
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--chunks", default="4,8,16")
    ap.add_argument("--unrolls", default="4,8")
    ap.add_argument("--vecs", default="2")
    ap.add_argument("--nts", default="1,3")
    ap.add_argument("--xcds", default="0,1")
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--x0", type=int, default=1, help="interior rect offset (perf_hide-like)")
    ap.add_argument("--y0", type=int, default=1)
    ap.add_argument("--no-roof", action="store_true")
    ap.add_argument("--tb-chunks", default="", help="two-step kernel chunk_rows list")
    ap.add_argument("--tb-unrolls", default="2,4")
    ap.add_argument("--tb-xcds", default="0,1")
    ap.add_argument("--no-march", action="store_true")
    ap.add_argument("--tbk", default="", help="K-step kernel: K list, e.g. 2,3,4")
    ap.add_argument("--tbk-chunks", default="16")
    ap.add_argument("--tbk-xcds", default="0")
    ap.add_argument("--tbk-vecs", default="2")
    ap.add_argument("--tbk-kernels", default="march",
                    help="comma list of ops.KERNELS names: march, lds, dpp, lds_dpp, fast, fast5")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)

    import torch

    from rocm_mpi_amd import ops
    from rocm_mpi_amd._native import native

    n = a.n
    dev = torch.device("cuda", 0)
    f = dict(dtype=torch.float64, device=dev)
    T = torch.empty((n, n), **f)
    ops.init_random_(T, ops.TileGeometry(0, 0, n, n, 1.0, 1.0), seed=1)
    T2 = torch.empty_like(T)
    iCp = torch.empty_like(T)
    ops.fill_(iCp, 1.0)
    coef = ops.StencilCoef(-1.0, 1.0, 1.0, 0.2)
    cells = (n - 2) * (n - 2)
    bytes_model = 24.0 * n * n  # T_eff model: local nx*ny incl. halo
    nat = native()
    s = torch.cuda.current_stream().cuda_stream

    variants = {}
    chunks = [int(c) for c in a.chunks.split(",")]
    unrolls = [int(u) for u in a.unrolls.split(",")]
    if a.quick:
        chunks, unrolls = [64], [4]
    vecs = [int(v) for v in a.vecs.split(",")]
    nts = [int(v) for v in a.nts.split(",")]
    if a.quick:
        vecs, nts = [2], [1]
    xcds = [int(v) for v in a.xcds.split(",")]
    rect = [(a.x0, n - 1 - a.x0, a.y0, n - 1 - a.y0)] if (a.x0 > 1 or a.y0 > 1) else None
    for c in chunks:
        for u in unrolls:
            for v in vecs:
                for nt in nts:
                    for x in xcds:
                        tn = ops.StencilTuning(chunk_rows=c, unroll=u, nontemporal=nt, vec=v,
                                               xcd_remap=x)
                        variants[f"march_c{c}_u{u}_v{v}_nt{nt}_x{x}"] = (
                            lambda tn=tn: ops.stencil_step(T2, T, iCp, coef, rect, tuning=tn),
                            bytes_model)
    if a.no_march:
        variants.clear()
    # two steps per call: T_eff-equivalent bytes = 2 x 24 B/cell (the metric's
    # per-step A_eff; the kernel itself moves 24 B/cell per call)
    for c in [int(v) for v in a.tb_chunks.split(",") if v]:
        for u in [int(v) for v in a.tb_unrolls.split(",")]:
            for x in [int(v) for v in a.tb_xcds.split(",")]:
                tn = ops.StencilTuning(chunk_rows=c, unroll=u, nontemporal=3, xcd_remap=x)
                variants[f"tb2_c{c}_u{u}_x{x}"] = (
                    lambda tn=tn: ops.stencil2_step(T2, T, iCp, coef, rect, tuning=tn),
                    2 * bytes_model)
    for K in [int(v) for v in a.tbk.split(",") if v]:
        for c in [int(v) for v in a.tbk_chunks.split(",")]:
            for x, vv, kk in [(int(x), int(vv), kk) for x in a.tbk_xcds.split(",")
                              for vv in a.tbk_vecs.split(",") for kk in a.tbk_kernels.split(",")]:
                tn = ops.StencilTuning(chunk_rows=c, nontemporal=3, xcd_remap=x, vec=vv,
                                       kernel=kk)
                variants[f"tbk{K}_c{c}_x{x}_v{vv}_{kk}"] = (
                    lambda K=K, tn=tn: ops.stencilk_step(K, T2, T, iCp, coef, rect, tuning=tn),
                    K * bytes_model)
    variants["lds"] = (lambda: ops.stencil_step(T2, T, iCp, coef,
                                                tuning=ops.StencilTuning(kernel="lds")),
                       bytes_model)
    nn = n * n
    for nt in ((0, 1) if not a.no_roof else ()):
        for blocks in (0, 4096, 16384):
            variants[f"roof_copy_nt{nt}_b{blocks}"] = (
                lambda nt=nt, b=blocks: nat.stream_copy(T2.data_ptr(), T.data_ptr(), nn, s, nt, b),
                16.0 * nn)
            variants[f"roof_triad_nt{nt}_b{blocks}"] = (
                lambda nt=nt, b=blocks: nat.stream_triad(T2.data_ptr(), T.data_ptr(),
                                                         iCp.data_ptr(), 0.5, nn, s, nt, b),
                24.0 * nn)
    times = {k: [] for k in variants}
    for fn, _ in variants.values():  # warm
        fn()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for k, (fn, _) in variants.items():
            ev0.record()
            for _ in range(a.iters):
                fn()
            ev1.record()
            ev1.synchronize()
            times[k].append(ev0.elapsed_time(ev1) / a.iters / 1e3)
    res = {}
    for k, (fn, b) in variants.items():
        med = statistics.median(times[k])
        res[k] = {"median_ms": med * 1e3, "min_ms": min(times[k]) * 1e3,
                  "GBps_median": b / med / 1e9, "GBps_best": b / min(times[k]) / 1e9}
    def best_of(prefix):
        return max((k for k in res if k.startswith(prefix)), key=lambda k: res[k]["GBps_median"])

    best = (best_of("march") if any(k.startswith("march") for k in res)
            else best_of("tb2") if any(k.startswith("tb2") for k in res) else None)
    doc = {"n": n, "cells": cells, "rounds": a.rounds, "iters": a.iters, "results": res,
           "best_march": best, "best_march_GBps": res[best]["GBps_median"] if best else None,
           "device": torch.cuda.get_device_name(0)}
    for K in [int(v) for v in a.tbk.split(",") if v]:
        bk = best_of(f"tbk{K}_")
        doc.update({f"best_tbk{K}": bk, f"best_tbk{K}_GBps_equiv": res[bk]["GBps_median"]})
    if any(k.startswith("tb2") for k in res):
        tb = best_of("tb2")
        doc.update({"best_tb2": tb, "best_tb2_GBps_equiv": res[tb]["GBps_median"]})
    if not a.no_roof:
        tri, cop = best_of("roof_triad"), best_of("roof_copy")
        doc.update({"best_triad": tri, "triad_GBps": res[tri]["GBps_median"],
                    "best_copy": cop, "copy_GBps": res[cop]["GBps_median"],
                    "best_vs_triad": (res[best]["GBps_median"] / res[tri]["GBps_median"]
                                      if best else None)})
    txt = json.dumps(doc, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt)


if __name__ == "__main__":
    main()
