#!/usr/bin/env python
"""Time one kernel pass of every depth K (the executor's pass planner input).

For each configuration (kernel family, K, stage split, chunk rows) one pass of
K steps over the interior of an n x n fp64 tile is timed with HIP events in
interleaved rounds (A/B in one process, median reported). The one-step march
kernel is the unit: ``rel`` = pass time / one-step time, the cost the planner
(csrc/runtime/plan.cpp default_pass_costs) minimises. Prints one JSON document.

    python bench/pass_sweep.py                       # 288 GB tile (auto), default set
    python bench/pass_sweep.py --n 16384 --pipe 1-24 --pipec 8,12,16
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def krange(spec: str) -> list[int]:
    out = []
    for part in filter(None, spec.split(",")):
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=0, help="tile edge (0: auto-size to 80%% of HBM)")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--pipe", default="1-24", help="fast5 pipelined kernel depths")
    ap.add_argument("--pipec", default="3-12,16", help="canonical pipelined kernel depths")
    ap.add_argument("--ldsdpp", default="3,4,6,8", help="canonical kernel-3 depths")
    ap.add_argument("--old", default="fast5p4:16,fast5p2:12,fast5:8", help="fixed-K kernels")
    ap.add_argument("--alt", default="12:3,16:8,24:8,8:4,8:1", help="pipe K:stages splits")
    ap.add_argument("--chunk", type=int, default=0, help="rows per task (0: executor default)")
    ap.add_argument("--chunks", default="", help="pipe K:c1/c2/..., extra chunk-row variants")
    ap.add_argument("--chunksc", default="", help="pipec K:c1/c2/..., chunk-row variants")
    ap.add_argument("--pipe2", default="", help="depths of the 2-column-wave pipe kernel")
    ap.add_argument("--chunks2", default="", help="pipe2 K:c1/c2/..., chunk-row variants")
    ap.add_argument("--pipe5", default="", help="depths of the pipe kernel at 5 cells per lane "
                    "(needs n %% 5 == 0)")
    ap.add_argument("--chunks5", default="", help="pipe5 K:c1/c2/..., chunk-row variants")
    ap.add_argument("--kinds", default="", help="other K-step kernels by name, kernel:K[:chunk],"
                    "... (e.g. piper:24,piper:24:4096,pipe_diag1:24; 4 cells per lane)")
    ap.add_argument("--coef-dims", default="1,1",
                    help="coefficients of this process grid at overlap 48 (K = 24): dx = "
                         "10/(dimx(n-48)+48), dy = 10/(dimy(n-48)+48); 1,1 = dx = dy (ry = 1), "
                         "4,2 = the headline 8-GPU grid (ry ~ 0.25), 2,1 the 2-GPU grid")
    ap.add_argument("--coef-alt", default="",
                    help="a second coefficient grid (e.g. 1,1): every kernel is timed at both, "
                         "interleaved in the same rounds (rows tagged with coef_dims)")
    ap.add_argument("--exec", dest="exec_k", default="",
                    help="depths timed with the executor's own fast-math kernel and tuning "
                         "(native fast_kernel_k: ring kernel or piper, chunk rows); rows "
                         "kernel='exec' (the planner's cost table input, scripts/fit_pass_costs.py)")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)

    import torch

    from rocm_mpi_amd import ops
    from rocm_mpi_amd._native import native

    dev = torch.device("cuda", 0)
    n = a.n
    if not n:
        free, _ = torch.cuda.mem_get_info()
        n = int(math.isqrt(int(0.80 * free / 24))) // 256 * 256
    f = dict(dtype=torch.float64, device=dev)
    T = torch.empty((n, n), **f)
    ops.init_random_(T, ops.TileGeometry(0, 0, n, n, 1.0, 1.0), seed=1)
    T2 = torch.empty_like(T)
    T2.copy_(T)
    iCp = torch.empty_like(T)
    ops.fill_(iCp, 1.0)
    def coef_of(spec):
        dxm, dym = (int(v) for v in spec.split(","))
        dx, dy = 10.0 / (dxm * (n - 48) + 48), 10.0 / (dym * (n - 48) + 48)
        return ops.StencilCoef.from_physics(1.0, dx, dy, min(dx, dy) ** 2 / 4.1)

    coefs = {a.coef_dims: coef_of(a.coef_dims)}
    if a.coef_alt:
        coefs[a.coef_alt] = coef_of(a.coef_alt)
    N = native()

    def chunk(K, c=0, kind="pipe"):
        # the executor's rows per task for this kernel and depth
        if c or a.chunk:
            return c or a.chunk
        if kind in ("pipe", "pipe2", "pipeb", "pipe5", "piper", "pipe_diag1", "piper6", "piper7",
                    "piper_u3", "piper_iso", "piper_diag_s0", "piper_w1", "piper_mask",
                    "piper_mask_ctl", "piper_nosb",
                    "piper_rot", "piper_diag_hb", "piper_u6s",
                    "piper_sp", "piper_sp2", "piper_prio", "piper_prio_nr", "piper2",
                    "piper_rot2"):
            return N.pipe_chunk_rows(K, n, False) or N.default_chunk_k(max(K, 3), n)
        if kind == "pipec":
            return N.pipe_chunk_rows(K, n, True) or N.default_chunk_k(max(K, 3), n)
        return N.default_chunk_k(max(K, 3), n)

    cfgs = [("march", 1, 0)]
    cfgs += [("pipe", K, 0) for K in krange(a.pipe)]
    cfgs += [("pipec", K, 0) for K in krange(a.pipec)]
    cfgs += [("lds_dpp", K, 0) for K in krange(a.ldsdpp)]
    cfgs += [("two_step", 2, 0)]
    for item in filter(None, a.old.split(",")):
        k, K = item.split(":")
        cfgs.append((k, int(K), 0))
    for item in filter(None, a.alt.split(",")):
        K, S = item.split(":")
        cfgs.append(("pipe", int(K), int(S)))
    for item in filter(None, a.chunks.split(",")):
        K, cs = item.split(":")
        for c in cs.split("/"):
            cfgs.append(("pipe", int(K), 0, int(c)))
    for item in filter(None, a.chunksc.split(",")):
        K, cs = item.split(":")
        for c in cs.split("/"):
            cfgs.append(("pipec", int(K), 0, int(c)))
    cfgs += [("pipe2", K, 0) for K in krange(a.pipe2)]
    cfgs += [("pipe5", K, 0) for K in krange(a.pipe5)]
    cfgs += [("exec", K, 0) for K in krange(a.exec_k)]
    for item in filter(None, a.kinds.split(",")):
        k, K, *c = item.split(":")  # kernel:K[:chunk_rows]
        cfgs.append((k, int(K), 0, int(c[0])) if c else (k, int(K), 0))
    for item in filter(None, a.chunks5.split(",")):
        K, cs = item.split(":")
        for c in cs.split("/"):
            cfgs.append(("pipe5", int(K), 0, int(c)))
    for item in filter(None, a.chunks2.split(",")):
        K, cs = item.split(":")
        for c in cs.split("/"):
            cfgs.append(("pipe2", int(K), 0, int(c)))

    rect = [ops.interior_rect(n, n)]
    names = {v: k for k, v in {**ops.KERNELS, **ops.LAB_KERNELS}.items()}
    # every configuration at every coefficient grid: (spec, kind, K, S[, chunk])
    cfgs = [(cs,) + c for c in cfgs for cs in coefs]

    def launch(cs, kind, K, S, c=0):
        coef = coefs[cs]
        if kind == "march":
            ops.stencil_step(T2, T, iCp, coef, rect, ops.StencilTuning())
        elif kind == "two_step":
            ops.stencil2_step(T2, T, iCp, coef, rect, ops.StencilTuning(chunk_rows=16, unroll=2))
        elif kind == "exec":
            kid, vec, ch = N.fast_kernel_k(K, n, tuple(coef))
            tn = ops.StencilTuning(chunk_rows=ch, kernel=names[kid], vec=vec, xcd_remap=1)
            ops.stencilk_step(K, T2, T, iCp, coef, rect, tn)
        else:
            vec = 2 if kind in ("lds_dpp", "fast5") else 5 if kind == "pipe5" else 4
            # "<kernel>2": two column waves per stage (pipe2, piper2, piper_rot2)
            cols2 = kind in ("pipe2", "piper2", "piper_rot2")
            kern = "pipe" if kind in ("pipe2", "pipe5") else kind[:-1] if cols2 else kind
            tn = ops.StencilTuning(chunk_rows=chunk(K, c, kind), kernel=kern,
                                   vec=vec, xcd_remap=1, stages=S, cols=2 if cols2 else 0)
            ops.stencilk_step(K, T2, T, iCp, coef, rect, tn)

    times: dict = {c: [] for c in cfgs}
    for c in cfgs:  # warm every kernel once (first launches)
        launch(*c)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in cfgs]
    for r in range(a.rounds):
        for i, c in enumerate(cfgs):
            e0, e1 = ev[i]
            e0.record()
            launch(*c)
            e1.record()
        torch.cuda.synchronize()
        for i, c in enumerate(cfgs):
            times[c].append(ev[i][0].elapsed_time(ev[i][1]))
        print(f"[pass_sweep] round {r + 1}/{a.rounds} done", flush=True)
    base = statistics.median(times[(a.coef_dims, "march", 1, 0)])
    rows = []
    for c in cfgs:
        cs, c = c[0], c[1:]
        kind, K, S = c[:3]
        med = statistics.median(times[(cs,) + c])
        ek = (names[N.fast_kernel_k(K, n, tuple(coefs[cs]))[0]] if kind == "exec" else None)
        rows.append({"coef_dims": cs, "ry": round(ops.fast5_constants(coefs[cs])[0], 6),
                     "kernel": kind, "exec_kernel": ek, "K": K, "stages": S or (native().pipe_default_stages(K)
                                                             if kind in ops.PIPE + ("pipe2", "pipe5")
                                                             else 0),
                     "chunk_rows": (N.fast_kernel_k(K, n, tuple(coefs[cs]))[2] if kind == "exec"
                                    else chunk(K, c[3] if len(c) > 3 else 0, kind)
                                    if kind not in ("march", "two_step") else None),
                     "vec": (N.pipe_vec(K, S, 0, n, 5, True) if kind == "pipe5" else None),
                     "ms_per_pass": round(med, 3), "ms_min": round(min(times[(cs,) + c]), 3),
                     "ms_per_step": round(med / K, 4), "rel": round(med / base, 4),
                     "teff_equiv_GBps": round(K * 24 * n * n / 1e9 / (med / 1e3), 1)})
    doc = {"tile": n, "rounds": a.rounds, "one_step_ms": round(base, 3), "rows": rows,
           "note": "rel = pass time / one-step march kernel time (the planner's cost unit)"}
    s = json.dumps(doc, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
