#!/usr/bin/env python
"""Pass time, package power and SCLK of K-step kernel configurations.

The deep passes are fp64-VALU- and power-bound (profiles/pmc_pipe_r2.md): this
probe runs each configuration back to back for a few seconds on the 288 GB
tile while a thread samples ``rocm-smi --showpower --showclocks`` once per
second, and reports the median pass time with the median power and clock of
the samples taken inside that window. Prints one JSON document.

    python bench/power_probe.py --configs pipe:16,pipe:20,pipe:24,pipeb:20 --seconds 6
    python bench/power_probe.py --configs pipe:24:iso,pipe:24:aniso,pipe:24:pow2

A third field picks the coefficients: iso (dx = dy = 10/n: ry = (dx/dy)^2 = 1, the
default), aniso (dx = 10/(n - 48), dy = 10/n: a single x-periodic rank's ry), pow2
(dx = 10/(2n) = dy/2 exactly: ry = 0.25, a power of two) -- the pass energy at the
power cap depends on the constant multipliers (profiles/SUMMARY_r3.md section 1).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import re
import statistics
import subprocess
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def smi_sample() -> dict:
    try:
        out = subprocess.run(["rocm-smi", "--showpower", "--showclocks"], capture_output=True,
                             text=True, timeout=10).stdout
    except Exception as e:  # noqa: BLE001
        return {"error": str(e)}
    d = {}
    m = re.search(r"Power \(W\):\s*([0-9.]+)", out)
    if m:
        d["power_W"] = float(m.group(1))
    m = re.search(r"sclk clock level:\s*\S+:\s*\(([0-9]+)Mhz\)", out, re.I)
    if m:
        d["sclk_MHz"] = float(m.group(1))
    return d


def smi_power_cap() -> float | None:
    """The board's power cap (rocm-smi --showmaxpower), recorded next to the readings."""
    try:
        out = subprocess.run(["rocm-smi", "--showmaxpower"], capture_output=True, text=True,
                             timeout=10).stdout
    except Exception:  # noqa: BLE001
        return None
    m = re.search(r"Max Graphics Package Power \(W\):\s*([0-9.]+)", out)
    return float(m.group(1)) if m else None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--configs", default="march:1,pipe:16,pipe:20,pipe:24,pipeb:16,pipeb:20")
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)

    import torch

    from rocm_mpi_amd import ops
    from rocm_mpi_amd._native import native

    n = a.n
    if not n:
        free, _ = torch.cuda.mem_get_info()
        n = int(math.isqrt(int(0.80 * free / 24))) // 256 * 256
    f = dict(dtype=torch.float64, device="cuda")
    T = torch.empty((n, n), **f)
    ops.init_random_(T, ops.TileGeometry(0, 0, n, n, 1.0, 1.0), seed=1)
    T2 = T.clone()
    iCp = torch.empty_like(T)
    ops.fill_(iCp, 1.0)
    def coef_of(which: str) -> ops.StencilCoef:
        dy = 10.0 / n
        dx = {"iso": dy, "aniso": 10.0 / (n - 48), "pow2": 10.0 / (2 * n)}[which]
        return ops.StencilCoef.from_physics(1.0, dx, dy, min(dx * dx, dy * dy) / 4.1)

    rect = [ops.interior_rect(n, n)]
    samples: list = []
    stop = threading.Event()

    def sampler():
        while not stop.is_set():
            s = smi_sample()
            s["t"] = time.perf_counter()
            samples.append(s)
            stop.wait(1.0)

    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    idle = smi_sample()
    cap = smi_power_cap()
    rows = []
    for item in a.configs.split(","):
        kind, K, *rest = item.split(":")
        K = int(K)
        which = rest[0] if rest else "iso"
        coef = coef_of(which)
        if kind == "march":
            def launch():
                ops.stencil_step(T2, T, iCp, coef, rect, ops.StencilTuning())
        else:
            tn = ops.StencilTuning(chunk_rows=native().default_chunk_k(max(K, 3), n), kernel=kind,
                                   vec=4, xcd_remap=1)

            def launch():
                ops.stencilk_step(K, T2, T, iCp, coef, rect, tn)
        launch()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        times = []
        while time.perf_counter() - t0 < a.seconds:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch()
            e1.record()
            e1.synchronize()
            times.append(e0.elapsed_time(e1))
        t1 = time.perf_counter()
        win = [s for s in samples if t0 + 1.0 <= s["t"] <= t1]
        pw = [s["power_W"] for s in win if "power_W" in s]
        ck = [s["sclk_MHz"] for s in win if "sclk_MHz" in s]
        rows.append({"kernel": kind, "K": K, "coef": which,
                     "ry": ops.fast5_constants(coef)[0],
                     "ms_per_pass": round(statistics.median(times), 3),
                     "ms_per_step": round(statistics.median(times) / K, 4), "launches": len(times),
                     "power_W": statistics.median(pw) if pw else None,
                     "sclk_MHz": statistics.median(ck) if ck else None, "samples": len(win)})
        print(json.dumps(rows[-1]), flush=True)
    stop.set()
    th.join(5)
    doc = {"tile": n, "idle": idle, "power_cap_W": cap, "rows": rows}
    print(json.dumps(doc), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(doc, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
