"""Run the five BASELINE.json configurations and report T_eff + weak scaling.

BASELINE.json names five configs (ap 256² on CPU, kp 16384² on 1 GPU, perf
2x1 on 2 GPUs, perf_hide 2x2 on 4 and 4x2 on 8 with the tile sized to the
288 GB HBM). Each is an ``--preset`` of the entry points
(``rocm_mpi_amd/apps/cli.py``); this driver launches them through
``rocm_mpi_amd.launch`` (one process per GPU), collects every run's JSON
record and computes the weak-scaling efficiency the reference never defines
(SURVEY.md §5.5): ``E(N) = T_eff_per_gpu(N) / T_eff_per_gpu(1)`` at the SAME
local tile, using a 1-GPU run of the same variant and tile as denominator.

Configs needing more GPUs than ``--max-gpus`` are reported as skipped (the
8-GPU numbers come from the driver's scaling run of ``bench.py``), unless
``--shared-gpu``: then the multi-rank presets run as FUNCTIONAL checks with all
ranks on the one visible GPU, real RCCL between the processes
(``RMA_RCCL_SHARED_GPU``: RCCL's socket transport instead of xGMI) and a
``--shared-nx`` tile; their records say so and carry no efficiency.

    python bench/baseline_configs.py --out profiles/baseline_configs.json
    python bench/baseline_configs.py --only kp16k,perf_2x1 --nt 200
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from rocm_mpi_amd.apps.cli import PRESETS  # noqa: E402

# GPUs each preset needs (its process grid); ap256_cpu runs one CPU rank
NPROCS = {"ap256_cpu": 1, "kp16k": 1, "perf_2x1": 2, "hide_2x2": 4, "hide_4x2_288GB": 8}


def gpu_count() -> int:
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return 0


def run(preset: str, nprocs: int, nt: int | None, extra: list[str], timeout: float,
        env: dict | None = None) -> dict:
    """Launch one preset (or its 1-rank reference run) and return the JSON record."""
    variant = PRESETS[preset]["variant"]
    args = ["--preset", preset, "--json", "--quiet", "--no-vis"]
    if nt:
        args += ["--nt", str(nt)]
    if nprocs != NPROCS[preset]:
        args += ["--dims", "1,1"]  # the single-GPU denominator of E(N)
    cmd = [sys.executable, "-m", "rocm_mpi_amd.launch", "-n", str(nprocs), "-m",
           f"rocm_mpi_amd.apps.diffusion_2D_{variant}", "--", *args, *extra]
    t0 = time.time()
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, **(env or {})))
    rec = {"preset": preset, "nprocs": nprocs, "cmd": " ".join(cmd), "rc": p.returncode,
           "wall_s": round(time.time() - t0, 2)}
    for line in p.stdout.splitlines():
        s = line.split("] ", 1)[-1].strip()  # launcher prefixes "[rank] "
        if s.startswith("{") and '"teff"' in s:
            rec["result"] = json.loads(s)
    if p.returncode != 0 or "result" not in rec:
        rec["error"] = (p.stderr or p.stdout)[-2000:]
    return rec


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--only", default="", help="comma-separated preset names")
    ap.add_argument("--max-gpus", type=int, default=None)
    ap.add_argument("--nt", type=int, default=None, help="override the 1000 steps")
    ap.add_argument("--no-reference-runs", action="store_true",
                    help="skip the 1-GPU runs that give E(N)")
    ap.add_argument("--timeout", type=float, default=1800)
    ap.add_argument("--shared-gpu", action="store_true",
                    help="run the multi-rank presets on ONE GPU (functional, RCCL between "
                         "processes over its socket transport)")
    ap.add_argument("--shared-nx", type=int, default=2048, help="local tile of --shared-gpu runs")
    ap.add_argument("--out", default="")
    a, extra = ap.parse_known_args(argv)
    ngpu = gpu_count() if a.max_gpus is None else a.max_gpus
    names = [n for n in PRESETS if not a.only or n in a.only.split(",")]

    report = {"gpus_visible": ngpu, "configs": []}
    single = {}  # (variant, auto/nx) -> 1-GPU per-GPU T_eff
    for name in names:
        need = NPROCS[name]
        on_gpu = PRESETS[name].get("device") != "cpu"
        shared = on_gpu and need > ngpu and a.shared_gpu and ngpu >= 1
        if on_gpu and need > ngpu and not shared:
            report["configs"].append({"preset": name, "skipped": f"needs {need} GPUs, {ngpu} visible"})
            print(f"{name:16s} skipped (needs {need} GPUs)", flush=True)
            continue
        if shared:
            rec = run(name, need, a.nt,
                      extra + ["--no-auto-size", "--nx", str(a.shared_nx), "--ny", str(a.shared_nx)],
                      a.timeout, env={"RMA_RCCL_SHARED_GPU": "1", "RMA_TRANSPORT": "rccl"})
            rec["shared_gpu_functional"] = True
            res = rec.get("result")
            report["configs"].append(rec)
            print(f"{name:16s} n={need} on ONE GPU (functional, RCCL sockets): "
                  + (f"transport {res.get('transport')} local {res['nx']}x{res['ny']} global "
                     f"{res['nxg']}x{res['nyg']}" if res else f"FAILED rc={rec['rc']}\n"
                     f"{rec.get('error', '')}"), flush=True)
            continue
        rec = run(name, need, a.nt, extra, a.timeout)
        res = rec.get("result")
        if res and need > 1 and not a.no_reference_runs:
            key = (res["variant"], res["nx"], res["ny"])
            if key not in single:
                one = run(name, 1, a.nt, extra + ["--no-auto-size", "--nx", str(res["nx"]), "--ny", str(res["ny"])]
                          if PRESETS[name].get("auto_size") else extra, a.timeout)
                single[key] = one.get("result", {}).get("teff")
                rec["reference_1gpu"] = one
            if single[key]:
                rec["weak_scaling_eff"] = res["teff"] / single[key]
        report["configs"].append(rec)
        if res:
            e = rec.get("weak_scaling_eff")
            print(f"{name:16s} n={need} local {res['nx']}x{res['ny']} T_eff/GPU "
                  f"{res['teff']:.1f} GB/s  aggregate {res.get('teff_total', float('nan')):.1f} GB/s"
                  + (f"  E={e:.3f}" if e else ""), flush=True)
        else:
            print(f"{name:16s} FAILED rc={rec['rc']}\n{rec.get('error', '')}", flush=True)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(report, f, indent=1)
    return 0 if all("error" not in c for c in report["configs"]) else 1


if __name__ == "__main__":
    sys.exit(main())
