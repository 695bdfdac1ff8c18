"""Checkpoint / resume of a distributed diffusion run.

The reference has none; here every rank writes its local tile (halo
included) as ``rank<r>.npy`` plus a shared ``meta.json`` (grid, dims, step
count, physics), and ``load_checkpoint`` refuses a checkpoint whose
decomposition or physics differ. Files are plain NumPy (``allow_pickle=False``)
and JSON: nothing executable is ever deserialised.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch


def _meta(model) -> dict:
    g = model.g
    c = model.cfg
    return {"format": "rocm_mpi_amd.checkpoint/1", "variant": c.variant, "nx": c.nx, "ny": c.ny,
            "dims": list(g.dims), "periods": list(g.periods), "nprocs": g.nprocs,
            "nxyz_g": list(g.nxyz_g), "overlaps": list(g.overlaps), "temporal": c.temporal,
            "fast_math": bool(c.fast_math), "steps_done": model.steps_done, "dt": model.dt,
            "dx": model.dx, "dy": model.dy, "lam": c.lam, "Cp0": c.Cp0}


def save_checkpoint(model, path: str) -> str:
    os.makedirs(path, exist_ok=True)
    g = model.g
    model.synchronize()
    np.save(os.path.join(path, f"rank{g.me}.npy"), model.field.detach().cpu().numpy())
    if g.me == 0:
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump(_meta(model), f, indent=1)
    g.comm.barrier()
    return path


def load_checkpoint(model, path: str) -> dict:
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    mine = _meta(model)
    for k in ("nx", "ny", "dims", "periods", "nprocs", "nxyz_g"):
        if meta[k] != mine[k]:
            hint = ""
            if k == "nxyz_g" and meta.get("overlaps") and meta["overlaps"] != mine["overlaps"]:
                hint = (f": written with grid overlaps {meta['overlaps']} (temporal "
                        f"{meta.get('temporal')}), this run has {mine['overlaps']} (--temporal)")
            raise ValueError(f"checkpoint {k}={meta[k]} does not match this run ({mine[k]}){hint}")
    for k in ("dt", "dx", "dy", "lam", "Cp0"):
        if meta[k] != mine[k]:
            raise ValueError(f"checkpoint physics {k}={meta[k]} differs from this run ({mine[k]})")
    arr = np.load(os.path.join(path, f"rank{model.g.me}.npy"), allow_pickle=False)
    t = torch.from_numpy(arr).to(model.device)
    if tuple(t.shape) != tuple(model.T.shape):
        raise ValueError("checkpoint tile shape mismatch")
    model.synchronize()
    # restore into the buffer the model reads next; keep the double buffer consistent
    model.field.copy_(t)
    other = model.T if model.field is model.T2 else model.T2
    if other is not None:
        other.copy_(t)
    model.steps_done = int(meta["steps_done"])
    model.synchronize()
    return meta
