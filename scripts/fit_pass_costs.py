#!/usr/bin/env python
"""Emit the planner's per-depth pass-cost tables (csrc/runtime/plan.cpp) from
bench/pass_sweep.py results: rel = pass time / one-step march kernel time on
the same tile, for the kernel the executor runs at each depth (fast5: the
pipelined kernel; canonical: march K=1, two-step K=2, lds_dpp K=3/4, the
canonical pipelined kernel from K=5), missing depths interpolated linearly.

    python scripts/fit_pass_costs.py profiles/pass_sweep_r2.json profiles/pass_sweep_{16384,8192,4096}_r2.json
"""
import json
import os
import sys

KMAX = 24


def fill(vals: dict) -> list:
    ks = sorted(vals)
    out = []
    for K in range(1, KMAX + 1):
        if K in vals:
            out.append(vals[K])
            continue
        lo = max([k for k in ks if k < K], default=None)
        hi = min([k for k in ks if k > K], default=None)
        if lo is not None and hi is not None:
            out.append(vals[lo] + (vals[hi] - vals[lo]) * (K - lo) / (hi - lo))
        else:  # extrapolate from the last two points
            a, b = ks[-2], ks[-1]
            out.append(vals[b] + (vals[b] - vals[a]) / (b - a) * (K - b))
    return out


def tables(path: str):
    d = json.load(open(path))
    rows = d["rows"]

    def rel(kind, K, stages=None):
        for r in rows:
            if r["kernel"] == kind and r["K"] == K and (r.get("chunk_rows") is None or True):
                if stages is None or r["stages"] == stages:
                    return r["rel"]
        return None

    from_default = {}
    # the executor's own kernel per depth (pass_sweep.py --exec) when present,
    # else the first (default-chunk, default-stage) ring-kernel row per depth
    src = "exec" if any(r["kernel"] == "exec" for r in rows) else "pipe"
    for r in rows:
        if r["kernel"] == src and r["K"] not in from_default:
            from_default[r["K"]] = r["rel"]
    fast = fill(from_default)
    can = {1: 1.0}
    if rel("two_step", 2):
        can[2] = rel("two_step", 2)
    for K in (3, 4):
        if rel("lds_dpp", K):
            can[K] = rel("lds_dpp", K)
    for r in rows:
        if r["kernel"] == "pipec" and r["K"] >= 5 and r["K"] not in can:
            can[r["K"]] = r["rel"]
    return d["tile"], fast, fill(can)


def piper_ratios(paths) -> dict:
    """Per-depth piper / pipe pass-time ratios from same-run sweeps (round 3:
    the executor's fast kernel from K = 10 on the 288 GB tile class)."""
    r = {}
    for path in paths:
        rows = json.load(open(path))["rows"]
        pipe = {x["K"]: x["ms_per_pass"] for x in rows if x["kernel"] == "pipe"}
        for x in rows:
            if x["kernel"] == "piper" and x["K"] in pipe and x.get("chunk_rows") == next(
                    y["chunk_rows"] for y in rows if y["kernel"] == "pipe" and y["K"] == x["K"]):
                r[x["K"]] = x["ms_per_pass"] / pipe[x["K"]]
    return r


def apply_ratios(fast: list, ratios: dict, kmin: int) -> list:
    """Scale the fast5 table by the piper ratios at K >= kmin (depths between
    measured ones interpolated)."""
    ks = sorted(k for k in ratios if k >= kmin)
    out = list(fast)
    for K in range(kmin, KMAX + 1):
        if K in ratios:
            f = ratios[K]
        else:
            lo = max([k for k in ks if k < K], default=ks[0])
            hi = min([k for k in ks if k > K], default=ks[-1])
            f = ratios[lo] if lo == hi else ratios[lo] + (ratios[hi] - ratios[lo]) * (K - lo) / (hi - lo)
        out[K - 1] = fast[K - 1] * f
    return out


PIPER_SWEEPS_101376 = ["r3/pass_sweep_piper_lowK_101120.json", "r3/pass_sweep_piper_glds_boxE.json"]

# round 4: piper's row loop unrolled by 6 at K = 17..20; same-box A/B against the
# round-3 unroll by 3 (lab kernel piper_u3) per tile class
U6_SWEEPS = {101376: "r4/u6_ab_all_stages.json", 16384: "r4/u6_16384.json",
             8192: "r4/u6_8192.json", 4096: "r4/u6_4096.json"}


def u6_ratios(path: str) -> dict:
    """Per-depth piper / piper_u3 pass-time ratios of one same-run sweep."""
    rows = json.load(open(path))["rows"]
    u3 = {x["K"]: x["ms_per_pass"] for x in rows if x["kernel"] == "piper_u3"}
    return {x["K"]: x["ms_per_pass"] / u3[x["K"]] for x in rows
            if x["kernel"] == "piper" and x["K"] in u3}


def apply_u6(fast: list, ratios: dict) -> list:
    """Scale the measured depths (K = 17..20) by the unroll-by-6 ratios
    (rounded to the table's 3 decimals after the round-3 scaling, as committed)."""
    out = list(fast)
    for K, f in ratios.items():
        out[K - 1] = round(round(fast[K - 1], 3) * f, 3)
    return out


# round 6 (profiles/r6/sched_strategy_ab.md): the K = 20 unit under the iterative-ILP
# scheduler (288 GB class, previous vs adopted library, 3 alternations) and the K = 24
# kernel without in-level sched_barriers under it (same process as the previous piper,
# per tile class)
R6_K20 = {101376: ("r6/sched_ab/r20_sweep_base_{}.json", "r6/sched_ab/r20_sweep_r20_{}.json")}
R6_K24 = {101376: "r6/sched_ab/r24/sweep_0.json", 16384: "r6/sched_ab/r24/sweep_16384.json",
          8192: "r6/sched_ab/r24/sweep_8192.json"}


def _exec_ms(path: str, K: int, kernel: str = "exec") -> float:
    with open(path) as f:
        d = json.load(f)
    return next(r["ms_per_pass"] for r in d["rows"] if r["kernel"] == kernel and r["K"] == K)


def r6_ratios(tile: int, root: str) -> dict:
    """{K: new / old pass time} of the round-6 kernel changes measured at this tile class."""
    out = {}
    if tile in R6_K20:
        old, new = R6_K20[tile]
        o = [_exec_ms(os.path.join(root, old.format(i)), 20) for i in (1, 2, 3)]
        n = [_exec_ms(os.path.join(root, new.format(i)), 20) for i in (1, 2, 3)]
        out[20] = sum(n) / sum(o)
    if tile in R6_K24:
        p = os.path.join(root, R6_K24[tile])
        out[24] = _exec_ms(p, 24) / _exec_ms(p, 24, "piper")
    return out


def apply_r6(fast: list, ratios: dict) -> list:
    """Scale the committed table entries (3 decimals) by the round-6 ratios."""
    out = list(fast)
    for K, f in ratios.items():
        out[K - 1] = round(round(fast[K - 1], 3) * f, 3)
    return out


def fmt(name, vals):
    body = ", ".join(f"{v:.3f}" for v in vals)
    return f"    {{{body}}},  // {name}"


if __name__ == "__main__":
    for p in sys.argv[1:]:
        tile, fast, can = tables(p)
        print(f"// tile {tile}: {p}")
        print(fmt(f"fast5 {tile}", fast))
        print(fmt(f"canonical {tile}", can))
