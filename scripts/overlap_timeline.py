#!/usr/bin/env python
"""Overlap of the boundary work with the interior from a rocprofv3 kernel trace.

Reads ``run_kernel_trace.csv`` (``rocprofv3 --kernel-trace``; memory copies
done by blit kernels appear there too, ``run_memory_copy_trace.csv`` is read
when present) of a perf_hide run and classifies every GPU operation by its
HIP stream: the stream(s) whose kernels are the long pipelined interior passes
are "interior", every other operation (frame kernels, pack/unpack, copies) is
"boundary". Reports how much boundary time runs while an interior kernel is
running (1.0 = the exchange and frame are fully hidden), plus a per-stream
table. Usage:

    python scripts/overlap_timeline.py gpurun_out/r2t/trace [--md out.md]
    python scripts/overlap_timeline.py profiles/traces_r2/loopback2_k24_kernel_trace.csv --from-pass 4
"""
from __future__ import annotations

import argparse
import collections
import csv
import os


def load(d: str) -> list:
    ops = []
    kt = d if os.path.isfile(d) else os.path.join(d, "run_kernel_trace.csv")
    d = os.path.dirname(kt)
    for r in csv.DictReader(open(kt)):
        ops.append(("kernel", r["Kernel_Name"].replace("(anonymous namespace)::", "")
                    .split("(")[0].replace("void ", ""),
                    r.get("Stream_Id", r.get("Queue_Id")), int(r["Start_Timestamp"]),
                    int(r["End_Timestamp"])))
    mt = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(mt):
        for r in csv.DictReader(open(mt)):
            ops.append(("copy", r.get("Direction", "copy"), r.get("Stream_Id", "?"),
                        int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return ops


def union(iv: list) -> list:
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def covered(s: int, e: int, u: list) -> int:
    tot = 0
    for a, b in u:
        if b <= s:
            continue
        if a >= e:
            break
        tot += min(b, e) - max(a, s)
    return tot


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--md", default="")
    ap.add_argument("--from-pass", type=int, default=0,
                    help="start the window at the n-th long interior kernel (skip warm-up passes)")
    ap.add_argument("--interior-frac", type=float, default=0.5,
                    help="a stream is 'interior' if its longest pipelined kernel lasts at least "
                         "this fraction of the longest one in the trace")
    ap.add_argument("--window", default="",
                    help="restrict to [first start, last end] of operations whose name contains "
                         "this (e.g. rccl: the run with RCCL traffic)")
    a = ap.parse_args(argv)
    ops = load(a.trace_dir)
    # skip setup work (init / fill kernels) before the first pipelined pass
    t1 = max(o[4] for o in ops)
    if a.window:
        sel = [o for o in ops if a.window in o[1]]
        ops = [o for o in ops if o[3] >= min(x[3] for x in sel) and o[4] <= max(x[4] for x in sel)]
    longest = max((o[4] - o[3] for o in ops if "pipe_kernel" in o[1]), default=0)
    thr = a.interior_frac * longest
    t0 = min((o[3] for o in ops if "pipe_kernel" in o[1]), default=0)
    long_starts = sorted(o[3] for o in ops if "pipe_kernel" in o[1] and o[4] - o[3] >= thr)
    if a.from_pass and len(long_starts) > a.from_pass:
        t0 = long_starts[a.from_pass]
    ops = [o for o in ops if o[3] >= t0 and o[4] <= t1]
    streams = collections.defaultdict(list)
    for o in ops:
        streams[o[2]].append(o)
    interior_streams = {s for s, L in streams.items()
                        if any("pipe_kernel" in o[1] and o[4] - o[3] >= thr for o in L)}
    iu = union([(o[3], o[4]) for s in interior_streams for o in streams[s]])
    bnd = [o for s, L in streams.items() if s not in interior_streams for o in L]
    b_total = sum(o[4] - o[3] for o in bnd)
    b_hidden = sum(covered(o[3], o[4], iu) for o in bnd)
    wall = max(o[4] for o in ops) - min(o[3] for o in ops)
    busy = sum(b - a_ for a_, b in iu)
    lines = ["| stream | role | ops | busy ms | under an interior kernel | kernels (top 3 by time) |",
             "|---|---|---|---|---|---|"]
    for s, L in sorted(streams.items(), key=lambda kv: str(kv[0])):
        by = collections.Counter()
        for o in L:
            by[o[1][:60]] += o[4] - o[3]
        top = ", ".join(f"{k} {v / 1e6:.2f}" for k, v in by.most_common(3))
        role = "interior" if s in interior_streams else "boundary"
        tot = sum(o[4] - o[3] for o in L)
        hid = "" if role == "interior" else \
            f"{sum(covered(o[3], o[4], iu) for o in L) / max(tot, 1):.1%}"
        lines.append(f"| {s} | {role} | {len(L)} | {tot / 1e6:.2f} | {hid} | {top} |")
    summary = (f"window {wall / 1e6:.2f} ms; interior streams busy {busy / 1e6:.2f} ms "
               f"({busy / max(wall, 1):.1%} of the window); boundary work {b_total / 1e6:.3f} ms, "
               f"of which {b_hidden / 1e6:.3f} ms ({b_hidden / max(b_total, 1):.1%}) ran while an "
               f"interior kernel was running")
    text = summary + "\n\n" + "\n".join(lines) + "\n"
    print(text)
    if a.md:
        with open(a.md, "w") as f:
            f.write(text)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
