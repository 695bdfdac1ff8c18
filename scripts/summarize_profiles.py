#!/usr/bin/env python
"""Turn gpurun_out/ measurements into committed summaries under profiles/.

    python scripts/summarize_profiles.py [--tag r1]
Reads (when present): gpurun_out/sweep16k.json, gpurun_out/pmc_{fetch,write}/
run_counter_collection.csv, gpurun_out/prof*/run_kernel_stats.csv,
gpurun_out/bench*.log; writes profiles/*.md / *.json / *.csv copies.
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def sweep_md(path):
    d = json.load(open(path))
    r = d["results"]
    lines = [f"## Kernel sweep, {d['n']}x{d['n']} fp64, {d['rounds']} rounds x {d['iters']} "
             f"launches (interleaved, one process) on {d.get('device', 'MI355X')}", "",
             "GB/s = T_eff model bytes (24 B/cell for the stencil; 16 B/elem copy, 24 B/elem "
             "triad) / median kernel time.", "",
             "| variant | median ms | GB/s (median) | GB/s (best) |", "|---|---|---|---|"]
    for k in sorted(r, key=lambda k: -r[k]["GBps_median"]):
        v = r[k]
        lines.append(f"| {k} | {v['median_ms']:.3f} | {v['GBps_median']:.0f} | "
                     f"{v['GBps_best']:.0f} |")
    lines += ["", f"best stencil: **{d['best_march']} = {d['best_march_GBps']:.0f} GB/s**; "
              f"best copy probe {d['copy_GBps']:.0f} GB/s; best triad probe (same 2R+1W byte "
              f"mix) {d['triad_GBps']:.0f} GB/s; stencil / triad = {d['best_vs_triad']:.3f}", ""]
    return "\n".join(lines)


def pmc_md(fetch_csv, write_csv, n=16384):
    by = collections.OrderedDict()
    for f, key in ((fetch_csv, "FETCH_SIZE"), (write_csv, "WRITE_SIZE")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            by.setdefault(k, {}).setdefault(key, []).append(float(r["Counter_Value"]))
    arr_kb = n * n * 8 / 1024
    lines = ["## HBM bytes per dispatch (rocprofv3 PMC, KB; FETCH_SIZE reads half of wide "
             "streaming reads on gfx950 (MI355X_MICROARCH.md §HBM), so reads = 2 x FETCH)", "",
             f"array = {n}^2 fp64 = {arr_kb:.0f} KB", "",
             "| kernel | FETCH_SIZE | 2xFETCH / array | WRITE_SIZE / array |", "|---|---|---|---|"]
    for k, v in by.items():
        if "FETCH_SIZE" not in v or "WRITE_SIZE" not in v:
            continue
        f = sorted(v["FETCH_SIZE"])[len(v["FETCH_SIZE"]) // 2]
        w = sorted(v["WRITE_SIZE"])[len(v["WRITE_SIZE"]) // 2]
        lines.append(f"| {k} | {f:.0f} | {2 * f / arr_kb:.3f} | {w / arr_kb:.3f} |")
    lines += ["", "Ideal stencil: 2 arrays read (T, 1/Cp) + 1 written (T2) = 2.000 / 1.000.", ""]
    return "\n".join(lines)


def stats_md(path):
    rows = list(csv.DictReader(open(path)))
    lines = ["| kernel | calls | avg us | total % |", "|---|---|---|---|"]
    for r in rows[:12]:
        lines.append(f"| {short(r['Name'])[:70]} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['Percentage']):.2f} |")
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r1")
    a = ap.parse_args()
    os.makedirs(P, exist_ok=True)
    md = [f"# Measured profiles ({a.tag})", ""]
    sw = os.path.join(G, "sweep16k.json")
    if os.path.exists(sw):
        shutil.copy(sw, os.path.join(P, f"sweep_16k_{a.tag}.json"))
        md.append(sweep_md(sw))
    fc = os.path.join(G, "pmc_fetch", "run_counter_collection.csv")
    wc = os.path.join(G, "pmc_write", "run_counter_collection.csv")
    if os.path.exists(fc) and os.path.exists(wc):
        shutil.copy(fc, os.path.join(P, f"pmc_fetch_16k_{a.tag}.csv"))
        shutil.copy(wc, os.path.join(P, f"pmc_write_16k_{a.tag}.csv"))
        md.append(pmc_md(fc, wc))
    for st in sorted(glob.glob(os.path.join(G, "prof*", "run_kernel_stats.csv"))):
        name = os.path.basename(os.path.dirname(st))
        shutil.copy(st, os.path.join(P, f"kernel_stats_{name}_{a.tag}.csv"))
        md += [f"## rocprofv3 --kernel-trace --stats: {name}", "", stats_md(st), ""]
    benches = sorted(glob.glob(os.path.join(G, "bench*.log")))
    if benches:
        md += ["## bench.py runs", ""]
        for b in benches:
            for line in open(b):
                if line.startswith("{"):
                    d = json.loads(line)
                    c = d["config"]
                    md.append(f"- `{os.path.basename(b)}`: {c['model']} local {c['local_grid']} "
                              f"x{d['n_gpus']} GPU: **{d['value']} GB/s**, {d['ms_per_step']} "
                              f"ms/step ({d['steps']} steps)")
        md.append("")
    out = os.path.join(P, f"SUMMARY_{a.tag}.md")
    open(out, "w").write("\n".join(md))
    print(out)


if __name__ == "__main__":
    main()
