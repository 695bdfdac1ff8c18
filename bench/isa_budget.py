"""ISA-level instruction budget of the deep-pass kernels.

Compiles one pipelined K-step translation unit to gfx950 assembly (or reads a
given ``.s``), finds every row loop of a kernel instantiation (a basic block
range closed by a backward branch) and sorts its instructions into
categories. Per loop the counts are divided by the cell-updates one loop trip
performs per lane (one update = 2 ``v_add_f64`` + 3 ``v_fma_f64`` in the fast5
form, so updates = fma / 3), giving wave-instructions per lane-update; the
arithmetic floor is 5. The whole pass then also pays the strip windows'
recompute, ``W / (W - 2K)`` with ``W = 64 * V`` columns per wave window.

    python bench/isa_budget.py --K 20 24 --out profiles/r5/isa_budget.md

CPU only (hipcc cross-compiles); reference: the update of
``/root/reference/scripts/diffusion_2D_perf.jl:3-13`` (5 fp64 operations per
cell in the fast5 form).
"""
from __future__ import annotations

import argparse
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CATS = [
    ("fp64 arithmetic", re.compile(r"^v_(fma|add|mul|fmac)_f64")),
    ("DPP lane moves", re.compile(r"^v_mov_b32_dpp|^v_mov_b32.*(row_|wave_|quad_perm|row_newbcast)")),
    ("row-register moves", re.compile(r"^v_mov_b64|^v_mov_b32|^v_accvgpr|^v_pk_mov_b32")),
    ("LDS", re.compile(r"^ds_")),
    ("global / LDS-DMA", re.compile(r"^(global_|buffer_|flat_)")),
    ("VALU other (int, select, cmp)", re.compile(r"^v_")),
    ("waitcnt", re.compile(r"^s_waitcnt")),
    ("barrier", re.compile(r"^s_barrier")),
    ("SALU / branch / other scalar", re.compile(r"^s_")),
]
VALU_CATS = ("fp64 arithmetic", "DPP lane moves", "row-register moves",
             "VALU other (int, select, cmp)")


def compile_asm(unit: str, out: str) -> str:
    """The unit's gfx950 assembly, with the unit's own flags of the build
    (rocm_mpi_amd/_build.py UNIT_FLAGS: the K = 20 / 24 scheduler units)."""
    sys.path.insert(0, ROOT)
    from rocm_mpi_amd._build import UNIT_FLAGS

    cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17",
           "-fPIC", "-ffp-contract=off", f"-I{ROOT}/csrc/include", "-munsafe-fp-atomics",
           *UNIT_FLAGS.get(os.path.basename(unit), []),
           "--cuda-device-only", "-S", "-o", out, os.path.join(ROOT, unit)]
    subprocess.run(cmd, check=True, capture_output=True)
    return out


def kernel_body(lines: list[str], mangled_prefix: str) -> list[str]:
    start = None
    for i, ln in enumerate(lines):
        if start is None and ln.startswith(mangled_prefix) and ln.rstrip().endswith(
                ":") is False and ":" in ln.split(";")[0]:
            start = i
            continue
        if start is not None and (ln.startswith(".Lfunc_end") or ln.strip().startswith(".size")):
            return lines[start:i]
    raise SystemExit(f"kernel {mangled_prefix} not found")


def parse(body: list[str]):
    """[(label or None, mnemonic, full text)] and label -> index."""
    insts, labels = [], {}
    for ln in body:
        s = ln.split(";")[0].strip()
        if not s:
            continue
        if s.endswith(":"):
            labels[s[:-1]] = len(insts)
            continue
        if s.startswith("."):
            continue
        insts.append((s.split()[0], s))
    return insts, labels


def category(mn: str, text: str) -> str:
    for name, rx in CATS:
        if rx.search(mn if "dpp" not in name.lower() else text):
            return name
    return "other"


def loops(insts, labels):
    out = []
    for j, (mn, text) in enumerate(insts):
        if mn.startswith("s_cbranch") or mn == "s_branch":
            tgt = text.split()[-1]
            if tgt in labels and labels[tgt] <= j:
                out.append((labels[tgt], j))
    return out


def budget(insts, lo, hi):
    c = collections.Counter()
    fma = add = 0
    for mn, text in insts[lo:hi + 1]:
        cat = category(mn, text)
        c[cat] += 1
        if mn.startswith("v_fma_f64") or mn.startswith("v_fmac_f64"):
            fma += 1
        elif mn.startswith("v_add_f64"):
            add += 1
    return c, fma, add


def mangled(K: int, S: int, V: int, C: int, Ar: int) -> str:
    return f"_ZN3rma4pipe11pipe_kernelILi{K}ELi{S}ELi{V}ELi{Ar}ELi{C}EE"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--K", type=int, nargs="+", default=[20, 24])
    ap.add_argument("--S", type=int, default=4)
    ap.add_argument("--V", type=int, default=4)
    ap.add_argument("--ar", type=int, default=-1,
                    help="arithmetic template (-1: the executor's: 13 = piper without in-level "
                         "barriers at K = 24, 3 = piper elsewhere)")
    ap.add_argument("--unit", default="auto",
                    help="translation unit (auto: the one holding the executor's kernel per K: "
                         "stencil_pipe_r20.hip / _r24.hip / _r.hip)")
    ap.add_argument("--asm", default="", help="an existing .s instead of compiling")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    def unit_of(K):
        if a.unit != "auto":
            return a.unit
        return {20: "csrc/kernels/stencil_pipe_r20.hip",
                24: "csrc/kernels/stencil_pipe_r24.hip"}.get(K, "csrc/kernels/stencil_pipe_r.hip")

    asms = {}
    rows = []
    md = ["| K | loop (stage) | trip insts | lane-updates / trip | " +
          " | ".join(n for n, _ in CATS) + " | VALU total | VALU per update x recompute |",
          "|" + "---|" * (len(CATS) + 5)]
    for K in a.K:
        # the instantiation is named pipe_kernel<K, S, V, C, Ar>? find by prefix K,S,V
        ar = a.ar if a.ar >= 0 else (13 if K == 24 else 3)
        asm = a.asm or asms.setdefault(unit_of(K), compile_asm(
            unit_of(K), f"/tmp/isa_budget_{os.path.basename(unit_of(K))}.s"))
        lines = open(asm).read().splitlines()
        # the plain instantiation (Dir = false; the direct-store variant is Lb1)
        pref = f"_ZN3rma4pipe11pipe_kernelILi{K}ELi{a.S}ELi{a.V}ELi{ar}ELi1ELb0EE"
        body = [ln for ln in lines]
        try:
            kb = kernel_body(body, pref)
        except SystemExit:
            print(f"K={K}: {pref} not in {asm}", file=sys.stderr)
            continue
        insts, labels = parse(kb)
        W = 64 * a.V
        recompute = W / (W - 2 * K)
        found = []
        lps = loops(insts, labels)
        for lo, hi in lps:
            c, fma, add = budget(insts, lo, hi)
            if fma < 12:
                continue  # not a row loop
            text = " ".join(t for _, t in insts[lo:hi + 1])
            lds_dma, store = "global_load_lds" in text, "global_store" in text
            if lds_dma and store:
                continue  # spans the code of two stages (prologue structure)
            role = ("stage 0 (streams T, 1/Cp)" if lds_dma
                    else "last stage (stores T2)" if store else "middle stage")
            found.append((lo, hi, c, fma, add, role))
        # the steady-state row loop of each role: the most updates per trip
        # (the whole unrolled body once; the unrolled loop's side exits to the
        # remainder rows are ranges with fewer updates), then the shortest span
        best = {}
        for t in found:
            b = best.get(t[5])
            if b is None or t[3] > b[3] or (t[3] == b[3] and t[1] - t[0] < b[1] - b[0]):
                best[t[5]] = t
        found = sorted(best.values(), key=lambda t: t[0])
        for n, (lo, hi, c, fma, add, role) in enumerate(found):
            upd = fma / 3.0
            valu = sum(c[k] for k in VALU_CATS)
            per = {k: c[k] / upd for k, _ in CATS}
            rows.append({"K": K, "loop": role, "insts": hi - lo + 1, "updates": upd,
                         "fma": fma, "add": add, "per_update": per,
                         "valu_per_update": valu / upd, "recompute": recompute})
            md.append(f"| {K} | {role} | {hi - lo + 1} | {upd:.0f} | " +
                      " | ".join(f"{per[k]:.3f}" for k, _ in CATS) +
                      f" | {valu / upd:.3f} | {valu / upd * recompute:.3f} |")
    text = "\n".join(md)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
