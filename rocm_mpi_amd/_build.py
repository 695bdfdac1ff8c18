"""In-tree build of the native core ``rocm_mpi_amd._C`` for gfx950.

The reference has no build system: its GPU code is Julia JIT-compiled by
AMDGPU.jl at run time and its environment bootstrap is
``startup.sh:3-17``. Here the HIP kernels and the C++ runtime are compiled
ahead of time with ``hipcc --offload-arch=gfx950`` into one pybind11
extension that lives next to this file (so it ships with the repository
snapshot to a GPU box and is what every process loads).

Usage::

    python -m rocm_mpi_amd._build            # incremental
    python -m rocm_mpi_amd._build --clean    # from scratch

Objects go to ``build/native`` and are rebuilt when their source or any header
under ``csrc/include`` is newer. All device code is compiled with
``-ffp-contract=off`` so the stencil is bit-reproducible against NumPy.

Two libraries: ``librma_core.so`` holds every kernel the executor and the ops
run plus the runtime and the C ABI; ``librma_lab.so`` (``csrc/lab``) holds the
superseded and experimental kernels kept as test oracles and for sweeps. The
lab library is loaded only on request (``_native.load_lab()``) and installs
its kernels in the core's dispatchers.

A stamp next to the libraries (``.build_stamp``) records a hash of every
source and header, the compile flags and the offload arch: a snapshot whose
stamp matches is used as is (no rebuild on a GPU box, whatever the file
mtimes); otherwise the objects are rebuilt incrementally by mtime.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
INC = CSRC / "include"
BUILD = ROOT / "build" / "native"
PKG = ROOT / "rocm_mpi_amd"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("RMA_OFFLOAD_ARCH", "gfx950")
# gfx950 only: the core kernels use CDNA4 instructions (e.g. the 16-byte
# global_load_lds of piper's stage-0 prefetch, csrc/kernels/stencil_pipe.h)
SUPPORTED_ARCHS = ("gfx950",)

# librma_core.so: every kernel the executor / ops run + the runtime + the C ABI
# (usable without Python)
HIP_SOURCES = sorted((CSRC / "kernels").glob("*.hip")) + sorted((CSRC / "runtime").glob("*.cpp"))
# librma_lab.so: superseded / experimental kernels (test oracles, sweeps)
LAB_SOURCES = sorted((CSRC / "lab").glob("*.hip"))
CORE_HOST_SOURCES = sorted((CSRC / "kernels").glob("*.cpp"))
# _C*.so: the pybind11 bindings, linked against librma_core.so ($ORIGIN rpath)
BIND_SOURCES = [CSRC / "bindings" / "module.cpp"]
HOST_SOURCES = CORE_HOST_SOURCES + BIND_SOURCES
EXAMPLES = sorted((ROOT / "examples").glob("*.cpp"))
TOOLS = sorted((ROOT / "bench" / "native").glob("*.hip"))  # standalone probes -> build/bench/


def ext_path() -> Path:
    return PKG / ("_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def core_path() -> Path:
    return PKG / "librma_core.so"


def lab_path() -> Path:
    return PKG / "librma_lab.so"


STAMP = PKG / ".build_stamp"


def _pybind_include() -> str:
    import pybind11

    return pybind11.get_include()


def _hipcc() -> str:
    p = ROCM / "bin" / "hipcc"
    return str(p) if p.exists() else "hipcc"


COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"-I{INC}", "-Wall",
          "-Wno-unused-function", "-Wno-unknown-pragmas"]


# compressed device code objects (the runtime inflates them at load): the
# gfx950 fatbins are ~3.7x smaller, which shrinks every GPU-box push
OFFLOAD = [f"--offload-arch={ARCH}", "--offload-compress"]


# per-unit compiler flags (measured; the unit's header comment says why)
UNIT_FLAGS = {"stencil_pipe_r20.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
              "stencil_pipe_r24.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]}


def _hip_cmd(src: Path, obj: Path) -> list[str]:
    return [_hipcc(), "-x", "hip", *OFFLOAD, *COMMON, *UNIT_FLAGS.get(src.name, []),
            "-munsafe-fp-atomics", "-c", str(src), "-o", str(obj)]


def _host_cmd(src: Path, obj: Path) -> list[str]:
    cxx = os.environ.get("CXX", "g++")
    if src in BIND_SOURCES:  # pybind11 module: hide everything but PyInit__C
        py_inc = sysconfig.get_paths()["include"]
        return [cxx, *COMMON, "-fvisibility=hidden", f"-I{_pybind_include()}", f"-I{py_inc}",
                "-c", str(src), "-o", str(obj)]
    return [cxx, *COMMON, "-c", str(src), "-o", str(obj)]


def _headers() -> list[Path]:
    return sorted(list(INC.rglob("*.h")) + list((CSRC / "kernels").glob("*.h")))


def source_stamp() -> str:
    """Hash of every source and header, the flags and the arch."""
    h = hashlib.sha1()
    # flags with the checkout's absolute path taken out: a snapshot of the same
    # tree under another directory (a GPU box) has the same stamp
    flags = " ".join(COMMON + OFFLOAD + [sysconfig.get_config_var("EXT_SUFFIX") or ""] +
                     [f"{k}:{' '.join(v)}" for k, v in sorted(UNIT_FLAGS.items())])
    h.update(flags.replace(str(ROOT), "<root>").encode())
    for p in sorted(set(HIP_SOURCES + LAB_SOURCES + HOST_SOURCES + EXAMPLES + TOOLS + _headers())):
        h.update(str(p.relative_to(ROOT)).encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def _stale(src: Path, obj: Path, newest_header: float) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or newest_header > t


def build(clean: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    """Compile (incrementally) and link ``rocm_mpi_amd/_C*.so``; returns its path."""
    if ARCH not in SUPPORTED_ARCHS:
        raise SystemExit(f"rocm_mpi_amd builds for {', '.join(SUPPORTED_ARCHS)} (MI355X) only, "
                         f"RMA_OFFLOAD_ARCH={ARCH!r}: the core kernels use CDNA4 instructions "
                         "(16-byte LDS-DMA loads in the pipelined K-step kernel)")
    if clean and BUILD.exists():
        shutil.rmtree(BUILD)
    headers = _headers()
    newest_header = max((p.stat().st_mtime for p in headers), default=0.0)
    out, core, lab = ext_path(), core_path(), lab_path()
    stamp = source_stamp()
    old = STAMP.read_text().strip() if STAMP.exists() else None
    missing = [p.name for p in (out, core, lab) if not p.exists()]
    if not clean and not missing and old == stamp:
        # the libraries were built from exactly these sources, flags and arch
        # (a repository snapshot on a GPU box carries the .so files and the
        # stamp but not the object files)
        print(f"[build] reused {out.name}, {core.name}, {lab.name}: stamp {stamp[:12]} matches "
              "the sources, flags and arch", flush=True)
        return out
    reason = ("--clean" if clean else f"missing {', '.join(missing)}" if missing
              else "no stamp" if old is None else f"stamp {old[:12]} != sources {stamp[:12]}")
    BUILD.mkdir(parents=True, exist_ok=True)
    jobs = jobs or min(16, os.cpu_count() or 4)
    todo = []
    objs = []
    for src in HIP_SOURCES + LAB_SOURCES + HOST_SOURCES:
        obj = BUILD / (src.parent.name + "_" + src.name + ".o")
        objs.append(obj)
        if _stale(src, obj, newest_header):
            cmd = _host_cmd(src, obj) if src in HOST_SOURCES else _hip_cmd(src, obj)
            todo.append((src, cmd))

    def run(item):
        src, cmd = item
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return src

    print(f"[build] compiled {len(todo)} of {len(objs)} sources ({reason})", flush=True)
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for src in ex.map(run, todo):
                print(f"[rocm_mpi_amd build] compiled {src.relative_to(ROOT)}", flush=True)
    core = core_path()
    pairs = list(zip(objs, HIP_SOURCES + LAB_SOURCES + HOST_SOURCES))
    core_objs = [o for o, src in pairs if src not in BIND_SOURCES and src not in LAB_SOURCES]
    lab_objs = [o for o, src in pairs if src in LAB_SOURCES]
    bind_objs = [o for o, src in pairs if src in BIND_SOURCES]

    def newer(target: Path, deps) -> bool:
        return not target.exists() or any(d.stat().st_mtime > target.stat().st_mtime for d in deps)

    def link(target: Path, cmd: list[str]) -> None:
        tmp = target.with_suffix(".tmp.so")
        full = cmd + ["-o", str(tmp)]
        if verbose:
            print(" ".join(full), flush=True)
        r = subprocess.run(full, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(full)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, target)
        print(f"[rocm_mpi_amd build] linked {target.relative_to(ROOT)}", flush=True)

    if newer(core, core_objs):
        link(core, [_hipcc(), "-shared", "-fPIC", *OFFLOAD, *map(str, core_objs),
                    "-Wl,-soname,librma_core.so", f"-L{ROCM / 'lib'}", "-lrccl", "-lamdhip64",
                    "-ldl", "-lpthread", f"-Wl,-rpath,{ROCM / 'lib'}"])
    if newer(lab, lab_objs + [core]):
        link(lab, [_hipcc(), "-shared", "-fPIC", *OFFLOAD, *map(str, lab_objs),
                   "-Wl,-soname,librma_lab.so", f"-L{PKG}", "-lrma_core", "-Wl,-rpath,$ORIGIN",
                   f"-L{ROCM / 'lib'}", "-lamdhip64", f"-Wl,-rpath,{ROCM / 'lib'}"])
    out = ext_path()
    if newer(out, bind_objs + [core]):
        link(out, ["g++", "-shared", "-fPIC", *map(str, bind_objs), f"-L{PKG}", "-lrma_core",
                   "-Wl,-rpath,$ORIGIN"])
    exdir = ROOT / "build" / "examples"
    for src in EXAMPLES:
        exe = exdir / src.stem
        if newer(exe, [src, core]) or newest_header > exe.stat().st_mtime:
            exdir.mkdir(parents=True, exist_ok=True)
            cmd = [_hipcc(), "-x", "hip", *OFFLOAD, *COMMON, str(src), "-o",
                   str(exe), f"-L{PKG}", "-lrma_core", f"-Wl,-rpath,{PKG}",
                   f"-L{ROCM / 'lib'}", "-lamdhip64", f"-Wl,-rpath,{ROCM / 'lib'}"]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"example build failed: {src}\n{r.stdout}\n{r.stderr}")
            print(f"[rocm_mpi_amd build] built {exe.relative_to(ROOT)}", flush=True)
    tooldir = ROOT / "build" / "bench"
    for src in TOOLS:
        exe = tooldir / src.stem
        if newer(exe, [src]):
            tooldir.mkdir(parents=True, exist_ok=True)
            cmd = [_hipcc(), "-x", "hip", *OFFLOAD, "-O3", "-std=c++17", str(src),
                   "-o", str(exe), f"-L{ROCM / 'lib'}", "-lrccl", f"-Wl,-rpath,{ROCM / 'lib'}"]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"tool build failed: {src}\n{r.stdout}\n{r.stderr}")
            print(f"[rocm_mpi_amd build] built {exe.relative_to(ROOT)}", flush=True)
    STAMP.write_text(stamp + "\n")
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    build(clean=a.clean, jobs=a.jobs, verbose=a.verbose)
    return 0


if __name__ == "__main__":
    sys.exit(main())
