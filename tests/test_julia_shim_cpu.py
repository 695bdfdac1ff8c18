"""The Julia front end (julia/ImplicitGlobalGridMI355X.jl) is a ccall shim over
the C ABI; Julia is not installed here, so its behaviour stays unpinned. What
can be pinned on the CPU: every C function the shim calls is declared in
csrc/include/rma/capi.h and exported by the built librma_core.so, with the
same number of arguments as the ccall passes."""
import os
import re
import subprocess

import pytest

from helpers import ROOT

JL = os.path.join(ROOT, "julia", "ImplicitGlobalGridMI355X.jl")
CAPI = os.path.join(ROOT, "csrc", "include", "rma", "capi.h")
LIB = os.path.join(ROOT, "rocm_mpi_amd", "librma_core.so")


def _ccalls():
    src = open(JL).read()
    out = {}
    # ccall(sym(:name), Ret, (T1, T2, ...), args...)
    for m in re.finditer(r"ccall\(sym\(:(\w+)\),\s*[\w{}]+,\s*\(([^()]*(?:\([^()]*\)[^()]*)*)\)",
                         src):
        types = [t for t in m.group(2).split(",") if t.strip()]
        out.setdefault(m.group(1), set()).add(len(types))
    return out


def _capi_arity():
    src = re.sub(r"/\*.*?\*/|//[^\n]*", "", open(CAPI).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(rma_\w+)\s*\(([^;{]*?)\)\s*;", src):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_every_shim_ccall_is_declared_with_its_arity():
    calls, decl = _ccalls(), _capi_arity()
    assert len(calls) >= 10
    for name, arities in calls.items():
        assert name in decl, f"{name} is called by the Julia shim but not declared in capi.h"
        assert arities == {decl[name]}, (name, arities, decl[name])


@pytest.mark.skipif(not os.path.exists(LIB), reason="librma_core.so not built")
def test_every_shim_ccall_is_exported():
    nm = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True)
    if nm.returncode != 0:
        pytest.skip("nm unavailable")
    exported = {line.split()[-1] for line in nm.stdout.splitlines() if line.strip()}
    missing = sorted(set(_ccalls()) - exported)
    assert not missing, missing


def test_shim_device_index_is_node_local_never_global():
    """the shim's device index comes from the MPI
    shared-memory split when a comm is given (the reference's
    ``Comm_split_type(COMM_TYPE_SHARED)``, scripts/rocmaware_test_selectdevice.jl:7-9),
    else from the launcher's node-local rank variables (the same list as the
    Python side, comm.env_world), and never from the global rank."""
    src = open(JL).read()
    dev_line = [ln for ln in src.splitlines() if re.match(r"\s*dev\s*=", ln)]
    assert len(dev_line) == 1, dev_line
    assert "local_rank" in dev_line[0] and "launcher_local_rank()" in dev_line[0]
    assert not re.search(r"\brank\b", dev_line[0].replace("local_rank", "")), dev_line[0]
    assert "MPI.Comm_split_type(comm, MPI.COMM_TYPE_SHARED" in src
    assert re.search(r"local_rank\s*=\s*MPI\.Comm_rank\(comm_l\)", src)
    m = re.search(r"function launcher_local_rank\(\)(.*?)\nend", src, re.S)
    assert m, "launcher_local_rank missing"
    names = re.findall(r'"([A-Z_]+)"', m.group(1))
    from rocm_mpi_amd.parallel import comm as C
    import inspect
    py = inspect.getsource(C.env_world)
    py_local = re.search(r'local = first\(([^)]*)\)', py).group(1)
    assert names == re.findall(r'"([A-Z_]+)"', py_local)
    assert "return 0" in m.group(1)  # no launcher variable: the node's only rank
