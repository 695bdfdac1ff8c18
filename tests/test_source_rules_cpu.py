"""Source rules of the native runtime that tests cannot catch by running.

The executor's and transports' device work runs on NON-blocking HIP streams,
which are not ordered after the legacy null stream. A null-stream
``hipMemset`` / ``hipMemcpy`` on memory those streams use next is therefore a
race (round 5: the fused-pass counter zeroed that way was sometimes still
garbage at the first signalling launch and the bounded frame wait timed out,
profiles/SUMMARY_r5.md section 6). Initialise such memory with the ``*Async``
form on the consuming stream (and wait for it when the host reads it)."""
import os
import re

from helpers import ROOT

RUNTIME = os.path.join(ROOT, "csrc", "runtime")


def test_no_null_stream_memset_or_memcpy_in_the_runtime():
    bad = []
    for name in sorted(os.listdir(RUNTIME)):
        if not name.endswith(".cpp"):
            continue
        src = open(os.path.join(RUNTIME, name)).read()
        src = re.sub(r"//[^\n]*", "", src)  # comments may name the rule
        for m in re.finditer(r"\bhip(Memset|Memcpy)(2D)?\s*\(", src):
            line = src.count("\n", 0, m.start()) + 1
            bad.append(f"{name}:{line}: {m.group(0)}")
    assert not bad, "null-stream memory ops in the runtime: " + ", ".join(bad)


# --- configuration surface ------------------------------
TUNING = {"RMA_TRANSPORT", "RMA_RCCL_STRICT", "RMA_RCCL_BLOCKING", "RMA_RCCL_LIB",
          "RMA_RCCL_SHARED_GPU", "RMA_SHARED_GPU", "RMA_COMM_TIMEOUT", "RMA_TEARDOWN_TIMEOUT",
          "RMA_IPC_MODE", "RMA_IPC_MAILBOX_MB", "RMA_EXEC_FUSED", "RMA_EXEC_FUSED_TIMEOUT",
          "RMA_GATHER_MAX_BYTES", "RMA_NUM_THREADS", "RMA_AUTOBUILD", "RMA_OFFLOAD_ARCH",
          "RMA_DIAG"}


def _env_reads():
    """Every RMA_* variable the package, the native sources and bench.py read."""
    pats = [re.compile(r'getenv\(\s*"(RMA_[A-Z0-9_]+)"'),
            re.compile(r'environ(?:\.get|\.setdefault|\.pop)?\(\s*"(RMA_[A-Z0-9_]+)"'),
            re.compile(r'environ\[\s*"(RMA_[A-Z0-9_]+)"\s*\]'),
            re.compile(r'env_(?:double|choice)\(\s*"(RMA_[A-Z0-9_]+)"'),
            re.compile(r'for \(const char\* var : \{"(RMA_[A-Z0-9_]+)"')]
    found = {}
    roots = [os.path.join(ROOT, d) for d in ("csrc", "rocm_mpi_amd")] + [os.path.join(ROOT, "bench.py")]
    for r in roots:
        files = [r] if os.path.isfile(r) else [os.path.join(dp, f) for dp, _, fs in os.walk(r)
                                                 for f in fs if f.endswith((".py", ".cpp", ".h", ".hip"))]
        for f in files:
            src = open(f, errors="replace").read()
            for p in pats:
                for m in p.finditer(src):
                    found.setdefault(m.group(1), set()).add(os.path.relpath(f, ROOT))
    return found


def test_every_env_knob_is_a_documented_tuning_variable_or_rma_diag():
    found = _env_reads()
    extra = {k: sorted(v) for k, v in found.items() if k not in TUNING}
    assert not extra, f"undocumented RMA_* variables (fold them into RMA_DIAG): {extra}"
    assert len(TUNING) <= 20
    doc = open(os.path.join(ROOT, "docs", "TUNING.md")).read()
    table = set(re.findall(r"^\| `(RMA_[A-Z0-9_]+)` \|", doc, re.M))
    assert table == TUNING, (sorted(table - TUNING), sorted(TUNING - table))


def test_rma_diag_keys_agree_between_python_and_cpp():
    from rocm_mpi_amd.config import DIAG_KEYS

    src = open(os.path.join(ROOT, "csrc", "runtime", "config.cpp")).read()
    body = src[src.index("kDiagKeys[] = {"):src.index("nullptr};")]
    cpp = re.findall(r'^\s*"([a-z0-9_]+)",', body, re.M)
    assert cpp == list(DIAG_KEYS)
    doc = open(os.path.join(ROOT, "docs", "TUNING.md")).read()
    for k in cpp:
        assert f"`{k}" in doc, f"RMA_DIAG key {k} not documented in docs/TUNING.md"
