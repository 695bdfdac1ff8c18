import faulthandler
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
# the multi-process GPU tests run every rank on the one GPU of the test box:
# select_device refuses that outside this functional mode (inherited by the
# ranks the tests spawn; tests of the refusal unset it)
os.environ.setdefault("RMA_SHARED_GPU", "1")

# Crash evidence that survives a truncated stdout tail (the
# faulting thread's frames of the round-4 SIGSEGV fell into the bytes the
# driver cut): every thread's stack on a fatal signal, plus breadcrumbs of the
# multi-rank case that was running (tests/helpers.py), in a small log under
# the run's output directory.
LOG_DIR = os.environ.get("RMA_TEST_LOG_DIR", os.path.join(ROOT, "gpurun_out", "pytest_faults"))
_fault_file = None


def breadcrumb(msg: str) -> None:
    """Append one line to the crash log (flushed: it must be on disk before a
    native crash can take the process down)."""
    if _fault_file is not None:
        _fault_file.write(msg.rstrip() + "\n")
        _fault_file.flush()


def pytest_configure(config):
    global _fault_file
    try:
        os.makedirs(LOG_DIR, exist_ok=True)
        _fault_file = open(os.path.join(LOG_DIR, f"faults_{os.getpid()}.log"), "a", buffering=1)
        faulthandler.enable(file=_fault_file, all_threads=True)
    except OSError:
        _fault_file = None
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")
    # build the native core once per session (incremental; a no-op when fresh)
    from rocm_mpi_amd import _build

    _build.build()


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _fresh_grid(request):
    """Every test starts and ends without a global grid."""
    from rocm_mpi_amd.parallel import implicit_grid as gg

    breadcrumb(f"test {request.node.nodeid}")
    yield
    if gg.grid_is_initialized():
        try:
            gg.finalize_global_grid()
        except Exception:
            gg._set_grid(None, False)
