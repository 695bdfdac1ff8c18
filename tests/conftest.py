import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
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
def _fresh_grid():
    """Every test starts and ends without a global grid."""
    from rocm_mpi_amd.parallel import implicit_grid as gg

    yield
    if gg.grid_is_initialized():
        try:
            gg.finalize_global_grid()
        except Exception:
            gg._set_grid(None, False)
