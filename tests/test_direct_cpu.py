"""Direct-store halos, host side (the GPU behaviour: tests/test_direct_halo_gpu.py):
the direction table the executor and the model share, the refusal on the CPU
path, and the IPC export format checks that run before any HIP call."""
import pytest

from helpers import run_loopback
from rocm_mpi_amd._native import native
from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
from rocm_mpi_amd.parallel import implicit_grid as gg


def test_direction_table_is_the_executors():
    """kDirI / kDirJ order: (-1,-1), (0,-1), (1,-1), (-1,0), (1,0), (-1,1),
    (0,1), (1,1); opposite(d) = 7 - d, which the pass-count words rely on."""
    dirs = native().Executor.direct_dirs
    assert dirs == [(-1, -1), (0, -1), (1, -1), (-1, 0), (1, 0), (-1, 1), (0, 1), (1, 1)]
    for d, (i, j) in enumerate(dirs):
        assert dirs[7 - d] == (-i, -j)


def _ranks(rank, hub, dims, periods):
    gg.init_global_grid(40, 30, 1, dimx=dims[0], dimy=dims[1], periodx=periods[0],
                        periody=periods[1], quiet=True, loopback=(hub, rank))
    m = Diffusion2D(DiffusionConfig(variant="perf", nx=40, ny=30, nt=1, quiet=True,
                                    dims=dims, periods=(*periods, 0), device="cpu"))
    try:
        return m.g.coords[:2], m._direct_ranks()
    finally:
        m.close()
        gg.finalize_global_grid()


@pytest.mark.parametrize("dims,periods", [((2, 2), (0, 0)), ((3, 2), (1, 1)), ((2, 1), (1, 0))])
def test_direct_ranks_are_the_neighbours_in_each_direction(dims, periods):
    """Every direction's rank is the one at coords + (i, j) (wrapped where
    periodic), -1 outside a non-periodic grid; diagonals only where both axis
    neighbours exist (the corner cells need both)."""
    res = run_loopback(dims[0] * dims[1], _ranks, dims, periods)
    at = {tuple(c): r for r, (c, _) in enumerate(res)}
    dirs = native().Executor.direct_dirs
    for c, ranks in res:
        for (i, j), got in zip(dirs, ranks):
            x, y = c[0] + i, c[1] + j
            if periods[0]:
                x %= dims[0]
            if periods[1]:
                y %= dims[1]
            inside = 0 <= x < dims[0] and 0 <= y < dims[1]
            assert got == (at[(x, y)] if inside else -1), (c, (i, j), got)


def test_halo_direct_refused_on_the_cpu_path():
    gg.init_global_grid(40, 30, 1, periodx=1, periody=1, quiet=True)
    try:
        with pytest.raises(ValueError, match="native GPU executor"):
            Diffusion2D(DiffusionConfig(variant="perf_hide", nx=40, ny=30, nt=4, quiet=True,
                                        periods=(1, 1, 0), device="cpu", fast_math=True,
                                        temporal=4, halo_direct=True))
    finally:
        gg.finalize_global_grid()


def test_ipc_map_rejects_malformed_exports_before_any_hip_call():
    m = native().IpcMap()
    with pytest.raises(RuntimeError, match="IPC pointer export"):
        m.open(b"too short")
    assert m.mappings == 0


def test_entry_points_take_halo_direct():
    """--halo-direct reaches the model config of the perf / perf_hide entry
    points (the reference-named scripts) and is refused for the others."""
    from rocm_mpi_amd.apps.cli import resolve

    cfg, _ = resolve("perf_hide", ["--nx", "260", "--ny", "260", "--nt", "40", "--temporal", "8",
                                   "--halo-direct", "--device", "cpu"])
    assert cfg.halo_direct and cfg.fast_math and cfg.temporal > 1
    cfg, _ = resolve("perf", ["--nx", "130", "--ny", "130", "--nt", "20", "--device", "cpu"])
    assert not cfg.halo_direct
    with pytest.raises(SystemExit):
        resolve("kp", ["--nx", "130", "--ny", "130", "--halo-direct"])
