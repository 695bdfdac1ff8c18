"""Randomised decomposition-invariance of the native GPU path.

P loopback ranks run the native executor on the GPU (planned passes, width-K
exchanges, frame/interior streams) for random configurations (fuzz_cases.py);
every tile must equal the same region of a 1-rank CPU run of the global grid
bitwise (the CPU twins of the same arithmetic). Complements the hand-picked
cases of test_multirank_gpu.py with sizes and depths nobody chose."""
import pytest

from fuzz_cases import check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", range(128))
def test_random_decompositions_match_one_cpu_rank(seed):
    check(seed, "cuda")


@pytest.mark.parametrize("seed", range(12))
def test_random_rccl_self_send_matches_cpu(seed):
    """One rank, periodic in both dims, every halo plane through RCCL
    send/recv to itself (the multi-GPU message pattern on one GPU), random
    tile / K / steps / arithmetic == the CPU run of the same periodic grid."""
    import random

    from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
    from rocm_mpi_amd.parallel import implicit_grid as gg

    r = random.Random(1000 + seed)
    K = r.randint(1, 24)
    nx, ny, nt = 4 * K + r.randint(6, 150), 4 * K + r.randint(6, 90), r.randint(1, 2 * K + 5)
    variant, fast = r.choice(["perf", "perf_hide"]), r.random() < 0.6
    outs = []
    for dev in ("cuda", "cpu"):
        kw = dict(transport="rccl", self_via_transport=True) if dev == "cuda" else dict(device="cpu")
        gg.init_global_grid(nx, ny, 1, periodx=1, periody=1, quiet=True,
                            overlaps=(2 * K, 2 * K, 2), halowidths=(K, K, 1), **kw)
        m = Diffusion2D(DiffusionConfig(variant=variant, nx=nx, ny=ny, nt=nt, quiet=True,
                                        init="random", periods=(1, 1, 0), temporal=K,
                                        fast_math=fast, device=dev))
        m.step(nt)
        outs.append(m.field.cpu().clone())
        m.close()
        gg.finalize_global_grid()
    assert outs[0].equal(outs[1]), (K, nx, ny, nt, variant, fast)


# seeds whose process grid has 2..8 ranks (fuzz_cases.DIMS), a mix of K,
# periodic dimensions and arithmetics
_PROC_SEEDS = [s for s in range(64) if __import__("fuzz_cases").case(s)["dims"] != (1, 1)][:6]


@pytest.mark.parametrize("seed", _PROC_SEEDS)
@pytest.mark.parametrize("transport", ["rccl", "ipc"])
def test_random_decompositions_between_processes(tmp_path, seed, transport):
    """The same random configurations with one PROCESS per rank on cuda:0:
    multi-rank RCCL (RMA_RCCL_SHARED_GPU: its socket transport) and the HIP
    IPC transport; every tile == the 1-rank CPU run's window, bitwise."""
    import numpy as np

    from fuzz_cases import case, spmd
    from helpers import run_loopback, run_procs

    c = case(seed)
    P = c["dims"][0] * c["dims"][1]
    env = {"RMA_TRANSPORT": transport}
    if transport == "rccl":
        env["RMA_RCCL_SHARED_GPU"] = "1"
    run_procs(P, "mp_targets:fuzz_tile", str(tmp_path), seed, env=env, timeout=240)
    metas = [open(tmp_path / f"meta{r}.txt").read().split() for r in range(P)]
    assert all(m[4] == transport for m in metas)
    nxg, nyg = int(metas[0][2]), int(metas[0][3])
    K, ol = c["K"], 2 * c["K"]
    one = dict(c, nx=nxg + ol * c["periods"][0], ny=nyg + ol * c["periods"][1], dims=(1, 1))
    ref = run_loopback(1, spmd, one, "cpu", timeout=180)[0][1]
    for r in range(P):
        cx, cy = int(metas[r][0]), int(metas[r][1])
        T = np.load(tmp_path / f"tile{r}.npy")
        gx0, gy0 = cx * (c["nx"] - ol), cy * (c["ny"] - ol)
        assert np.array_equal(T, ref[gy0:gy0 + c["ny"], gx0:gx0 + c["nx"]]), (c, (cx, cy))
