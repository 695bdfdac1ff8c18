"""update_halo_ / gather_ semantics against a global ground truth (CPU).

Each rank's local block is a slice of one global array; after corrupting the
halo planes that face a neighbour, update_halo_ must restore exactly the
global values — for 1-D/2-D/3-D fields, several fields per call, staggered
fields (size n+-1), halowidth 2 (overlap 4) and periodic dimensions.
"""

import pytest
import torch

from helpers import run_loopback
from rocm_mpi_amd.parallel import implicit_grid as gg
from rocm_mpi_amd.parallel.halo import gather_, has_halo, update_halo_


def local_block(G, g, shape_local, stagger):
    idx = []
    nd = len(shape_local)
    for ax in range(nd):
        d = nd - 1 - ax
        off = g.coords[d] * (g.nxyz[d] - g.overlaps[d])
        idx.append(torch.arange(off, off + shape_local[ax]) % G.shape[ax])
    return G[torch.meshgrid(*idx, indexing="ij")].clone()


def corrupt(A, g):
    nd = A.dim()
    for d in range(nd):
        if not has_halo(g, A, d):  # e.g. size n-1: no halo along d, left untouched
            continue
        ax = nd - 1 - d
        hw = g.halowidths[d]
        n = A.shape[ax]
        if g.neighbors[d][0] >= 0:
            A.narrow(ax, 0, hw).fill_(-1.0)
        if g.neighbors[d][1] >= 0:
            A.narrow(ax, n - hw, hw).fill_(-1.0)


def spmd(rank, hub, nxyz, dims, periods, overlaps, staggers, nfields):
    gg.init_global_grid(*nxyz, dimx=dims[0], dimy=dims[1], dimz=dims[2], periodx=periods[0],
                        periody=periods[1], periodz=periods[2], overlaps=overlaps, quiet=True,
                        loopback=(hub, rank), select_device=False)
    g = gg.global_grid()
    nd = 3 if nxyz[2] > 1 else (2 if nxyz[1] > 1 else 1)
    fields, expect = [], []
    for f in range(nfields):
        st = staggers[f % len(staggers)]
        shp_l = tuple(nxyz[d] + st[d] for d in reversed(range(nd)))
        shp_g = tuple(g.nxyz_g[d] + st[d] + (0 if not periods[d] else 0) for d in reversed(range(nd)))
        gen = torch.Generator().manual_seed(100 + f)
        G = torch.rand(shp_g, generator=gen, dtype=torch.float64)
        A = local_block(G, g, shp_l, st)
        expect.append(A.clone())
        corrupt(A, g)
        fields.append(A)
    update_halo_(*fields)
    ok = all(torch.equal(a, e) for a, e in zip(fields, expect))
    gg.finalize_global_grid()
    return ok


CASES = [
    # nxyz, dims, periods, overlaps, staggers, nfields
    ((9,), (3, 1, 1), (0, 0, 0), (2, 2, 2), [(0, 0, 0)], 1),
    ((9, 7), (2, 2, 1), (0, 0, 0), (2, 2, 2), [(0, 0, 0)], 1),
    ((9, 7), (2, 2, 1), (0, 0, 0), (2, 2, 2), [(0, 0, 0), (1, 0, 0), (0, 1, 0), (-1, 0, 0)], 4),
    ((12, 10), (2, 2, 1), (0, 0, 0), (4, 4, 2), [(0, 0, 0)], 2),
    ((6, 5, 7), (2, 2, 2), (0, 0, 0), (2, 2, 2), [(0, 0, 0), (0, 0, 1)], 2),
    ((9, 7), (4, 1, 1), (0, 0, 0), (2, 2, 2), [(0, 0, 0)], 1),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"n{c[0]}-d{c[1]}-ol{c[3][0]}-f{c[5]}")
def test_update_halo_matches_global(case):
    nxyz, dims, periods, overlaps, staggers, nf = case
    nxyz3 = tuple(nxyz) + (1,) * (3 - len(nxyz))
    P = dims[0] * dims[1] * dims[2]
    assert all(run_loopback(P, spmd, nxyz3, dims, periods, overlaps, staggers, nf))


def spmd_periodic(rank, hub, P):
    # periodic x on P ranks (P=1 -> local self copy), field values = global index
    n, ol = 8, 2
    gg.init_global_grid(n, 6, 1, dimx=P, periodx=1, quiet=True, loopback=(hub, rank),
                        select_device=False)
    g = gg.global_grid()
    nxg = g.nxyz_g[0]
    off = g.coords[0] * (n - ol)
    gx = (torch.arange(off, off + n) - 1) % nxg  # first local cell is the ghost
    A = gx.to(torch.float64).repeat(6, 1).contiguous()
    want = A.clone()
    A[:, 0] = -1
    A[:, -1] = -1
    update_halo_(A)
    ok = torch.equal(A, want)
    gg.finalize_global_grid()
    return ok


@pytest.mark.parametrize("P", [1, 2, 3])
def test_periodic_halo(P):
    assert all(run_loopback(P, spmd_periodic, P))


def spmd_gather(rank, hub):
    gg.init_global_grid(5, 4, 3, dimx=2, dimy=1, dimz=2, quiet=True, loopback=(hub, rank),
                        select_device=False)
    g = gg.global_grid()
    A = torch.full((3, 4, 5), float(rank), dtype=torch.float64)
    out = gather_(A)
    coords = list(g.coords)
    gg.finalize_global_grid()
    return out, coords


def test_gather_3d_places_blocks_by_coords():
    res = run_loopback(4, spmd_gather)
    G = res[0][0]
    assert G.shape == (6, 4, 10)
    for r, (_, c) in enumerate(res):
        blk = G[c[2] * 3:(c[2] + 1) * 3, c[1] * 4:(c[1] + 1) * 4, c[0] * 5:(c[0] + 1) * 5]
        assert torch.all(blk == r)
    assert all(o is None for o, _ in res[1:])


def spmd_nohalo(rank, hub):
    gg.init_global_grid(9, 7, 1, dimx=2, dimy=2, quiet=True, loopback=(hub, rank),
                        select_device=False)
    try:
        update_halo_(torch.zeros(6, 8, dtype=torch.float64))  # n-1 in x and y: no halo at all
    except ValueError:
        return True
    finally:
        gg.finalize_global_grid()
    return False


def test_field_without_halo_is_rejected():
    assert all(run_loopback(4, spmd_nohalo))


def spmd_dead_peer(rank, hub):
    gg.init_global_grid(9, 7, 1, dimx=2, quiet=True, loopback=(hub, rank), select_device=False)
    try:
        if rank == 1:
            return "died"  # never joins the exchange
        A = torch.zeros(7, 9, dtype=torch.float64)
        try:
            update_halo_(A)
        except RuntimeError as e:
            return str(e)
        return "no error"
    finally:
        gg.finalize_global_grid()


def test_dead_peer_times_out_instead_of_hanging():
    """Failure detection: a missing peer raises after the
    transport timeout rather than blocking forever."""
    out = run_loopback(2, spmd_dead_peer, timeout=2)
    assert out[1] == "died"
    assert "no message from 1" in out[0]


def test_copy_planes_cpu_twin():
    """The batched pack/unpack entry point on host tensors (CPU twin of the
    GPU batch kernel): every copy of the batch lands, nothing else moves."""
    from rocm_mpi_amd import ops

    A = torch.arange(37 * 53, dtype=torch.float64).reshape(37, 53)
    B = torch.zeros_like(A)
    planes = [(slice(0, 37), slice(3, 5)), (slice(2, 6), slice(0, 53)), (slice(0, 0), slice(0, 2)),
              (slice(10, 30), slice(20, 41))]
    ops.copy_planes([(B[r, c], A[r, c]) for r, c in planes])
    ref = torch.zeros_like(A)
    for r, c in planes:
        ref[r, c] = A[r, c]
    assert torch.equal(B, ref)
    with pytest.raises(ValueError):
        ops.copy_planes([(B[:, :1], A[:, :1])] * 9)


def test_ipc_transport_selection():
    """transport="ipc" needs GPU fields; one rank needs no transport."""
    import torch

    from rocm_mpi_amd.parallel.implicit_grid import _choose_transport

    with pytest.raises(ValueError, match="needs a GPU"):
        _choose_transport("ipc", 2, torch.device("cpu"))
    assert _choose_transport("ipc", 1, torch.device("cuda", 0)) == "self"
    assert _choose_transport("ipc", 4, torch.device("cuda", 0)) == "ipc"
    assert _choose_transport("ipc", 4, torch.device("cuda", 0), 4) == "ipc"
    # ranks on several nodes: IPC cannot reach them
    with pytest.raises(ValueError, match="ONE node"):
        _choose_transport("ipc", 8, torch.device("cuda", 0), 4)


def test_shared_gpu_rccl_gives_each_rank_its_own_host(monkeypatch):
    """RMA_RCCL_SHARED_GPU=1: a per-rank NCCL_HOSTID (RCCL then refuses no
    duplicate GPU and uses its socket transport), only with > 1 rank, never
    overriding an explicit setting."""
    import os

    from rocm_mpi_amd.parallel import comm as C

    for k in ("NCCL_HOSTID", "RMA_RCCL_SHARED_GPU"):
        monkeypatch.delenv(k, raising=False)
    assert not C.shared_gpu_rccl(1, 4) and "NCCL_HOSTID" not in os.environ
    monkeypatch.setenv("RMA_RCCL_SHARED_GPU", "1")
    assert not C.shared_gpu_rccl(0, 1) and "NCCL_HOSTID" not in os.environ
    assert C.shared_gpu_rccl(3, 4) and os.environ["NCCL_HOSTID"] == "rma-shared-gpu-rank-3"
    monkeypatch.setenv("NCCL_HOSTID", "mine")
    assert C.shared_gpu_rccl(2, 4) and os.environ["NCCL_HOSTID"] == "mine"


def test_bench_record_rc_is_atomic_across_threads(tmp_path, monkeypatch):
    """bench.record_rc from two threads of one rank (the check watchdog and
    the main thread exiting at once) never leaves an empty rc file."""
    import os
    import sys
    import threading

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    monkeypatch.setenv("RMA_DIAG", f"bench_rc_dir={tmp_path}")
    for it in range(50):
        ts = [threading.Thread(target=bench.record_rc, args=(1, 4 + (j % 3))) for j in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert int((tmp_path / "rc1").read_text()) in (4, 5, 6)
    assert not [p for p in tmp_path.iterdir() if p.name.endswith(".tmp")]
