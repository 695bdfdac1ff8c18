"""update_halo_ on device fields through the native halo engine (loopback
ranks on cuda:0): the CPU suite's global-truth cases (tests/test_halo_cpu.py)
-- 1-D/2-D/3-D, several fields per call, staggered sizes, halowidth 2,
periodic dims. 2-D fields with x AND y neighbours take the merged group
(corner blocks to the diagonal ranks); 3-D fields the per-dimension groups;
RMA_DIAG=no_halo_merged the per-dimension groups everywhere.
"""
import pytest
import torch

from helpers import run_loopback
from rocm_mpi_amd.parallel import implicit_grid as gg
from rocm_mpi_amd.parallel.halo import update_halo_
from test_halo_cpu import CASES, corrupt


def local_block(G, g, shape_local):
    """The rank's block of the global array G; along a periodic dim the first
    local cell is the ghost of global index off - 1 (IGG's periodic layout)."""
    idx = []
    nd = len(shape_local)
    for ax in range(nd):
        d = nd - 1 - ax
        off = g.coords[d] * (g.nxyz[d] - g.overlaps[d]) - (1 if g.periods[d] else 0)
        idx.append(torch.arange(off, off + shape_local[ax]) % G.shape[ax])
    return G[torch.meshgrid(*idx, indexing="ij")].clone()

pytestmark = pytest.mark.gpu


def spmd(rank, hub, nxyz, dims, periods, overlaps, staggers, nfields):
    gg.init_global_grid(*nxyz, dimx=dims[0], dimy=dims[1], dimz=dims[2], periodx=periods[0],
                        periody=periods[1], periodz=periods[2], overlaps=overlaps, quiet=True,
                        loopback=(hub, rank), device="cuda:0")
    g = gg.global_grid()
    assert g.halo is not None
    nd = 3 if nxyz[2] > 1 else (2 if nxyz[1] > 1 else 1)
    fields, expect = [], []
    for f in range(nfields):
        st = staggers[f % len(staggers)]
        shp_l = tuple(nxyz[d] + st[d] for d in reversed(range(nd)))
        shp_g = tuple(g.nxyz_g[d] + st[d] for d in reversed(range(nd)))
        gen = torch.Generator().manual_seed(100 + f)
        G = torch.rand(shp_g, generator=gen, dtype=torch.float64)
        A = local_block(G, g, shp_l)
        expect.append(A.clone())
        corrupt(A, g)
        fields.append(A.to("cuda:0"))
    update_halo_(*fields)
    torch.cuda.current_stream().synchronize()
    ok = all(torch.equal(a.cpu(), e) for a, e in zip(fields, expect))
    gg.finalize_global_grid()
    return ok


PERIODIC = [((9, 7), (2, 2, 1), (1, 1, 0), (2, 2, 2), [(0, 0, 0)], 1),
            ((9, 7), (1, 2, 1), (1, 0, 0), (2, 2, 2), [(0, 0, 0)], 2),
            ((12, 10), (2, 2, 1), (0, 1, 0), (4, 4, 2), [(0, 0, 0), (1, 0, 0)], 2)]


@pytest.mark.parametrize("merged", ["1", "0"])
@pytest.mark.parametrize("case", CASES + PERIODIC,
                         ids=lambda c: f"n{c[0]}-d{c[1]}-p{c[2]}-ol{c[3][0]}-f{c[5]}")
def test_update_halo_on_device_matches_global(case, merged, monkeypatch):
    monkeypatch.setenv("RMA_DIAG", "no_halo_merged" if merged == "0" else "")
    nxyz, dims, periods, overlaps, staggers, nf = case
    nxyz3 = tuple(nxyz) + (1,) * (3 - len(nxyz))
    P = dims[0] * dims[1] * dims[2]
    assert all(run_loopback(P, spmd, nxyz3, dims, periods, overlaps, staggers, nf))
