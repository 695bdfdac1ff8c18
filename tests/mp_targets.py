"""Process entry points for multi-process (gloo) tests; see helpers.run_procs."""
import os

import numpy as np


def diffusion(rank, world, outdir, variant, nx, ny, nt, dims, transport="gloo", init="gaussian"):
    from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
    from rocm_mpi_amd.parallel import implicit_grid as gg

    m = Diffusion2D(DiffusionConfig(variant=variant, nx=nx, ny=ny, nt=nt, dims=tuple(dims) + (0,),
                                    transport=transport, quiet=True, init=init, init_on="host",
                                    b_width=(4, 2), device="cpu"))
    res = m.run() if nt > 10 else None
    if res is None:
        m.step(nt)
    Tv = m.gather_interior()
    if gg.global_grid().me == 0:
        np.save(os.path.join(outdir, "Tv.npy"), Tv.numpy())
        with open(os.path.join(outdir, "meta.txt"), "w") as f:
            g = gg.global_grid()
            f.write(f"{g.nxyz_g[0]} {g.nxyz_g[1]} {g.transport}")
            if res is not None:
                f.write(f" {res.teff_total} {res.timed_steps}")
    m.close()


def ring(rank, world, outdir):
    from rocm_mpi_amd.apps import rocmaware_test_selectdevice as app

    vals = app.run(4, transport="gloo", verbose=False)
    np.save(os.path.join(outdir, f"ring{rank}.npy"), np.array(vals))
    from rocm_mpi_amd.parallel import comm as C

    C.shutdown_distributed()


def collectives(rank, world, outdir):
    from rocm_mpi_amd.parallel import implicit_grid as gg

    me, dims, nprocs, coords, comm = gg.init_global_grid(6, 6, 1, quiet=True, device="cpu")
    s = comm.allreduce(float(rank + 1), "sum")
    mx = comm.allreduce(float(rank), "max")
    gg.tic()
    t = gg.toc()
    np.save(os.path.join(outdir, f"coll{rank}.npy"), np.array([s, mx, t, nprocs] + list(dims)))
    gg.finalize_global_grid()


def diffusion_gpu(rank, world, outdir, variant, nx, ny, nt, dims):
    from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
    from rocm_mpi_amd.parallel import implicit_grid as gg

    m = Diffusion2D(DiffusionConfig(variant=variant, nx=nx, ny=ny, nt=nt, dims=tuple(dims) + (0,),
                                    quiet=True, init="gaussian", init_on="host", b_width=(4, 2),
                                    device="cuda:0"))
    m.step(nt)
    Tv = m.gather_interior()
    g = gg.global_grid()
    if g.me == 0:
        np.save(os.path.join(outdir, "Tv.npy"), Tv.numpy())
        with open(os.path.join(outdir, "meta.txt"), "w") as f:
            f.write(f"{g.nxyz_g[0]} {g.nxyz_g[1]} {g.transport}")
    m.close()


def diffusion_tiles(rank, world, outdir, variant, nx, ny, nt, dims, temporal, device="cpu"):
    """Each rank saves its full local field (halo incl.) and coords: temporal
    blocking uses overlap 2K, so tiles are compared with golden windows."""
    from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
    from rocm_mpi_amd.parallel import implicit_grid as gg

    m = Diffusion2D(DiffusionConfig(variant=variant, nx=nx, ny=ny, nt=nt, dims=tuple(dims) + (0,),
                                    quiet=True, init="random", device=device,
                                    temporal=temporal))
    m.step(nt)
    g = gg.global_grid()
    np.save(os.path.join(outdir, f"tile{g.me}.npy"), m.field.cpu().numpy())
    with open(os.path.join(outdir, f"meta{g.me}.txt"), "w") as f:
        f.write(f"{g.coords[0]} {g.coords[1]} {g.nxyz_g[0]} {g.nxyz_g[1]} {g.overlaps[0]} "
                f"{g.overlaps[1]} {g.transport}")
    m.close()


def node_local(rank, world, outdir, ranks_per_node):
    """Fake multi-node placement: no LOCAL_RANK / LOCAL_WORLD_SIZE in the
    environment, a per-'node' hostname instead (MPI.Comm_split_type analogue,
    SURVEY.md §4.5); the global grid's device choice follows the local rank."""
    for k in ("LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        os.environ.pop(k, None)
    from rocm_mpi_amd.config import diag_with

    os.environ["RMA_DIAG"] = diag_with(hostname=f"node{rank // ranks_per_node}")
    from rocm_mpi_amd.parallel import comm as C
    from rocm_mpi_amd.parallel import implicit_grid as gg

    C.init_distributed("gloo")
    local, lsize = C.node_local_rank(rank, world)
    gg.init_global_grid(8, 8, 1, quiet=True, device="cpu", init_dist=False)
    g = gg.global_grid()
    np.save(os.path.join(outdir, f"local{rank}.npy"),
            np.array([local, lsize, g.local_rank, g.local_size]))
    gg.finalize_global_grid()
    from rocm_mpi_amd.parallel import comm as C

    C.shutdown_distributed()


def slurm_env(rank, world, outdir):
    """srun-style launch (the reference's `srun -n N --mpi=pmix ./runme.sh`):
    only SLURM_PROCID / SLURM_NTASKS / SLURM_LOCALID in the environment."""
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        os.environ.pop(k, None)
    os.environ.update({"SLURM_PROCID": str(rank), "SLURM_NTASKS": str(world),
                       "SLURM_LOCALID": str(rank)})
    from rocm_mpi_amd.parallel import implicit_grid as gg

    me, dims, nprocs, coords, comm = gg.init_global_grid(10, 10, 1, quiet=True, device="cpu")
    s = comm.allreduce(float(me), "sum")
    g = gg.global_grid()
    np.save(os.path.join(outdir, f"slurm{rank}.npy"),
            np.array([me, nprocs, g.local_rank, g.local_size, s]))
    gg.finalize_global_grid()


def user_example(rank, world, outdir, nx, ny, nt, dims):
    """examples/diffusion_2D_user.py on gloo ranks (CPU twins)."""
    import importlib.util

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location(
        "diffusion_2D_user", os.path.join(root, "examples", "diffusion_2D_user.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    T0, T, _ = mod.diffusion2D(nx, ny, nt, device="cpu", dims=dims, quiet=True)
    if rank == 0:
        np.save(os.path.join(outdir, "T0.npy"), T0.numpy())
        np.save(os.path.join(outdir, "T.npy"), T.numpy())


def ring_gpu(rank, world, outdir, transport):
    """The reference smoke test's device-buffer ring on cuda (every rank on the
    one visible GPU)."""
    from rocm_mpi_amd.apps import rocmaware_test_selectdevice as app

    vals = app.run(4, transport=transport, verbose=False)
    np.save(os.path.join(outdir, f"ring{rank}.npy"), np.array(vals))
    from rocm_mpi_amd.parallel import comm as C

    C.shutdown_distributed()


def ipc_overflow(rank, world, outdir):
    """A halo message larger than the IPC mailbox fails loudly on every rank
    (before any rank waits for another), then the grid still finalizes."""
    import torch

    from rocm_mpi_amd.parallel import implicit_grid as gg
    from rocm_mpi_amd.parallel.halo import update_halo_

    gg.init_global_grid(130, 66, 1, dimx=world, quiet=True, device="cuda:0")
    assert gg.global_grid().transport == "ipc"
    A = torch.zeros((66, 130), dtype=torch.float64, device="cuda:0")
    msg = ""
    try:
        update_halo_(A)
    except RuntimeError as e:
        msg = str(e)
    torch.cuda.synchronize()
    gg.finalize_global_grid()
    with open(os.path.join(outdir, f"err{rank}.txt"), "w") as f:
        f.write(msg)


def ipc_overflow_then_ring(rank, world, outdir):
    """a group whose LATER peer overflows the mailbox must fail
    before any copy or flag of an EARLIER peer happened, so the transport
    stays in step: the next, valid ring exchange works on every rank."""
    import torch

    from rocm_mpi_amd.parallel import comm as C
    from rocm_mpi_amd.parallel import implicit_grid as gg

    gg.init_global_grid(130, 66, 1, dimx=world, periodx=1, quiet=True, device="cuda:0")
    comm = gg.global_grid().comm
    assert isinstance(comm, C.IpcComm)
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    small = torch.full((4,), float(rank), dtype=torch.float64, device="cuda:0")
    big = torch.zeros(comm.native.mailbox_bytes // 8 + 1, dtype=torch.float64, device="cuda:0")
    rs, rb = torch.zeros_like(small), torch.zeros_like(big)
    msg = ""
    try:  # small to the next rank first, then too many bytes to the previous one
        comm.exchange([C.P2P("send", small, nxt), C.P2P("send", big, prv),
                       C.P2P("recv", rs, prv), C.P2P("recv", rb, nxt)])
    except RuntimeError as e:
        msg = str(e)
    assert "RMA_IPC_MAILBOX_MB" in msg and not comm.native.poisoned, msg
    for it in range(3):
        recv = torch.full((4,), -1.0, dtype=torch.float64, device="cuda:0")
        comm.sendrecv(small + it, nxt, recv, prv)
        torch.cuda.synchronize()
        assert recv.tolist() == [float(prv + it)] * 4, (it, recv.tolist())
    gg.finalize_global_grid()
    with open(os.path.join(outdir, f"ok{rank}.txt"), "w") as f:
        f.write("1")


def halo_device(rank, world, outdir, nxyz, dims, periods, overlaps, staggers, nfields):
    """update_halo_ of device fields (the native engine over RMA_TRANSPORT's
    transport, every process on cuda:0) against the global truth."""
    import sys

    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_halo_cpu import corrupt
    from test_halo_gpu import local_block

    from rocm_mpi_amd.parallel import implicit_grid as gg
    from rocm_mpi_amd.parallel.halo import update_halo_

    gg.init_global_grid(*nxyz, dimx=dims[0], dimy=dims[1], dimz=dims[2], periodx=periods[0],
                        periody=periods[1], periodz=periods[2], overlaps=overlaps, quiet=True,
                        device="cuda:0")
    g = gg.global_grid()
    nd = 3 if nxyz[2] > 1 else (2 if nxyz[1] > 1 else 1)
    fields, expect = [], []
    for f in range(nfields):
        st = staggers[f % len(staggers)]
        shp_l = tuple(nxyz[d] + st[d] for d in reversed(range(nd)))
        shp_g = tuple(g.nxyz_g[d] + st[d] for d in reversed(range(nd)))
        G = torch.rand(shp_g, generator=torch.Generator().manual_seed(100 + f),
                       dtype=torch.float64)
        A = local_block(G, g, shp_l)
        expect.append(A.clone())
        corrupt(A, g)
        fields.append(A.to("cuda:0"))
    update_halo_(*fields)
    torch.cuda.synchronize()
    ok = all(torch.equal(a.cpu(), e) for a, e in zip(fields, expect))
    transport = g.transport
    gg.finalize_global_grid()
    with open(os.path.join(outdir, f"ok{rank}.txt"), "w") as fh:
        fh.write(f"{int(ok)} {transport}")


def fuzz_tile(rank, world, outdir, seed):
    """One random configuration of tests/fuzz_cases.py run by a real process
    per rank (RMA_TRANSPORT decides the transport); saves the tile + coords."""
    from fuzz_cases import case
    from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
    from rocm_mpi_amd.parallel import implicit_grid as gg

    c = case(seed)
    K, dims, per = c["K"], c["dims"], c["periods"]
    gg.init_global_grid(c["nx"], c["ny"], 1, dimx=dims[0], dimy=dims[1], periodx=per[0],
                        periody=per[1], overlaps=(2 * K, 2 * K, 2), halowidths=(K, K, 1),
                        quiet=True, device="cuda:0")
    g = gg.global_grid()
    m = Diffusion2D(DiffusionConfig(variant=c["variant"], nx=c["nx"], ny=c["ny"], nt=c["nt"],
                                    init="random", quiet=True, dims=(*dims, 0), temporal=K,
                                    fast_math=c["fast"], b_width=c["bw"], device="cuda:0",
                                    periods=(*per, 0)))
    assert m.executor is not None
    m.step(c["nt"])
    np.save(os.path.join(outdir, f"tile{g.me}.npy"), m.field.cpu().numpy())
    with open(os.path.join(outdir, f"meta{g.me}.txt"), "w") as f:
        f.write(f"{g.coords[0]} {g.coords[1]} {g.nxyz_g[0]} {g.nxyz_g[1]} {g.transport}")
    m.close()
    gg.finalize_global_grid()


def direct_tiles(rank, world, outdir, nx, ny, nt, dims, periods, K, direct):
    """Processes sharing cuda:0 (RMA_TRANSPORT decides the exchange when
    direct is off): perf_hide fast-math K-step passes; with direct on the
    kernels store the neighbours' halos into their IPC-mapped fields
    (DiffusionExecutor::set_direct). Saves the tile, coords and the direct
    counters."""
    from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
    from rocm_mpi_amd.parallel import implicit_grid as gg

    gg.init_global_grid(nx, ny, 1, dimx=dims[0], dimy=dims[1], periodx=periods[0],
                        periody=periods[1], overlaps=(2 * K, 2 * K, 2), halowidths=(K, K, 1),
                        quiet=True, device="cuda:0")
    g = gg.global_grid()
    m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=nx, ny=ny, nt=nt, init="random",
                                    quiet=True, dims=(*dims, 0), periods=(*periods, 0),
                                    temporal=K, fast_math=True, device="cuda:0",
                                    halo_direct=bool(direct)))
    m.step(nt)
    m.synchronize()
    ex = m.executor
    maps = m._ipc_map.mappings if getattr(m, "_ipc_map", None) is not None else 0
    info = f"{int(ex.direct)} {ex.direct_passes} {ex.passes_done} {maps}"
    np.save(os.path.join(outdir, f"tile{g.me}.npy"), m.field.cpu().numpy())
    with open(os.path.join(outdir, f"meta{g.me}.txt"), "w") as f:
        f.write(f"{g.coords[0]} {g.coords[1]} {g.transport} {info}")
    m.close()
    gg.finalize_global_grid()
