"""Multi-rank native GPU path on ONE MI355X.

RCCL refuses two ranks on one GPU, so the multi-rank production path (native
halo engine + overlapped executor with hi/lo-priority streams) is exercised
with the device loopback transport: N logical ranks = N threads, each with its
own streams, messages = D2D copies ordered by events with RCCL's completion
semantics. RCCL itself is exercised with send/recv-to-self (periodic
self-neighbours routed through the transport) and single-rank collectives.
"""
import numpy as np
import pytest
import torch

import golden
from helpers import run_loopback, run_procs
from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
from rocm_mpi_amd.parallel import implicit_grid as gg

pytestmark = pytest.mark.gpu


def spmd(rank, hub, variant, nx, ny, nt, dims, periods=(0, 0, 0), init="gaussian", bw=(5, 3),
         graph=False):
    gg.init_global_grid(nx, ny, 1, dimx=dims[0], dimy=dims[1], periodx=periods[0],
                        periody=periods[1], quiet=True, loopback=(hub, rank))
    g = gg.global_grid()
    assert g.device.type == "cuda" and g.halo is not None
    m = Diffusion2D(DiffusionConfig(variant=variant, nx=nx, ny=ny, nt=nt, init=init,
                                    init_on="host", b_width=bw, quiet=True, dims=dims,
                                    periods=periods, use_graph=graph, graph_steps=6))
    assert m.executor is not None
    m.step(nt)
    Tv = m.gather_interior()
    out = (Tv.numpy().copy() if Tv is not None else None, m.g.nxyz_g)
    m.close()
    gg.finalize_global_grid()
    return out


@pytest.mark.parametrize("variant", ["perf_hide", "perf", "kp"])
@pytest.mark.parametrize("P,dims", [(2, (2, 1)), (4, (2, 2)), (8, (4, 2))])
def test_loopback_gpu_equals_golden(variant, P, dims):
    nx, ny, nt = 260, 134, 23
    Tv, (nxg, nyg, _) = run_loopback(P, spmd, variant, nx, ny, nt, dims, timeout=120)[0]
    G = golden.run(nxg, nyg, nt)
    assert np.array_equal(Tv, G[1:-1, 1:-1])


def spmd_tiles(rank, hub, variant, nx, ny, nt, dims, K=2, periods=(0, 0, 0), graph=False):
    """temporal=K on an overlap-2K grid; returns (coords, local field, global sizes)."""
    gg.init_global_grid(nx, ny, 1, dimx=dims[0], dimy=dims[1], periodx=periods[0],
                        periody=periods[1], overlaps=(2 * K, 2 * K, 2), halowidths=(K, K, 1),
                        quiet=True, loopback=(hub, rank))
    m = Diffusion2D(DiffusionConfig(variant=variant, nx=nx, ny=ny, nt=nt, init="random",
                                    quiet=True, dims=dims, periods=periods, temporal=K,
                                    use_graph=graph, graph_steps=8, chunk2=0))
    assert m.executor is not None
    m.step(nt)
    out = (m.g.coords, m.field.cpu().numpy().copy(), m.g.nxyz_g)
    m.close()
    gg.finalize_global_grid()
    return out


@pytest.mark.parametrize("variant", ["perf_hide", "perf"])
@pytest.mark.parametrize("P,dims", [(1, (1, 1)), (2, (2, 1)), (4, (2, 2)), (8, (4, 2))])
@pytest.mark.parametrize("nt,K", [(22, 2), (15, 2), (27, 4), (40, 6), (19, 8)])
def test_loopback_gpu_temporal_equals_golden(variant, P, dims, nt, K):
    """Native executor, K-step kernel + width-K exchange (frame on the
    high-priority stream, interior on the low one): every tile == golden."""
    from rocm_mpi_amd import ops

    nx, ny = 300, 134
    res = run_loopback(P, spmd_tiles, variant, nx, ny, nt, dims, K, timeout=120)
    nxg, nyg, _ = res[0][2]
    T0 = torch.empty((nyg, nxg), dtype=torch.float64)
    ops.init_random_(T0, ops.TileGeometry(0, 0, nxg, nyg, 1.0, 1.0), seed=1234)
    G = golden.run(nxg, nyg, nt, T0=T0.numpy())
    for coords, T, _ in res:
        gx0, gy0 = coords[0] * (nx - 2 * K), coords[1] * (ny - 2 * K)
        assert np.array_equal(T, G[gy0:gy0 + ny, gx0:gx0 + nx])


@pytest.mark.parametrize("graph,K", [(False, 2), (True, 2), (False, 6), (True, 4)])
def test_temporal_single_rank_periodic_and_graph(graph, K):
    """1 rank, periodic (self exchange of width K), optional hipGraph replay
    == the 1-step executor."""
    def run(temporal, g):
        gg.init_global_grid(258, 130, 1, periodx=1, periody=1, overlaps=(2 * K, 2 * K, 2),
                            halowidths=(K, K, 1), quiet=True)
        m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=258, ny=130, nt=1,
                                        init="random", quiet=True, periods=(1, 1, 0),
                                        temporal=temporal, use_graph=g, graph_steps=8))
        m.step(19)
        f = m.field.cpu().clone()
        m.close()
        gg.finalize_global_grid()
        return f
    assert torch.equal(run(K, graph), run(1, False))


def test_loopback_gpu_reference_oracle():
    Tv, (nxg, nyg, _) = run_loopback(4, spmd, "perf_hide", 128, 128, 1000, (2, 2))[0]
    assert float(Tv.max()) == pytest.approx(0.397865, abs=5e-7)
    assert np.array_equal(Tv, golden.run(254, 254, 1000)[1:-1, 1:-1])


def test_loopback_gpu_periodic():
    a = run_loopback(4, spmd, "perf_hide", 200, 100, 30, (2, 2), periods=(1, 1, 0),
                     init="random")[0][0]
    b = run_loopback(4, spmd, "perf", 200, 100, 30, (2, 2), periods=(1, 1, 0),
                     init="random")[0][0]
    assert np.array_equal(a, b)


def test_graph_falls_back_on_non_capturable_transport():
    with pytest.warns(RuntimeWarning, match="cannot be stream-captured"):
        Tv, (nxg, nyg, _) = run_loopback(2, spmd, "perf_hide", 200, 100, 8, (2, 1), graph=True,
                                         timeout=60)[0]
    assert np.array_equal(Tv, golden.run(nxg, nyg, 8)[1:-1, 1:-1])


def test_native_executor_refuses_graph_on_loopback():
    from rocm_mpi_amd._native import native

    n = native()
    hub = n.LoopbackHub(2, 5.0)
    ep = n.LoopbackEndpoint(hub, 0)
    halo = n.HaloExchanger(ep, 0, [[1, 1], [-1, -1], [-1, -1]])
    assert not halo.capturable()
    T = torch.zeros(64, 64, dtype=torch.float64, device="cuda")
    with pytest.raises(RuntimeError, match="capturable"):
        n.Executor(T.data_ptr(), T.data_ptr(), T.data_ptr(), 64, 64, 0, (-1.0, 1.0, 1.0, 0.1),
                   use_graph=1, halo=halo)


@pytest.mark.parametrize("graph", [False, True])
def test_rccl_self_send_periodic(graph):
    """Single rank, periodic: halo planes travel through RCCL send/recv to self
    == local self-copy path (captured in a hipGraph when graph=True: the local
    copy path captures; the RCCL path refuses capture and runs eagerly)."""
    outs = []
    for via in (True, False):
        gg.init_global_grid(300, 200, 1, periodx=1, periody=1, quiet=True, transport="rccl",
                            self_via_transport=via)
        assert gg.global_grid().transport == "rccl"
        m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=300, ny=200, nt=20, quiet=True,
                                        init="random", periods=(1, 1, 0), b_width=(4, 4),
                                        use_graph=graph, graph_steps=6))
        assert m.use_graph == (graph and not via)
        m.step(20)
        outs.append(m.field.cpu().clone())
        m.close()
        gg.finalize_global_grid()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("K,fast,nt", [(16, True, 37), (8, False, 19)])
def test_rccl_self_send_periodic_kstep(K, fast, nt):
    """The bench's multi-rank message pattern through RCCL on one GPU: a
    periodic single rank with width-K halos (overlap 2K) sends its packed
    x-planes and contiguous y-planes to itself through RCCL send/recv once per
    K-step pass (plus the remainder pass) == the local self-copy path."""
    outs = []
    for via in (True, False):
        gg.init_global_grid(600, 300, 1, periodx=1, periody=1, quiet=True, transport="rccl",
                            overlaps=(2 * K, 2 * K, 2), halowidths=(K, K, 1),
                            self_via_transport=via)
        m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=600, ny=300, nt=nt, quiet=True,
                                        init="random", periods=(1, 1, 0), temporal=K,
                                        fast_math=fast))
        m.step(nt)
        outs.append(m.field.cpu().clone())
        m.close()
        gg.finalize_global_grid()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("blocking", [False, True])
def test_rccl_single_rank_collectives(blocking, monkeypatch):
    """Non-blocking init (default: ncclCommInitRankConfig blocking=0 + polled
    timeout) and the blocking communicator give the same results."""
    monkeypatch.setenv("RMA_RCCL_BLOCKING", "1" if blocking else "0")
    me, dims, n, coords, comm = gg.init_global_grid(64, 64, 1, quiet=True, transport="rccl")
    assert comm.name == "rccl"
    assert comm.native.nonblocking == (not blocking)
    comm.barrier()
    assert comm.allreduce(3.5, "sum") == 3.5
    t = torch.arange(10, dtype=torch.float64, device="cuda")
    parts = comm.gather(t)
    assert len(parts) == 1 and torch.equal(parts[0], t)
    gg.tic()
    assert gg.toc() >= 0
    gg.finalize_global_grid()


def test_staged_transport_two_processes(tmp_path):
    """IGG_ROCMAWARE_MPI=0 parity: GPU fields, host-staged exchange, 2 processes."""
    run_procs(2, "mp_targets:diffusion_gpu", str(tmp_path), "perf_hide", 130, 66, 25, (2, 1),
              env={"RMA_TRANSPORT": "staged"})
    Tv = np.load(tmp_path / "Tv.npy")
    nxg, nyg, transport = open(tmp_path / "meta.txt").read().split()[:3]
    assert transport == "staged"
    assert np.array_equal(Tv, golden.run(int(nxg), int(nyg), 25)[1:-1, 1:-1])


def spmd_fast(rank, hub, nx, ny, nt, dims, K, fast):
    gg.init_global_grid(nx, ny, 1, dimx=dims[0], dimy=dims[1], overlaps=(2 * K, 2 * K, 2),
                        halowidths=(K, K, 1), quiet=True, loopback=(hub, rank))
    m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=nx, ny=ny, nt=nt, init="random",
                                    quiet=True, dims=dims, temporal=K, fast_math=fast))
    m.step(nt)
    out = (m.g.coords, m.field.cpu().numpy().copy(), m.g.nxyz_g)
    m.close()
    gg.finalize_global_grid()
    return out


@pytest.mark.parametrize("K,nt", [(16, 37), (12, 29), (8, 21), (4, 13), (2, 9)])
def test_fast_math_decomposition_invariant_and_close(K, nt):
    """fast_math: 4 ranks (2x2) == 1 rank on the same global grid, bitwise
    (same fast-math expression everywhere), and within 1e-13 of the
    canonical arithmetic (canonical K-step passes go up to K=8; one rank's
    global grid does not depend on the overlap)."""
    nx, ny = 300, 134
    res = run_loopback(4, spmd_fast, nx, ny, nt, (2, 2), K, True, timeout=120)
    nxg, nyg, _ = res[0][2]
    one = run_loopback(1, spmd_fast, nxg, nyg, nt, (1, 1), K, True, timeout=120)[0][1]
    can = run_loopback(1, spmd_fast, nxg, nyg, nt, (1, 1), min(K, 8), False,
                       timeout=120)[0][1]
    for coords, T, _ in res:
        gx0, gy0 = coords[0] * (nx - 2 * K), coords[1] * (ny - 2 * K)
        assert np.array_equal(T, one[gy0:gy0 + ny, gx0:gx0 + nx])
    np.testing.assert_allclose(one, can, rtol=1e-13, atol=1e-13)
    assert not np.array_equal(one, can)  # it really is the other arithmetic


def spmd_planned(rank, hub, nx, ny, steps, dims, K, fast, timing=False):
    """A run split into several step() calls so the planner mixes pass depths
    (e.g. 5 + 20 + 13 steps with at most K per pass); returns (coords, field,
    global sizes, plans, per-pass timings)."""
    gg.init_global_grid(nx, ny, 1, dimx=dims[0], dimy=dims[1], overlaps=(2 * K, 2 * K, 2),
                        halowidths=(K, K, 1), quiet=True, loopback=(hub, rank))
    m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=nx, ny=ny, nt=sum(steps),
                                    init="random", quiet=True, dims=dims, temporal=K,
                                    fast_math=fast))
    assert m.executor is not None
    plans, ts = [], []
    if timing:
        m.enable_pass_timing(True)
    for s in steps:
        plans.append(m.plan(s))
        m.step(s)
    if timing:
        ts = m.pass_timings()
        m.enable_pass_timing(False)
    out = (m.g.coords, m.field.cpu().numpy().copy(), m.g.nxyz_g, plans, ts)
    m.close()
    gg.finalize_global_grid()
    return out


@pytest.mark.parametrize("fast", [True, False])
@pytest.mark.parametrize("K,steps", [(24, (5, 20, 13)), (16, (1, 17, 3)), (7, (9, 2, 11))])
def test_planned_mixed_depth_passes_decomposition_invariant(fast, K, steps):
    """The executor's planner runs passes of several depths (<= K) between
    width-K exchanges (the bench's warmup [5] + timed [20] shape): 4 loopback
    ranks (2x2, frames on the high-priority stream) == 1 rank of the global
    grid, bitwise, for both arithmetics."""
    nx = ny = 6 * K + 40
    res = run_loopback(4, spmd_planned, nx, ny, steps, (2, 2), K, fast, timeout=180)
    nxg, nyg, _ = res[0][2]
    assert [sum(p) for p in res[0][3]] == list(steps)
    assert any(len(set(p)) > 1 or p[0] != K for p in res[0][3])  # really mixed depths
    one = run_loopback(1, spmd_planned, nxg, nyg, steps, (1, 1), K, fast, timeout=180)[0][1]
    for coords, T, _, _, _ in res:
        gx0, gy0 = coords[0] * (nx - 2 * K), coords[1] * (ny - 2 * K)
        assert np.array_equal(T, one[gy0:gy0 + ny, gx0:gx0 + nx])


def test_pass_timing_and_solo_on_loopback_ranks():
    """bench.py's instrumentation on the native multi-rank path: per-pass
    HIP-event timings show a frame and an exchange for ranks with neighbours;
    solo mode (exchange off, one launch per pass) keeps the run going and
    restores the neighbours afterwards (a later run == a fresh one)."""
    K, nx, ny = 16, 300, 260

    def body(rank, hub):
        gg.init_global_grid(nx, ny, 1, dimx=2, dimy=1, overlaps=(2 * K, 2 * K, 2),
                            halowidths=(K, K, 1), quiet=True, loopback=(hub, rank))
        m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=nx, ny=ny, nt=60, init="random",
                                        quiet=True, dims=(2, 1, 0), temporal=K, fast_math=True))
        m.enable_pass_timing(True)
        m.step(20)
        ts = m.pass_timings()
        m.enable_pass_timing(False)
        m.set_solo(True)
        m.step(20)
        assert m.executor.solo
        m.set_solo(False)
        assert not m.executor.solo
        out = (ts, m.executor.plan(20))
        m.close()
        gg.finalize_global_grid()
        return out

    res = run_loopback(2, body, timeout=120)
    for ts, plan in res:
        assert [t["K"] for t in ts] == plan and sum(plan) == 20  # the plan of this tile class
        t = ts[0]
        assert t["frame_ms"] > 0 and t["halo_ms"] > 0 and t["interior_ms"] > 0
        assert t["pass_ms"] >= t["interior_ms"] and t["exposed_halo_ms"] >= 0


def test_p2p_smoke_test_through_rccl_on_one_gpu(capsys):
    """rocmaware_test_selectdevice.jl's ring on device buffers, one rank: the
    4-element buffer goes out and back through RCCL send/recv (to itself)."""
    from rocm_mpi_amd.apps import rocmaware_test_selectdevice as app

    vals = app.run(4, transport="rccl", verbose=True, self_ring=True)
    assert vals == [0.0] * 4
    out = capsys.readouterr().out
    assert "transport=rccl" in out and "recv_mesg on proc 0: [0.0, 0.0, 0.0, 0.0]" in out


def spmd_aligned(rank, hub, nx, ny, nt, dims, K, fast):
    """One rank of an open (non-periodic) grid: its pass geometry at depth K
    and its field after nt steps; also the halo plan cache counters."""
    gg.init_global_grid(nx, ny, 1, dimx=dims[0], dimy=dims[1], overlaps=(2 * K, 2 * K, 2),
                        halowidths=(K, K, 1), quiet=True, loopback=(hub, rank))
    m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=nx, ny=ny, nt=nt, init="random",
                                    quiet=True, dims=dims, temporal=K, fast_math=fast))
    geo = m.executor.geometry(K)
    plan = m.plan(nt)
    m.step(nt)
    halo = m.g.halo
    out = (m.g.coords, m.field.cpu().numpy().copy(), m.g.nxyz_g, geo, plan,
           halo.plan_hits, halo.plan_misses)
    m.close()
    gg.finalize_global_grid()
    return out


@pytest.mark.parametrize("dims", [(2, 1), (1, 2), (2, 2)])
@pytest.mark.parametrize("K,fast,nt", [(24, True, 53), (12, False, 29)])
def test_aligned_frames_on_partial_sides_bitwise(dims, K, fast, nt):
    """tiles big enough for the aligned frame layout
    (frame = whole tasks of the interior's grid) on ranks with neighbours on
    only one to three sides: every tile == its window of a 1-rank run of the
    global grid, bitwise; the deepest passes really are aligned. The halo plan
    is built once per field (T, T2) and served from the cache afterwards."""
    nx = ny = 1100
    P = dims[0] * dims[1]
    res = run_loopback(P, spmd_aligned, nx, ny, nt, dims, K, fast, timeout=180)
    nxg, nyg, _ = res[0][2]
    one = run_loopback(1, spmd_aligned, nxg, nyg, nt, (1, 1), K, fast, timeout=180)[0][1]
    for coords, T, _, geo, plan, hits, misses in res:
        assert geo["aligned"], (coords, geo)
        assert len(geo["frame"]) == len(geo["frame_wide"]) + len(geo["frame_tall"]) >= 1
        gx0, gy0 = coords[0] * (nx - 2 * K), coords[1] * (ny - 2 * K)
        assert np.array_equal(T, one[gy0:gy0 + ny, gx0:gx0 + nx]), coords
        assert misses <= 2 and hits + misses == len(plan)


def spmd_bands(rank, hub, nx, ny, nt, dims, K, chunk2):
    gg.init_global_grid(nx, ny, 1, dimx=dims[0], dimy=dims[1], overlaps=(2 * K, 2 * K, 2),
                        halowidths=(K, K, 1), quiet=True, loopback=(hub, rank))
    m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=nx, ny=ny, nt=nt, init="random",
                                    quiet=True, dims=dims, temporal=K, fast_math=True,
                                    chunk2=chunk2))
    geo = m.executor.geometry(K)
    m.step(nt)
    out = (m.g.coords, m.field.cpu().numpy().copy(), m.g.nxyz_g, geo)
    m.close()
    gg.finalize_global_grid()
    return out


@pytest.mark.parametrize("dims", [(1, 2), (2, 2)])
def test_aligned_frames_with_ol_bands_bitwise(dims):
    """Tasks taller than 1024 rows (the 288 GB tile's 3072): the tall frames
    are whole strip columns of the interior's grid, the bands only the ol-K
    rows the exchange needs; every tile == the 1-rank run, bitwise."""
    K, nx, ny, nt = 8, 800, 2600, 19  # 800 >= 3 strip columns of 240 + 2K
    res = run_loopback(dims[0] * dims[1], spmd_bands, nx, ny, nt, dims, K, 1100, timeout=180)
    nxg, nyg, _ = res[0][2]
    one = run_loopback(1, spmd_bands, nxg, nyg, nt, (1, 1), K, 1100, timeout=180)[0][1]
    for coords, T, _, geo in res:
        assert geo["aligned"], (coords, geo)
        for r in geo["frame_wide"]:
            assert r[3] - r[2] < 2 * K  # the rows the exchange needs, not a 1100-row task row
        gx0, gy0 = coords[0] * (nx - 2 * K), coords[1] * (ny - 2 * K)
        assert np.array_equal(T, one[gy0:gy0 + ny, gx0:gx0 + nx]), coords


def test_halo_plan_cache_hits_evicts_and_stays_correct():
    """HaloExchanger caches the plan + resolved copy batches per field
    geometry: alternating T/T2 exchanges hit after the
    first of each; a field needing larger pack buffers reallocates them and
    drops the cache (stale pointers), and an LRU of 4 entries bounds it. Every
    exchange (x periodic through RCCL send/recv to self: strided planes are
    packed) leaves the halo columns equal to the periodic copies."""
    from rocm_mpi_amd._native import native
    from rocm_mpi_amd.parallel import comm as C

    n = native()
    rc = C.RcclComm(torch.device("cuda", torch.cuda.current_device()))
    halo = n.HaloExchanger(rc.native, 0, [[0, 0], [-1, -1], [-1, -1]])
    halo.set_self_via_transport(True)
    s = torch.cuda.current_stream().cuda_stream

    def field(ny, nx, seed):
        g = torch.Generator(device="cpu").manual_seed(seed)
        return torch.rand(ny, nx, generator=g, dtype=torch.float64).cuda()

    def check(T, hw, ol):
        ref = T.clone()
        nx = T.shape[1]
        ref[:, :hw] = T[:, nx - ol:nx - ol + hw]
        ref[:, nx - hw:] = T[:, ol - hw:ol]
        return ref

    def run(T, hw=1, ol=2):
        ref = check(T, hw, ol)
        halo.exchange([(T.data_ptr(), (T.shape[1], T.shape[0], 1), 8, (ol, ol, 2), (hw, hw, 1))],
                      s, 1)
        torch.cuda.synchronize()
        assert torch.equal(T, ref)

    A, B = field(40, 64, 1), field(40, 64, 2)
    for T in (A, B, A, B, A):
        run(T)
    assert (halo.plan_misses, halo.plan_hits) == (2, 3)
    Cbig = field(40, 64, 3)
    run(Cbig, hw=3, ol=6)  # larger pack buffers: reallocated, cache dropped
    run(A)
    assert halo.plan_misses == 4
    fs = [field(40, 64, 10 + i) for i in range(5)]
    m0 = halo.plan_misses
    for _ in range(2):
        for T in fs:  # 5 fields cycling through a 4-entry LRU: every one misses
            run(T)
    assert halo.plan_misses - m0 == 10
    rc.finalize()


@pytest.mark.parametrize("K,gs,nt", [(8, 10, 43), (8, 8, 43), (6, 10, 43), (4, 10, 43), (8, 20, 61)])
@pytest.mark.parametrize("fast", [False, True])
def test_graph_replay_matches_eager_periodic(K, gs, nt, fast):
    """hipGraph replay of planned mixed-depth passes (a captured plan of gs
    steps replayed, the remainder eager) == the eager run, on a periodic
    single-rank tile (local periodic copies: capturable)."""
    def run(graph):
        gg.init_global_grid(514, 300, 1, periodx=1, periody=1, overlaps=(2 * K, 2 * K, 2),
                            halowidths=(K, K, 1), quiet=True)
        m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=514, ny=300, nt=nt,
                                        init="random", quiet=True, periods=(1, 1, 0),
                                        temporal=K, fast_math=fast, use_graph=graph,
                                        graph_steps=gs))
        m.step(nt)
        f = m.field.cpu().clone()
        m.close()
        gg.finalize_global_grid()
        return f
    assert torch.equal(run(True), run(False))


@pytest.mark.parametrize("dims,ny", [((2, 2), 3500), ((1, 2), 3500), ((2, 1), 3500),
                                     ((1, 2), 7000)])
def test_small_tile_frame_layouts_bitwise(dims, ny):
    """The per-tile frame layout (plan.cpp frame_layout):
    4096-class tiles run half-height frame tasks (ol-K bands with x AND y
    neighbours), 8192-class tiles with y neighbours half-height frame tasks;
    every tile == its window of the 1-rank run, bitwise."""
    from rocm_mpi_amd._native import native

    K, nx, nt = 24, 1100, 53
    P = dims[0] * dims[1]
    res = run_loopback(P, spmd_bands, nx, ny, nt, dims, K, 0, timeout=240)
    nxg, nyg, _ = res[0][2]
    one = run_loopback(1, spmd_bands, nxg, nyg, nt, (1, 1), K, 0, timeout=240)[0][1]
    for coords, T, _, geo in res:
        nb = [[-1, -1], [-1, -1], [-1, -1]]
        for d in (0, 1):
            if dims[d] > 1:
                nb[d] = [0 if coords[d] > 0 else -1, 0 if coords[d] < dims[d] - 1 else -1]
        div, bands = native().frame_layout(ny, nb)
        xy = dims[0] > 1 and dims[1] > 1
        if ny < 6144:
            assert div == 2 and bands == (0 if xy else -1)
        else:  # 8192 class, y neighbours only: ol-K bands, whole-task rows per frame task
            assert (div, bands) == (1, 0)
        assert geo["aligned"], (coords, geo)
        if bands == 0:
            for r in geo["frame_wide"]:
                assert r[3] - r[2] < 2 * K
        gx0, gy0 = coords[0] * (nx - 2 * K), coords[1] * (ny - 2 * K)
        assert np.array_equal(T, one[gy0:gy0 + ny, gx0:gx0 + nx]), coords


def spmd_fused(rank, hub, nx, ny, nt, dims, K, graph=False):
    gg.init_global_grid(nx, ny, 1, dimx=dims[0], dimy=dims[1], overlaps=(2 * K, 2 * K, 2),
                        halowidths=(K, K, 1), quiet=True, loopback=(hub, rank))
    m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=nx, ny=ny, nt=nt, init="random",
                                    quiet=True, dims=dims, temporal=K, fast_math=True,
                                    use_graph=graph))
    plan = list(m.executor.plan(nt))
    geos = {k: m.executor.geometry(k) for k in set(plan)}
    # the passes the executor fuses: aligned frames (whole tasks of the pass's
    # grid) around a non-empty interior
    def fusable(g):
        x0, x1, y0, y1 = g["interior"]
        return g["aligned"] and x1 > x0 and y1 > y0 and any(r[1] > r[0] and r[3] > r[2]
                                                            for r in g["frame"])
    want = sum(1 for k in plan if fusable(geos[k]))
    m.step(nt)
    out = (m.g.coords, m.field.cpu().numpy().copy(), m.g.nxyz_g,
           (m.executor.fused_passes, want, plan, geos))
    m.close()
    gg.finalize_global_grid()
    return out


@pytest.mark.parametrize("dims,K,nx,ny,nt,some", [((2, 2), 24, 1100, 3500, 53, True),
                                                  ((2, 1), 20, 1100, 1500, 47, True),
                                                  ((1, 2), 8, 800, 2600, 19, True),
                                                  ((2, 2), 16, 700, 900, 37, False),
                                                  ((2, 2), 12, 1000, 3000, 31, True)])
def test_fused_frame_first_passes_bitwise(dims, K, nx, ny, nt, some, monkeypatch):
    """RMA_EXEC_FUSED=1: every K-step pass with a neighbour is ONE pipelined
    launch, frame tasks first, whose last frame block raises the flag the
    exchange stream waits on (flags.hip); every tile == its window of the
    1-rank run, bitwise, and the passes with aligned frames (whole tasks of
    the pass's grid) really ran fused -- the others (all of them in the
    700x900 case: tiles too small for aligned frames) keep the split launches."""
    monkeypatch.setenv("RMA_EXEC_FUSED", "1")
    P = dims[0] * dims[1]
    res = run_loopback(P, spmd_fused, nx, ny, nt, dims, K, timeout=240)
    nxg, nyg, _ = res[0][2]
    monkeypatch.setenv("RMA_EXEC_FUSED", "0")
    one = run_loopback(1, spmd_fused, nxg, nyg, nt, (1, 1), K, timeout=240)[0][1]
    assert any(w for _, _, _, (_, w, _, _) in res) == some
    for coords, T, _, (fused, want, plan, geos) in res:
        assert fused == want, (coords, fused, want, plan, geos)
        gx0, gy0 = coords[0] * (nx - 2 * K), coords[1] * (ny - 2 * K)
        assert np.array_equal(T, one[gy0:gy0 + ny, gx0:gx0 + nx]), coords


@pytest.mark.parametrize("graph", [False, True])
def test_fused_passes_over_rccl_self_equal_the_split_passes(graph, monkeypatch):
    """Fused passes behind the production exchange (RCCL send/recv to self, x
    and y periodic, merged groups) eagerly, and replayed from a hipGraph (the
    flag kernels are captured nodes; the periodic halos then go through local
    copies, since RCCL is not captured in a torch process), leave the field
    bitwise equal to the split frame / interior passes."""
    K, n, nt = 24, 1536, 240

    def run(fused):
        monkeypatch.setenv("RMA_EXEC_FUSED", "1" if fused else "0")
        gg.init_global_grid(n, n, 1, periodx=1, periody=1, quiet=True, transport="rccl",
                            overlaps=(2 * K, 2 * K, 2), halowidths=(K, K, 1),
                            self_via_transport=not graph)
        m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=n, ny=n, nt=nt, init="random",
                                        quiet=True, periods=(1, 1, 0), temporal=K,
                                        fast_math=True, use_graph=graph and fused))
        assert m.use_graph == (graph and fused)
        m.step(nt)
        f = m.field.cpu().numpy().copy()
        nf = m.executor.fused_passes
        m.close()
        gg.finalize_global_grid()
        return f, nf

    a, nfa = run(True)
    b, nfb = run(False)
    assert nfb == 0 and nfa >= 2, nfa  # (graph: counted once per captured pass)
    assert np.array_equal(a, b)


def test_fused_pass_wait_timeout_is_reported_not_hung(monkeypatch):
    """The exchange stream's wait for the frame flag is bounded: with a
    timeout far below a frame's run time every wait gives up, the passes still
    drain (no hang; halos of those passes are wrong) and synchronize() and
    the next run() raise the timeout instead of returning silently."""
    K, n = 24, 1536
    monkeypatch.setenv("RMA_EXEC_FUSED", "1")
    monkeypatch.setenv("RMA_EXEC_FUSED_TIMEOUT", "1e-7")
    gg.init_global_grid(n, n, 1, periodx=1, periody=1, quiet=True, transport="rccl",
                        overlaps=(2 * K, 2 * K, 2), halowidths=(K, K, 1), self_via_transport=True)
    m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=n, ny=n, nt=48, init="random",
                                    quiet=True, periods=(1, 1, 0), temporal=K, fast_math=True))
    try:
        m.step(48)
        with pytest.raises(RuntimeError, match="timed out"):  # the native module's NativeError
            m.synchronize()
        assert m.executor.fused_passes == 2
        with pytest.raises(RuntimeError, match="timed out"):
            m.step(K)
    finally:
        with pytest.raises(RuntimeError, match="timed out"):  # and close() still releases
            m.close()
        assert m.executor is None
        gg.finalize_global_grid()


@pytest.mark.parametrize("via_rccl", [False, True])
@pytest.mark.parametrize("hw,ol", [(1, 2), (8, 16), (24, 48)])
def test_merged_exchange_equals_dimension_ordered(via_rccl, hw, ol):
    """HaloExchanger.exchange_merged (x and y in ONE group, the corner blocks
    sent to the diagonal neighbours -- all of them this rank on a periodic
    single-rank tile; through RCCL send/recv to itself or local copies) leaves
    the field bitwise equal to the dimension-ordered exchange, corners
    included."""
    from rocm_mpi_amd._native import native
    from rocm_mpi_amd.parallel import comm as C

    n = native()
    rc = C.RcclComm(torch.device("cuda", torch.cuda.current_device())) if via_rccl else None
    nb = [[0, 0], [0, 0], [-1, -1]]
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cpu").manual_seed(hw)
    A = torch.rand(203, 331, generator=g, dtype=torch.float64).cuda()
    B = A.clone()
    f = lambda T: [(T.data_ptr(), [331, 203, 1], 8, [ol, ol, 2], [hw, hw, 1])]  # noqa: E731
    h1 = n.HaloExchanger(rc.native if rc else None, 0, nb)
    h2 = n.HaloExchanger(rc.native if rc else None, 0, nb)
    for h in (h1, h2):
        if via_rccl:
            h.set_self_via_transport(True)
        h.set_diagonals([0, 0, 0, 0])
    h1.exchange(f(A), s, 3)
    h2.exchange_merged(f(B), s)
    torch.cuda.synchronize()
    assert torch.equal(A, B)
    assert not torch.equal(A, torch.rand(203, 331, generator=torch.Generator().manual_seed(hw),
                                         dtype=torch.float64).cuda())  # the halos did change
    if rc:
        rc.finalize()


def _user_example():
    import importlib.util
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location(
        "diffusion_2D_user", os.path.join(root, "examples", "diffusion_2D_user.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def spmd_user_example(rank, hub, nx, ny, nt, dims, hide):
    T0, T, _ = _user_example().diffusion2D(nx, ny, nt, device="cuda", dims=dims, hide=hide,
                                           quiet=True, b_width=(8, 4),
                                           grid_kw=dict(loopback=(hub, rank)))
    return None if T is None else T.numpy()


@pytest.mark.parametrize("hide", [False, True])
@pytest.mark.parametrize("P,dims", [(1, (1, 1)), (4, (2, 2))])
def test_user_example_gpu_equals_golden(hide, P, dims):
    """examples/diffusion_2D_user.py on cuda:0 (--hide: frame and update_halo_
    on a high-priority stream, interior on a low-priority one; 2x2 loopback
    ranks: the merged x+y exchange) == the golden model, bitwise."""
    nx, ny, nt = 300, 134, 23
    T = run_loopback(P, spmd_user_example, nx, ny, nt, dims, hide, timeout=120)[0]
    nxg, nyg = dims[0] * (nx - 2) + 2, dims[1] * (ny - 2) + 2
    G0 = golden.initial_torch(nxg, nyg)
    assert np.array_equal(T, golden.run(nxg, nyg, nt, T0=G0)[1:-1, 1:-1])


@pytest.mark.parametrize("variant,world,dims", [("perf_hide", 2, (2, 1)), ("perf", 4, (2, 2)),
                                                ("kp", 2, (1, 2)), ("perf_hide", 4, (4, 1))])
def test_ipc_transport_processes(tmp_path, variant, world, dims):
    """transport="ipc": separate processes sharing cuda:0 move every halo
    device-to-device through HIP IPC mailboxes (no RCCL, no host staging);
    the gathered field == the golden model, bitwise (2x2: the merged x+y group
    with corner blocks to the diagonal ranks)."""
    run_procs(world, "mp_targets:diffusion_gpu", str(tmp_path), variant, 130, 66, 25, dims,
              env={"RMA_TRANSPORT": "ipc", "RMA_IPC_MAILBOX_MB": "1"})
    Tv = np.load(tmp_path / "Tv.npy")
    nxg, nyg, transport = open(tmp_path / "meta.txt").read().split()[:3]
    assert transport == "ipc"
    assert np.array_equal(Tv, golden.run(int(nxg), int(nyg), 25)[1:-1, 1:-1])


@pytest.mark.parametrize("K", [4, 8])
def test_ipc_transport_temporal_tiles(tmp_path, K):
    """K-step passes (width-K halos, one exchange per pass, frame on the
    high-priority stream) over the IPC transport, 2x2 processes: every tile ==
    the golden model's window, bitwise."""
    from rocm_mpi_amd import ops

    nx, ny, nt = 120, 90, 3 * K + 1
    run_procs(4, "mp_targets:diffusion_tiles", str(tmp_path), "perf_hide", nx, ny, nt, (2, 2), K,
              "cuda:0", env={"RMA_TRANSPORT": "ipc"})
    metas = [open(tmp_path / f"meta{r}.txt").read().split() for r in range(4)]
    nxg, nyg = int(metas[0][2]), int(metas[0][3])
    assert metas[0][6] == "ipc"
    T0 = torch.empty((nyg, nxg), dtype=torch.float64)
    ops.init_random_(T0, ops.TileGeometry(0, 0, nxg, nyg, 1.0, 1.0), seed=1234)
    G = golden.run(nxg, nyg, nt, T0=T0.numpy())
    for r in range(4):
        cx, cy, ol = int(metas[r][0]), int(metas[r][1]), int(metas[r][4])
        T = np.load(tmp_path / f"tile{r}.npy")
        gx0, gy0 = cx * (nx - ol), cy * (ny - ol)
        assert np.array_equal(T, G[gy0:gy0 + ny, gx0:gx0 + nx])


@pytest.mark.parametrize("world", [2, 4])
def test_ipc_ring_smoke_test(tmp_path, world):
    """The reference's rocmaware_test_selectdevice ring (4 doubles per rank on
    the device, sent to rank+1) over HIP IPC between processes on cuda:0."""
    run_procs(world, "mp_targets:ring_gpu", str(tmp_path), "ipc")
    for r in range(world):
        assert np.load(tmp_path / f"ring{r}.npy").tolist() == [float((r - 1) % world)] * 4


def test_ipc_mailbox_overflow_fails_on_every_rank(tmp_path):
    """RMA_IPC_MAILBOX_MB too small for a halo plane: every rank raises an
    error naming the setting (no rank waits for a peer that gave up)."""
    run_procs(2, "mp_targets:ipc_overflow", str(tmp_path),
              env={"RMA_TRANSPORT": "ipc", "RMA_IPC_MAILBOX_MB": "0.0001"})
    for r in range(2):
        assert "RMA_IPC_MAILBOX_MB" in open(tmp_path / f"err{r}.txt").read()


@pytest.mark.parametrize("mode", ["stream", "host"])
def test_ipc_overflow_of_a_later_peer_keeps_the_transport_in_step(tmp_path, mode):
    """the mailbox check covers every peer of a group before any
    copy or flag; after the error the next exchanges are correct."""
    run_procs(3, "mp_targets:ipc_overflow_then_ring", str(tmp_path),
              env={"RMA_TRANSPORT": "ipc", "RMA_IPC_MAILBOX_MB": "0.001", "RMA_IPC_MODE": mode})
    for r in range(3):
        assert open(tmp_path / f"ok{r}.txt").read() == "1"


@pytest.mark.parametrize("case", [
    ((9, 7, 1), (2, 2, 1), (0, 0, 0), (2, 2, 2), [(0, 0, 0), (1, 0, 0), (0, 1, 0), (-1, 0, 0)], 4),
    ((12, 10, 1), (2, 2, 1), (1, 1, 0), (4, 4, 2), [(0, 0, 0)], 2),
    ((6, 5, 7), (2, 2, 2), (0, 0, 0), (2, 2, 2), [(0, 0, 0), (0, 0, 1)], 2),
], ids=["2d-staggered", "2d-periodic-hw2", "3d"])
def test_ipc_update_halo_device_fields(tmp_path, case):
    """update_halo_ of device fields between PROCESSES over the IPC transport
    (merged x+y group for the 2-D fields, per-dimension groups in 3-D)."""
    nxyz, dims, periods, overlaps, staggers, nf = case
    world = dims[0] * dims[1] * dims[2]
    run_procs(world, "mp_targets:halo_device", str(tmp_path), nxyz, dims, periods, overlaps,
              staggers, nf, env={"RMA_TRANSPORT": "ipc", "RMA_IPC_MAILBOX_MB": "1"})
    for r in range(world):
        assert open(tmp_path / f"ok{r}.txt").read() == "1 ipc"


def _ipc_probe(*args, env=None, timeout=300):
    import json
    import os
    import subprocess
    import sys

    from helpers import ROOT, free_port

    e = dict(os.environ, MASTER_PORT=str(free_port()), **(env or {}))
    r = subprocess.run([sys.executable, "-m", "rocm_mpi_amd.launch", "-n", "4", "--",
                        os.path.join(ROOT, "bench", "ipc_transport_probe.py"), *args],
                       capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=e)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    # the launcher prefixes every line with the rank ("[0] {...}")
    lines = [ln.split("] ", 1)[1] for ln in r.stdout.splitlines()
             if ln.startswith("[0] {")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("mode", ["stream", "host"])
def test_ipc_modes_2000_exchanged_steps_bitwise(mode):
    """2000 one-step perf_hide steps of a 2x2 process grid
    (an exchange every step) over IPC == the golden model bitwise; the stream
    mode (the default) waits on the host zero times inside group_end, the host
    mode twice per peer and group."""
    d = _ipc_probe("--transport", "ipc", "--n", "258", "--K", "1", "--steps", "2000", "--check",
                   env={"RMA_IPC_MODE": mode})
    assert d["bitwise_golden"] is True and d["transport"] == "ipc" and d["ipc_mode"] == mode
    if mode == "stream":
        assert d["host_waits_in_group_end"] == 0
    else:
        assert d["host_waits_in_group_end"] > 2000


def test_ipc_stream_mode_graph_replay_matches_golden():
    """the executor's hipGraph replay with the IPC exchange
    captured in it (stream mode: copies plus the bounded flag kernels of
    csrc/kernels/flags.hip, no host handshake) == the golden model bitwise,
    like the eager run. (HIP's own hipStreamWaitValue64 / WriteValue64
    replayed to a wrong field once captured:
    profiles/r5/ipc_graph_replay_failure.log.)"""
    d = _ipc_probe("--transport", "ipc", "--n", "258", "--K", "1", "--steps", "100", "--check",
                   "--graph", env={"RMA_IPC_MODE": "stream"})
    assert d["graph"] is True and d["bitwise_golden"] is True
    assert d["host_waits_in_group_end"] == 0


RCCL_SHARED = {"RMA_TRANSPORT": "rccl", "RMA_RCCL_SHARED_GPU": "1"}


@pytest.mark.parametrize("variant,world,dims", [("perf_hide", 2, (2, 1)), ("perf", 4, (2, 2)),
                                                ("kp", 2, (1, 2)), ("perf_hide", 4, (4, 1))])
def test_rccl_between_processes_sharing_the_gpu(tmp_path, variant, world, dims):
    """The production RCCL halo path between SEPARATE processes (multi-rank
    communicator from the store's unique id, grouped send/recv between distinct
    ranks, merged x+y groups with diagonal corners on 2x2): every process on
    cuda:0, RCCL told that each rank is its own host (RMA_RCCL_SHARED_GPU ->
    NCCL_HOSTID), so it moves the halos over its socket transport instead of
    refusing the duplicate GPU. Gathered field == the golden model, bitwise."""
    run_procs(world, "mp_targets:diffusion_gpu", str(tmp_path), variant, 130, 66, 25, dims,
              env=RCCL_SHARED)
    Tv = np.load(tmp_path / "Tv.npy")
    nxg, nyg, transport = open(tmp_path / "meta.txt").read().split()[:3]
    assert transport == "rccl"
    assert np.array_equal(Tv, golden.run(int(nxg), int(nyg), 25)[1:-1, 1:-1])


def test_rccl_between_processes_temporal_tiles(tmp_path):
    """K-step passes (width-K halos, frame + RCCL exchange on the high-priority
    stream, interior beside it) between 4 processes over multi-rank RCCL."""
    from rocm_mpi_amd import ops

    K, nx, ny = 8, 120, 90
    nt = 3 * K + 1
    run_procs(4, "mp_targets:diffusion_tiles", str(tmp_path), "perf_hide", nx, ny, nt, (2, 2), K,
              "cuda:0", env=RCCL_SHARED)
    metas = [open(tmp_path / f"meta{r}.txt").read().split() for r in range(4)]
    nxg, nyg = int(metas[0][2]), int(metas[0][3])
    assert metas[0][6] == "rccl"
    T0 = torch.empty((nyg, nxg), dtype=torch.float64)
    ops.init_random_(T0, ops.TileGeometry(0, 0, nxg, nyg, 1.0, 1.0), seed=1234)
    G = golden.run(nxg, nyg, nt, T0=T0.numpy())
    for r in range(4):
        cx, cy, ol = int(metas[r][0]), int(metas[r][1]), int(metas[r][4])
        T = np.load(tmp_path / f"tile{r}.npy")
        gx0, gy0 = cx * (nx - ol), cy * (ny - ol)
        assert np.array_equal(T, G[gy0:gy0 + ny, gx0:gx0 + nx])


def test_rccl_ring_smoke_test_between_processes(tmp_path):
    """The reference smoke test's device-buffer ring (rocmaware_test_selectdevice.jl)
    over a 4-rank RCCL communicator of separate processes."""
    run_procs(4, "mp_targets:ring_gpu", str(tmp_path), "rccl", env=RCCL_SHARED)
    for r in range(4):
        assert np.load(tmp_path / f"ring{r}.npy").tolist() == [float((r - 1) % 4)] * 4
