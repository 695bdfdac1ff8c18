"""The C ABI (csrc/include/rma/capi.h) on the GPU, driven through ctypes the way
a C/Julia host would: grid, device init, executor with 1 and 8 steps per pass,
update_halo, gather, timers — checked against the Python model / golden."""
import ctypes
import os

import numpy as np
import pytest
import torch

import golden
from helpers import ROOT

pytestmark = pytest.mark.gpu

c_int_p = ctypes.POINTER(ctypes.c_int)


def lib():
    L = ctypes.CDLL(os.path.join(ROOT, "rocm_mpi_amd", "librma_core.so"))
    L.rma_last_error.restype = ctypes.c_char_p
    L.rma_nx_g.restype = ctypes.c_int64
    L.rma_ny_g.restype = ctypes.c_int64
    return L


def ck(L, rc):
    assert rc == 0, L.rma_last_error().decode()


def grid(L, nx, ny, K=1, periods=(0, 0, 0)):
    g = ctypes.c_void_p()
    me = ctypes.c_int()
    dims = (ctypes.c_int * 3)()
    coords = (ctypes.c_int * 3)()
    ol = (ctypes.c_int * 3)(2 * K, 2 * K, 2)
    hw = (ctypes.c_int * 3)(K, K, 1)
    per = (ctypes.c_int * 3)(*periods)
    ck(L, L.rma_init_global_grid(nx, ny, 1, None, per, ol, hw, 1, 0, None, 0, ctypes.byref(g),
                                 ctypes.byref(me), dims, coords))
    return g


def coef4(L, g, nx, ny):
    dx, dy = 10.0 / L.rma_nx_g(g), 10.0 / L.rma_ny_g(g)
    dt = min(dx * dx, dy * dy) / 4.1
    return (ctypes.c_double * 4)(-1.0, 1 / dx, 1 / dy, dt)


@pytest.mark.parametrize("mode,K", [(0, 1), (1, 1), (1, 8), (0, 6)])
def test_capi_executor_matches_model(mode, K):
    L = lib()
    nx, ny, nt = 514, 300, 37
    g = grid(L, nx, ny, K)
    s = torch.cuda.current_stream().cuda_stream
    T = torch.empty((ny, nx), dtype=torch.float64, device="cuda")
    T2 = torch.empty_like(T)
    iCp = torch.empty_like(T)
    ck(L, L.rma_fill(ctypes.c_void_p(iCp.data_ptr()), ctypes.c_int64(nx * ny),
                     ctypes.c_double(1.0), ctypes.c_void_p(s)))
    dx, dy = 10.0 / L.rma_nx_g(g), 10.0 / L.rma_ny_g(g)
    ck(L, L.rma_init_gaussian(g, ctypes.c_void_p(T.data_ptr()), ctypes.c_int64(nx),
                              ctypes.c_int64(ny), ctypes.c_double(dx), ctypes.c_double(dy),
                              ctypes.c_double(10.0), ctypes.c_double(10.0), ctypes.c_void_p(s)))
    G0 = golden.initial(nx, ny)  # device exp() may differ from NumPy's by an ulp
    np.testing.assert_allclose(T.cpu().numpy(), G0, rtol=4e-16, atol=1e-300)
    T.copy_(torch.from_numpy(G0))
    T2.copy_(T)
    ex = ctypes.c_void_p()
    ck(L, L.rma_executor_create_k(g, mode, ctypes.c_void_p(T.data_ptr()),
                                  ctypes.c_void_p(T2.data_ptr()), ctypes.c_void_p(iCp.data_ptr()),
                                  ctypes.c_int64(nx), ctypes.c_int64(ny), coef4(L, g, nx, ny),
                                  ctypes.c_int64(1), ctypes.c_int64(1), K, None, None, None,
                                  ctypes.byref(ex)))
    ck(L, L.rma_tic(g, ctypes.c_void_p(s)))
    ck(L, L.rma_executor_run(ex, ctypes.c_int64(nt), ctypes.c_void_p(s)))
    t = ctypes.c_double()
    ck(L, L.rma_toc(g, ctypes.c_void_p(s), ctypes.byref(t)))
    assert t.value > 0
    par = L.rma_executor_parity(ex)
    torch.cuda.synchronize()
    field = (T2 if par else T).cpu().numpy()
    ck(L, L.rma_executor_destroy(ex))
    ck(L, L.rma_finalize_global_grid(g))
    # single rank, open boundaries: the global problem is the local one
    G = golden.run(nx, ny, nt)
    assert np.array_equal(field, G)


@pytest.mark.parametrize("mode,K", [(1, 16), (0, 12)])
def test_capi_fast_math_executor_close(mode, K):
    """rma_executor_create_kf(fast_math=1): 12 / 16 steps per pass on the
    fast-math kernels, within rounding of the golden model."""
    L = lib()
    nx, ny, nt = 514, 300, 41
    g = grid(L, nx, ny, K)
    s = torch.cuda.current_stream().cuda_stream
    T = torch.from_numpy(golden.initial(nx, ny)).cuda()
    T2 = T.clone()
    iCp = torch.ones_like(T)
    ex = ctypes.c_void_p()
    ck(L, L.rma_executor_create_kf(g, mode, ctypes.c_void_p(T.data_ptr()),
                                   ctypes.c_void_p(T2.data_ptr()), ctypes.c_void_p(iCp.data_ptr()),
                                   ctypes.c_int64(nx), ctypes.c_int64(ny), coef4(L, g, nx, ny),
                                   ctypes.c_int64(1), ctypes.c_int64(1), K, 1, None, None, None,
                                   ctypes.byref(ex)))
    ck(L, L.rma_executor_run(ex, ctypes.c_int64(nt), ctypes.c_void_p(s)))
    par = L.rma_executor_parity(ex)
    torch.cuda.synchronize()
    field = (T2 if par else T).cpu().numpy()
    ck(L, L.rma_executor_destroy(ex))
    ck(L, L.rma_finalize_global_grid(g))
    np.testing.assert_allclose(field, golden.run(nx, ny, nt), rtol=1e-13, atol=1e-13)
    # without fast_math, 16 steps per pass run the canonical pipelined kernel:
    # bitwise equal to the golden model
    if K == 16:
        g = grid(L, nx, ny, K)
        T = torch.from_numpy(golden.initial(nx, ny)).cuda()
        T2 = T.clone()
        ck(L, L.rma_executor_create_kf(g, mode, ctypes.c_void_p(T.data_ptr()),
                                       ctypes.c_void_p(T2.data_ptr()),
                                       ctypes.c_void_p(iCp.data_ptr()), ctypes.c_int64(nx),
                                       ctypes.c_int64(ny), coef4(L, g, nx, ny), ctypes.c_int64(1),
                                       ctypes.c_int64(1), K, 0, None, None, None,
                                       ctypes.byref(ex)))
        ck(L, L.rma_executor_run(ex, ctypes.c_int64(nt), ctypes.c_void_p(s)))
        par = L.rma_executor_parity(ex)
        torch.cuda.synchronize()
        field = (T2 if par else T).cpu().numpy()
        ck(L, L.rma_executor_destroy(ex))
        assert np.array_equal(field, golden.run(nx, ny, nt))
        ck(L, L.rma_finalize_global_grid(g))


def test_capi_fused_passes_checked_and_bitwise(monkeypatch):
    """A periodic fast-math perf_hide executor through the C ABI: with
    RMA_EXEC_FUSED=1 its K=24 passes run as frame-first fused launches
    (rma_executor_check: no timed-out frame wait, the fused-pass count) and
    the field equals the split passes' bitwise."""
    L = lib()
    n, K, nt = 1536, 24, 72

    def run(fused):
        monkeypatch.setenv("RMA_EXEC_FUSED", "1" if fused else "0")
        g = grid(L, n, n, K, periods=(1, 1, 0))
        s = torch.cuda.current_stream().cuda_stream
        T = torch.from_numpy(golden.initial(n, n)).cuda()
        T2 = T.clone()
        iCp = torch.ones_like(T)
        ex = ctypes.c_void_p()
        ck(L, L.rma_executor_create_kf(g, 1, ctypes.c_void_p(T.data_ptr()),
                                       ctypes.c_void_p(T2.data_ptr()),
                                       ctypes.c_void_p(iCp.data_ptr()), ctypes.c_int64(n),
                                       ctypes.c_int64(n), coef4(L, g, n, n), ctypes.c_int64(1),
                                       ctypes.c_int64(1), K, 1, None, None, None,
                                       ctypes.byref(ex)))
        ck(L, L.rma_executor_run(ex, ctypes.c_int64(nt), ctypes.c_void_p(s)))
        par = L.rma_executor_parity(ex)
        torch.cuda.synchronize()
        nf = ctypes.c_int64(-1)
        ck(L, L.rma_executor_check(ex, ctypes.byref(nf)))
        field = (T2 if par else T).cpu().numpy()
        ck(L, L.rma_executor_destroy(ex))
        ck(L, L.rma_finalize_global_grid(g))
        return field, nf.value

    a, nfa = run(True)
    b, nfb = run(False)
    assert nfa == nt // K and nfb == 0
    assert np.array_equal(a, b)


def test_capi_update_halo_periodic_and_gather():
    L = lib()
    nx, ny = 130, 67
    g = grid(L, nx, ny, 1, periods=(1, 1, 0))
    s = torch.cuda.current_stream().cuda_stream
    A = torch.arange(nx * ny, dtype=torch.float64, device="cuda").view(ny, nx)
    ptrs = (ctypes.c_void_p * 1)(A.data_ptr())
    sizes = (ctypes.c_int64 * 3)(nx, ny, 1)
    eb = (ctypes.c_int * 1)(8)
    ck(L, L.rma_update_halo(g, 1, ptrs, sizes, eb, ctypes.c_void_p(s)))
    torch.cuda.synchronize()
    a = A.cpu()
    assert torch.equal(a[:, 0], a[:, nx - 2]) and torch.equal(a[:, nx - 1], a[:, 1])
    assert torch.equal(a[0, :], a[ny - 2, :]) and torch.equal(a[ny - 1, :], a[1, :])
    out = torch.empty_like(A)
    ck(L, L.rma_gather(g, ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                       ctypes.c_size_t(A.numel() * 8), 0, ctypes.c_void_p(s)))
    torch.cuda.synchronize()
    assert torch.equal(out, A)
    ck(L, L.rma_finalize_global_grid(g))


def test_capi_error_reporting():
    L = lib()
    g = grid(L, 64, 64, 1)
    ex = ctypes.c_void_p()
    T = torch.empty((64, 64), dtype=torch.float64, device="cuda")
    rc = L.rma_executor_create_k(g, 1, ctypes.c_void_p(T.data_ptr()),
                                 ctypes.c_void_p(T.data_ptr()), ctypes.c_void_p(T.data_ptr()),
                                 ctypes.c_int64(64), ctypes.c_int64(64),
                                 (ctypes.c_double * 4)(-1, 1, 1, 0.1), ctypes.c_int64(1),
                                 ctypes.c_int64(1), 25, None, None, None, ctypes.byref(ex))
    assert rc != 0 and b"temporal" in L.rma_last_error()
    ck(L, L.rma_finalize_global_grid(g))


@pytest.mark.parametrize("K,via_rccl", [(1, False), (8, False), (8, True)])
def test_capi_graph_executor_and_self_via_rccl(K, via_rccl):
    """rma_executor_create_g: a periodic single-rank perf_hide tile replayed
    from hipGraphs (local periodic copies are capturable) == the eager run;
    rma_grid_self_via_rccl routes the halos through RCCL send/recv to itself
    (eager: RCCL is not captured in a torch process) == the same field."""
    L = lib()
    nx, ny, nt = 514, 300, 43
    s = torch.cuda.current_stream().cuda_stream

    def run(graph_steps, rccl):
        g = grid(L, nx, ny, K, periods=(1, 1, 0))
        if rccl:
            ck(L, L.rma_grid_self_via_rccl(g))
        T = torch.from_numpy(golden.initial(nx, ny)).cuda()
        # periodic halos consistent with the owned cells first: the non-periodic
        # gaussian's halo is not, and a pass of depth k reads k stale halo layers,
        # so runs with different pass plans (graph of 10 steps + tail vs one plan
        # of nt) would otherwise differ at the 1e-12 level of the tail values
        ck(L, L.rma_update_halo(g, 1, (ctypes.c_void_p * 1)(T.data_ptr()),
                                (ctypes.c_int64 * 3)(nx, ny, 1), (ctypes.c_int * 1)(8),
                                ctypes.c_void_p(s)))
        T2 = T.clone()
        iCp = torch.ones_like(T)
        ex = ctypes.c_void_p()
        ck(L, L.rma_executor_create_g(g, 1, ctypes.c_void_p(T.data_ptr()),
                                      ctypes.c_void_p(T2.data_ptr()),
                                      ctypes.c_void_p(iCp.data_ptr()), ctypes.c_int64(nx),
                                      ctypes.c_int64(ny), coef4(L, g, nx, ny), ctypes.c_int64(1),
                                      ctypes.c_int64(1), K, 0, graph_steps, None, None, None,
                                      ctypes.byref(ex)))
        ck(L, L.rma_executor_run(ex, ctypes.c_int64(nt), ctypes.c_void_p(s)))
        par = L.rma_executor_parity(ex)
        torch.cuda.synchronize()
        out = (T2 if par else T).cpu().numpy()
        ck(L, L.rma_executor_destroy(ex))
        ck(L, L.rma_finalize_global_grid(g))
        return out

    eager = run(0, False)
    other = run(0, True) if via_rccl else run(10, False)
    assert np.array_equal(eager, other)


def test_capi_kp_executor_with_buffers_matches_golden():
    """rma_executor_create_g in kp mode (2) with the T-indexed qx / qy / dTdt
    buffers (what the Julia shim passes since r4: diffusion_2D_kp.jl:88-91's
    three kernels) == the golden model bitwise; without them the create call
    fails with a message naming kp."""
    L = lib()
    nx, ny, nt = 258, 131, 29
    g = grid(L, nx, ny, 1)
    s = torch.cuda.current_stream().cuda_stream
    T = torch.from_numpy(golden.initial(nx, ny)).cuda()
    iCp = torch.ones_like(T)
    qx, qy, dTdt = (torch.zeros_like(T) for _ in range(3))
    ex = ctypes.c_void_p()
    rc = L.rma_executor_create_g(g, 2, ctypes.c_void_p(T.data_ptr()), None,
                                 ctypes.c_void_p(iCp.data_ptr()), ctypes.c_int64(nx),
                                 ctypes.c_int64(ny), coef4(L, g, nx, ny), ctypes.c_int64(1),
                                 ctypes.c_int64(1), 1, 0, 0, None, None, None, ctypes.byref(ex))
    assert rc != 0 and b"kp" in L.rma_last_error()
    ck(L, L.rma_executor_create_g(g, 2, ctypes.c_void_p(T.data_ptr()), None,
                                  ctypes.c_void_p(iCp.data_ptr()), ctypes.c_int64(nx),
                                  ctypes.c_int64(ny), coef4(L, g, nx, ny), ctypes.c_int64(1),
                                  ctypes.c_int64(1), 1, 0, 0, ctypes.c_void_p(qx.data_ptr()),
                                  ctypes.c_void_p(qy.data_ptr()), ctypes.c_void_p(dTdt.data_ptr()),
                                  ctypes.byref(ex)))
    ck(L, L.rma_executor_run(ex, ctypes.c_int64(nt), ctypes.c_void_p(s)))
    torch.cuda.synchronize()
    field = T.cpu().numpy()
    ck(L, L.rma_executor_destroy(ex))
    ck(L, L.rma_finalize_global_grid(g))
    assert np.array_equal(field, golden.run(nx, ny, nt))


def test_capi_grid_lifetime_with_live_executors():
    """executors pin their grid. rma_grid_self_via_rccl is refused
    while one is alive (it would replace the exchanger under it), and
    finalize before destroy (any GC order of a host such as Julia) defers the
    teardown: the executor still runs, and its destroy frees the grid."""
    L = lib()
    nx, ny, K = 200, 120, 4
    g = grid(L, nx, ny, K, periods=(1, 1, 0))
    s = torch.cuda.current_stream().cuda_stream
    T = torch.from_numpy(golden.initial(nx, ny)).cuda()
    T2, iCp = T.clone(), torch.ones_like(T)
    ex = ctypes.c_void_p()
    ck(L, L.rma_executor_create_g(g, 1, ctypes.c_void_p(T.data_ptr()),
                                  ctypes.c_void_p(T2.data_ptr()), ctypes.c_void_p(iCp.data_ptr()),
                                  ctypes.c_int64(nx), ctypes.c_int64(ny), coef4(L, g, nx, ny),
                                  ctypes.c_int64(1), ctypes.c_int64(1), K, 1, 0, None, None, None,
                                  ctypes.byref(ex)))
    rc = L.rma_grid_self_via_rccl(g)
    assert rc != 0 and b"executor" in L.rma_last_error()
    ck(L, L.rma_finalize_global_grid(g))  # deferred: the executor still holds the grid
    ck(L, L.rma_executor_run(ex, ctypes.c_int64(13), ctypes.c_void_p(s)))
    torch.cuda.synchronize()
    assert bool(torch.isfinite(T).all()) and bool(torch.isfinite(T2).all())
    ck(L, L.rma_executor_destroy(ex))  # last reference: the grid goes with it
