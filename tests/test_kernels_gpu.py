"""GPU numerics of the hand-written gfx950 kernels vs plain PyTorch references.

Every kernel is compared against (a) a pure-torch formulation of the same op
(float64, same operation order => bitwise) and (b) the C++ CPU twin.
"""
import pytest
import torch

from rocm_mpi_amd import ops
from rocm_mpi_amd._native import native

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def rand(shape, seed=0, device=DEV):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g, dtype=torch.float64).to(device)


def coef():
    return ops.StencilCoef(-1.3, 1 / 0.037, 1 / 0.041, 0.00031)


SHAPES = [(3, 3), (5, 4), (66, 130), (130, 66), (389, 515), (257, 1024), (100, 2050), (31, 4097)]


@pytest.mark.parametrize("ny,nx", SHAPES)
@pytest.mark.parametrize("chunk", [1, 7, 64])
def test_stencil_march_bitwise(ny, nx, chunk):
    T = rand((ny, nx), 1)
    iCp = rand((ny, nx), 2) + 0.5
    out = torch.full_like(T, -7.0)
    ops.stencil_step(out, T, iCp, coef(), tuning=ops.StencilTuning(chunk_rows=chunk))
    ref = torch.full((ny, nx), -7.0, dtype=torch.float64)
    ops.stencil_torch(ref, T.cpu(), iCp.cpu(), coef(), [ops.interior_rect(nx, ny)])
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), ref)  # boundary untouched, interior bitwise


@pytest.mark.parametrize("kernel", ["march", "lds"])
@pytest.mark.parametrize("nt", [False, True])
def test_stencil_variants_and_rect_lists(kernel, nt):
    ny, nx = 300, 700
    T = rand((ny, nx), 3)
    iCp = rand((ny, nx), 4) + 0.5
    frame, interior = ops.hide_rects(nx, ny, 5, 3)
    tn = ops.StencilTuning(chunk_rows=16, nontemporal=nt, kernel=kernel)
    out = torch.zeros_like(T)
    ops.stencil_step(out, T, iCp, coef(), frame, tn)
    ops.stencil_step(out, T, iCp, coef(), [interior], tn)
    full = torch.zeros_like(T)
    ops.stencil_step(full, T, iCp, coef(), tuning=tn)
    ref = torch.zeros((ny, nx), dtype=torch.float64)
    ops.stencil_torch(ref, T.cpu(), iCp.cpu(), coef(), [ops.interior_rect(nx, ny)])
    assert torch.equal(out.cpu(), ref)
    assert torch.equal(full.cpu(), ref)


@pytest.mark.parametrize("w", [1, 2, 3, 8, 9])
def test_stencil_thin_column_rects(w):
    """Rects at most 8 cells wide run in column mode (one thread per row)."""
    ny, nx = 700, 300
    T = rand((ny, nx), 11)
    iCp = rand((ny, nx), 12) + 0.5
    rects = [(1, 1 + w, 2, ny - 2), (nx - 1 - w, nx - 1, 3, ny - 1), (150, 150 + w, 1, 40)]
    out = torch.zeros_like(T)
    ops.stencil_step(out, T, iCp, coef(), rects)
    ref = torch.zeros((ny, nx), dtype=torch.float64)
    ops.stencil_torch(ref, T.cpu(), iCp.cpu(), coef(), rects)
    assert torch.equal(out.cpu(), ref)


def test_stencil_unaligned_pointer_path():
    # a view starting one element in: 8-byte aligned only -> scalar (V=1) path
    base = rand(64 * 200 + 1, 5)
    T = base[1:].view(200, 64)
    iCp = torch.ones((200, 64), dtype=torch.float64, device=DEV)
    out = torch.zeros((200, 64), dtype=torch.float64, device=DEV)
    ops.stencil_step(out, T, iCp, coef())
    ref = torch.zeros((200, 64), dtype=torch.float64)
    ops.stencil_torch(ref, T.cpu(), iCp.cpu(), coef(), [ops.interior_rect(64, 200)])
    assert torch.equal(out.cpu(), ref)


def test_stencil_rejects_bad_rect():
    T = rand((10, 10))
    with pytest.raises(ValueError):
        ops.stencil_step(torch.empty_like(T), T, T, coef(), [(0, 5, 1, 5)])
    with pytest.raises(RuntimeError):  # native validation (bypassing Python checks)
        native().stencil_rects(T.data_ptr(), T.data_ptr(), T.data_ptr(), 10, 10, [(1, 10, 1, 9)],
                               tuple(coef()), 64, 0, 0, 0, True)


@pytest.mark.parametrize("ny,nx", [(3, 4), (3, 3), (67, 132), (67, 131), (256, 1024), (101, 514)])
def test_kp_kernels_bitwise(ny, nx):
    c = coef()
    T = rand((ny, nx), 6)
    iCp = rand((ny, nx), 7) + 0.5
    res = {}
    for dev in (DEV, "cpu"):
        Td, iCpd = T.to(dev).clone(), iCp.to(dev)
        QX, QY, D = (torch.zeros((ny, nx), dtype=torch.float64, device=dev) for _ in range(3))
        ops.flux(QX, QY, Td, c.mlam, c.rdx, c.rdy)
        ops.residual(D, QX, QY, iCpd, c.rdx, c.rdy)
        ops.update(Td, D, c.dt)
        res[dev] = tuple(v.cpu().clone() for v in ops.kp_views(QX, QY, D)) + (Td.cpu(),)
    for a, b in zip(res[DEV], res["cpu"]):
        assert torch.equal(a, b)
    # the reference-shaped views match the plain formulas of kp.jl:16-54
    Tc = T.cpu()
    qx = (c.mlam * (Tc[1:-1, 1:] - Tc[1:-1, :-1])) * c.rdx
    qy = (c.mlam * (Tc[1:, 1:-1] - Tc[:-1, 1:-1])) * c.rdy
    assert torch.equal(res[DEV][0], qx) and torch.equal(res[DEV][1], qy)
    # kp == fused stencil
    fused = Tc.clone()
    ops.stencil_torch(fused, Tc, iCp.cpu(), c, [ops.interior_rect(nx, ny)])
    assert torch.equal(res[DEV][3], fused)


def test_init_kernels():
    geom = ops.TileGeometry(gx0=126, gy0=0, nxg=254, nyg=254, dx=10 / 254, dy=10 / 254)
    a = torch.empty((128, 128), dtype=torch.float64, device=DEV)
    b = torch.empty((128, 128), dtype=torch.float64)
    ops.init_random_(a, geom, seed=42)
    ops.init_random_(b, geom, seed=42)
    assert torch.equal(a.cpu(), b)
    assert 0.0 <= float(b.min()) and float(b.max()) < 1.0
    ops.init_gaussian_(a, geom, 10.0, 10.0)
    ops.init_gaussian_(b, geom, 10.0, 10.0)
    torch.testing.assert_close(a.cpu(), b, rtol=4e-16, atol=1e-300)


def test_init_random_is_decomposition_invariant():
    geom_full = ops.TileGeometry(0, 0, 254, 254, 1.0, 1.0)
    full = torch.empty((254, 254), dtype=torch.float64, device=DEV)
    ops.init_random_(full, geom_full, seed=7)
    part = torch.empty((128, 128), dtype=torch.float64, device=DEV)
    ops.init_random_(part, ops.TileGeometry(126, 126, 254, 254, 1.0, 1.0), seed=7)
    assert torch.equal(part, full[126:, 126:])


@pytest.mark.parametrize("elem", [torch.float64, torch.float32, torch.float16])
def test_copy_plane_strided(elem):
    A = rand((37, 53), 8).to(elem)
    col = A[:, 3:5]  # strided plane: 37 rows of 2
    buf = torch.empty((37, 2), dtype=elem, device=DEV)
    ops.copy_plane(buf, col)
    assert torch.equal(buf, col)
    B = torch.zeros_like(A)
    ops.copy_plane(B[:, 50:52], buf)
    assert torch.equal(B[:, 50:52], col)
    assert float(B[:, :50].abs().sum()) == 0.0


@pytest.mark.parametrize("c0,w", [(2, 4), (3, 4), (16, 16), (2, 3)])
def test_copy_plane_fp64_wide_rows(c0, w):
    """fp64 planes with even rows, even leading dims and 16-B aligned rows are
    moved as 16-byte elements (width-K halos); the others element by element."""
    A = rand((41, 54), 10).to(DEV)
    col = A[:, c0:c0 + w]
    buf = torch.empty((41, w), dtype=torch.float64, device=DEV)
    ops.copy_plane(buf, col)
    assert torch.equal(buf, col)
    B = torch.zeros_like(A)
    ops.copy_plane(B[:, 30:30 + w], buf)
    assert torch.equal(B[:, 30:30 + w], col)
    assert float(B[:, :30].abs().sum()) == 0.0 and float(B[:, 30 + w:].abs().sum()) == 0.0


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32, torch.float16])
def test_copy_planes_batch(dtype):
    """One launch, copies of every shape class: narrow rows (n_k = 1, odd, K),
    rows wider than a block, a contiguous plane, an empty copy, unaligned
    columns (the batch falls back to 8-byte elements for all copies)."""
    A = rand((301, 700), 12).to(dtype)
    B = torch.zeros_like(A)
    planes = [(slice(0, 301), slice(3, 4)), (slice(0, 301), slice(10, 17)),
              (slice(0, 300), slice(40, 64)), (slice(5, 9), slice(0, 700)),
              (slice(100, 140), slice(65, 365)), (slice(0, 0), slice(0, 5)),
              (slice(200, 201), slice(1, 699)), (slice(7, 290), slice(400, 402))]
    ops.copy_planes([(B[r, c], A[r, c]) for r, c in planes])
    ref = torch.zeros_like(A)
    for r, c in planes:
        ref[r, c] = A[r, c]
    assert torch.equal(B, ref)


def test_copy_planes_halo_shapes_16b():
    """The halo engine's fp64 batch at K = 24: two x-planes packed into
    contiguous buffers (16-byte elements), unpacked into the halo columns."""
    n, K = 4099, 24
    T = rand((n, n + 1), 13)[:, :n]  # odd leading dim: 8-byte path
    U = rand((n, n), 14)
    for F in (T, U):
        bl = torch.empty((n, K), dtype=torch.float64, device=DEV)
        bh = torch.empty_like(bl)
        ops.copy_planes([(bl, F[:, K:2 * K]), (bh, F[:, n - 2 * K:n - K])])
        assert torch.equal(bl, F[:, K:2 * K]) and torch.equal(bh, F[:, n - 2 * K:n - K])
        G = F.clone()
        ops.copy_planes([(G[:, :K], bh), (G[:, n - K:], bl)])
        assert torch.equal(G[:, :K], F[:, n - 2 * K:n - K]) and torch.equal(G[:, n - K:], F[:, K:2 * K])
        assert torch.equal(G[:, K:n - K], F[:, K:n - K])


def test_copy_planes_rejects_mixed_and_oversized():
    A = rand((16, 16), 15)
    with pytest.raises(ValueError):
        ops.copy_planes([(A[:, :2], A[:, 4:6]), (A.float()[:, :2], A.float()[:, 4:6])])
    with pytest.raises(ValueError):
        ops.copy_planes([(A[:, :1], A[:, 1:2])] * 9)


@pytest.mark.parametrize("op", ["sum", "max", "min", "maxabs", "nonfinite"])
def test_reduce(op):
    A = rand((513, 257), 9) - 0.5
    A[3, 7] = float("nan") if op == "nonfinite" else A[3, 7]
    got = float(ops.reduce(A, op))
    c = A.cpu()
    want = {"sum": lambda: float(c.sum()), "max": lambda: float(c.max()),
            "min": lambda: float(c.min()), "maxabs": lambda: float(c.abs().max()),
            "nonfinite": lambda: 1.0}[op]()
    assert got == pytest.approx(want, rel=1e-12, abs=1e-12)


@pytest.mark.slow
def test_stencil_int64_indexing():
    """A tile beyond 2^31 cells (64-bit offsets), checked on the last rows."""
    free, _ = torch.cuda.mem_get_info()
    ny, nx = 33000, 65536  # 2.16e9 cells, 17.3 GB per array
    if free < 3 * ny * nx * 8 * 1.1:
        pytest.skip("not enough HBM")
    T = torch.empty((ny, nx), dtype=torch.float64, device=DEV)
    ops.init_random_(T, ops.TileGeometry(0, 0, nx, ny, 1.0, 1.0), seed=3)
    iCp = torch.empty_like(T)
    ops.fill_(iCp, 1.0)
    out = torch.zeros_like(T)
    ops.stencil_step(out, T, iCp, coef(), [(1, nx - 1, ny - 9, ny - 1)])
    ref = torch.zeros((10, nx), dtype=torch.float64)
    ops.stencil_torch(ref, T[ny - 10:].cpu(), iCp[ny - 10:].cpu(), coef(), [(1, nx - 1, 1, 9)])
    assert torch.equal(out[ny - 9:ny - 1].cpu(), ref[1:9])
    del T, iCp, out
    torch.cuda.empty_cache()


def test_flag_kernels_write_wait_and_bounded_timeout():
    """The IPC transport's flag kernels (csrc/kernels/flags.hip): a write is
    seen by a later wait on the same stream; a wait whose value never comes
    gives up after its timeout, records its code in the error word and lets
    the stream drain (every wave exits: no hang); neighbours untouched."""
    import time

    from rocm_mpi_amd._native import native

    n = native()
    s = torch.cuda.current_stream().cuda_stream
    guard = torch.full((3,), -7, dtype=torch.int64, device="cuda")  # [canary, flag, canary]
    err = torch.zeros(3, dtype=torch.int32, device="cuda")
    flag = guard.data_ptr() + 8
    n.flag_write(flag, 5, s)
    n.flag_wait(flag, 5, 5.0, err.data_ptr() + 4, 11, s)
    torch.cuda.synchronize()
    assert guard.tolist() == [-7, 5, -7] and err.tolist() == [0, 0, 0]
    t0 = time.perf_counter()
    n.flag_wait(flag, 6, 0.2, err.data_ptr() + 4, 12, s)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert err.tolist() == [0, 12, 0] and 0.15 < dt < 5.0, (err.tolist(), dt)
    assert guard.tolist() == [-7, 5, -7]


@pytest.mark.parametrize("n,offset", [(1, 0), (7, 0), (4097, 0), (4097, 1), (3 * 2**20 + 5, 1),
                                      (2**24, 0)])
def test_field_stats_gpu_equals_cpu_twin(n, offset):
    """One-pass field statistics (bench.py full-field check): non-finite
    count, min and max of the finite cells, on aligned and 8-byte-offset
    views, odd lengths, with NaN / +-inf planted; equal to the CPU twin."""
    g = torch.Generator().manual_seed(n + offset)
    base = torch.rand(n + offset, generator=g, dtype=torch.float64) * 6 - 3
    a = base[offset:]
    if n > 8:
        a[n // 3] = float("nan")
        a[n - 1] = float("inf")
        a[0] = -float("inf")
    ref = ops.field_stats(a.contiguous())
    d = base.to("cuda")[offset:]
    assert ops.field_stats(d) == ref
