"""Two-step (temporal blocking) kernel vs two one-step launches and the C++
CPU twin: bitwise, over odd/tiny shapes, chunk/unroll choices, rect lists,
unaligned views (scalar path) and both block orders."""
import pytest
import torch

from rocm_mpi_amd import ops
from rocm_mpi_amd._native import native

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def rand(shape, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g, dtype=torch.float64)


def coef():
    return ops.StencilCoef(-1.3, 1 / 0.037, 1 / 0.041, 0.00031)


def two_steps_cpu(T, iCp, rects, fill=-5.0):
    S1 = T.clone()
    ops.stencil_step(S1, T, iCp, coef())
    out = torch.full_like(T, fill)
    ops.stencil_step(out, S1, iCp, coef(), rects)
    return out


SHAPES = [(3, 3), (4, 5), (5, 4), (66, 130), (130, 66), (389, 515), (257, 1024), (100, 2050),
          (31, 4097), (300, 129), (9, 260)]


@pytest.mark.parametrize("ny,nx", SHAPES)
@pytest.mark.parametrize("chunk,unroll", [(1, 2), (8, 2), (6, 4), (13, 4), (64, 2)])
def test_two_step_bitwise(ny, nx, chunk, unroll):
    T, iCp = rand((ny, nx), 1), rand((ny, nx), 2) + 0.5
    ref = two_steps_cpu(T, iCp, [ops.interior_rect(nx, ny)])
    out = torch.full((ny, nx), -5.0, dtype=torch.float64, device=DEV)
    ops.stencil2_step(out, T.to(DEV), iCp.to(DEV), coef(),
                      tuning=ops.StencilTuning(chunk_rows=chunk, unroll=unroll))
    assert torch.equal(out.cpu(), ref)
    cpu = torch.full_like(T, -5.0)  # the C++ twin
    ops.stencil2_step(cpu, T, iCp, coef())
    assert torch.equal(cpu, ref)


@pytest.mark.parametrize("xcd", [0, 1])
def test_two_step_rect_lists(xcd):
    """Frame + interior rects (as the multi-rank executor issues them)."""
    ny, nx = 301, 700
    T, iCp = rand((ny, nx), 3), rand((ny, nx), 4) + 0.5
    rects = [(2, nx - 2, 2, 4), (2, nx - 2, ny - 4, ny - 2), (2, 4, 4, ny - 4),
             (nx - 4, nx - 2, 4, ny - 4)]
    interior = (4, nx - 4, 4, ny - 4)
    ref = two_steps_cpu(T, iCp, rects + [interior])
    out = torch.full((ny, nx), -5.0, dtype=torch.float64, device=DEV)
    Td, iCpd = T.to(DEV), iCp.to(DEV)
    tn = ops.StencilTuning(chunk_rows=8, unroll=2, xcd_remap=xcd)
    ops.stencil2_step(out, Td, iCpd, coef(), rects, tn)
    ops.stencil2_step(out, Td, iCpd, coef(), [interior], tn)
    assert torch.equal(out.cpu(), ref)


def test_two_step_unaligned_view():
    base = rand(64 * 200 + 1, 5).to(DEV)
    T = base[1:].view(200, 64)  # 8-byte aligned only -> V=1 path
    iCp = torch.ones((200, 64), dtype=torch.float64, device=DEV)
    out = torch.zeros((200, 64), dtype=torch.float64, device=DEV)
    ops.stencil2_step(out, T, iCp, coef())
    ref = two_steps_cpu(T.cpu(), iCp.cpu(), [ops.interior_rect(64, 200)], fill=0.0)
    assert torch.equal(out.cpu(), ref)


def test_two_step_rejects_in_place_and_bad_rects():
    T = rand((10, 10), 6).to(DEV)
    with pytest.raises(ValueError):
        ops.stencil2_step(T, T, T, coef())
    with pytest.raises(ValueError):
        ops.stencil2_step(torch.empty_like(T), T, T, coef(), [(0, 5, 1, 5)])


def k_steps_cpu(K, T, iCp, rects, fill=-5.0):
    a = T.clone()
    for _ in range(K - 1):
        b = a.clone()
        ops.stencil_step(b, a, iCp, coef())
        a = b
    out = torch.full_like(T, fill)
    ops.stencil_step(out, a, iCp, coef(), rects)
    return out


@pytest.mark.parametrize("K", [2, 3, 4, 6, 8])
@pytest.mark.parametrize("ny,nx", SHAPES)
@pytest.mark.parametrize("chunk,vec,kern", [(1, 2, "march"), (5, 4, "march"), (16, 2, "march"),
                                            (16, 4, "march"), (64, 2, "march"), (3, 2, "lds"),
                                            (16, 4, "lds"), (64, 2, "lds"), (7, 2, "dpp"),
                                            (16, 4, "dpp"), (5, 2, "lds_dpp"), (64, 2, "lds_dpp")])
def test_k_step_bitwise(K, ny, nx, chunk, vec, kern):
    """K-step kernel with face-flux reuse == K one-step launches, bitwise."""
    T, iCp = rand((ny, nx), 7), rand((ny, nx), 8) + 0.5
    ref = k_steps_cpu(K, T, iCp, [ops.interior_rect(nx, ny)])
    out = torch.full((ny, nx), -5.0, dtype=torch.float64, device=DEV)
    ops.stencilk_step(K, out, T.to(DEV), iCp.to(DEV), coef(),
                      tuning=ops.StencilTuning(chunk_rows=chunk, vec=vec, kernel=kern))
    assert torch.equal(out.cpu(), ref)
    cpu = torch.full_like(T, -5.0)  # the C++ twin
    ops.stencilk_step(K, cpu, T, iCp, coef())
    assert torch.equal(cpu, ref)


@pytest.mark.parametrize("K", [3, 4, 6, 8])
@pytest.mark.parametrize("xcd", [0, 1])
def test_k_step_rect_lists_and_unaligned(K, xcd):
    ny, nx = 203, 900
    T, iCp = rand((ny, nx), 9), rand((ny, nx), 10) + 0.5
    w = K
    rects = [(w, nx - w, w, 2 * w), (w, nx - w, ny - 2 * w, ny - w), (w, 2 * w, 2 * w, ny - 2 * w),
             (nx - 2 * w, nx - w, 2 * w, ny - 2 * w)]
    interior = (2 * w, nx - 2 * w, 2 * w, ny - 2 * w)
    ref = k_steps_cpu(K, T, iCp, rects + [interior])
    out = torch.full((ny, nx), -5.0, dtype=torch.float64, device=DEV)
    tn = ops.StencilTuning(chunk_rows=16, xcd_remap=xcd)
    Td, iCpd = T.to(DEV), iCp.to(DEV)
    ops.stencilk_step(K, out, Td, iCpd, coef(), rects, tn)
    ops.stencilk_step(K, out, Td, iCpd, coef(), [interior], tn)
    assert torch.equal(out.cpu(), ref)
    base = rand(64 * 150 + 1, 11).to(DEV)  # 8-byte aligned view -> V=1 path
    Tu = base[1:].view(150, 64)
    ones = torch.ones((150, 64), dtype=torch.float64, device=DEV)
    o2 = torch.zeros_like(ones)
    ops.stencilk_step(K, o2, Tu, ones, coef(), tuning=tn)
    assert torch.equal(o2.cpu(), k_steps_cpu(K, Tu.cpu(), ones.cpu(),
                                             [ops.interior_rect(64, 150)], fill=0.0))


@pytest.mark.parametrize("K", [2, 3, 4, 6, 8])
@pytest.mark.parametrize("ny,nx", [(3, 3), (67, 131), (257, 1024), (300, 129), (31, 4097)])
@pytest.mark.parametrize("kern,vec,chunk", [("fast", 2, 16), ("fast5", 2, 16), ("fast5", 4, 5),
                                            ("fast5", 2, 7), ("fast5", 2, 64), ("fast5", 2, 1)])
def test_k_step_fast_variant_close(K, ny, nx, kern, vec, chunk):
    """kernel='fast' reassociates the update (differences, folded constants,
    FMAs) and 'fast5' evaluates the 5-point sum with one folded
    per-cell factor: not bitwise, but within a few ulp of the canonical K
    steps, and boundary cells stay exactly fixed."""
    T, iCp = rand((ny, nx), 12), rand((ny, nx), 13) + 0.5
    ref = k_steps_cpu(K, T, iCp, [ops.interior_rect(nx, ny)])
    out = torch.full((ny, nx), -5.0, dtype=torch.float64, device=DEV)
    ops.stencilk_step(K, out, T.to(DEV), iCp.to(DEV), coef(),
                      tuning=ops.StencilTuning(chunk_rows=chunk, kernel=kern, vec=vec))
    o = out.cpu()
    assert torch.equal(o[0], ref[0]) and torch.equal(o[:, 0], ref[:, 0])
    torch.testing.assert_close(o, ref, rtol=1e-13, atol=1e-13)


def test_fast5_rejects_zero_lambda():
    """kernel 5 divides by lam/dx^2: lam == 0 is refused before any launch."""
    T = rand((40, 40), 14).to(DEV)
    with pytest.raises(ValueError):
        ops.stencilk_step(4, torch.empty_like(T), T, torch.ones_like(T),
                          ops.StencilCoef(0.0, 10.0, 10.0, 1e-3),
                          tuning=ops.StencilTuning(chunk_rows=16, kernel="fast5"))


@pytest.mark.parametrize("K", [12, 16])
@pytest.mark.parametrize("ny,nx", [(3, 3), (67, 131), (257, 1024), (300, 129), (41, 4097)])
@pytest.mark.parametrize("chunk,xcd", [(16, 1), (1, 0), (50, 1), (37, 0)])
def test_deep_k_step_fast5_close(K, ny, nx, chunk, xcd):
    """12 / 16 steps per pass (fast5 kernel only): within rounding of the
    canonical K steps, boundary cells fixed."""
    T, iCp = rand((ny, nx), 15), rand((ny, nx), 16) + 0.5
    ref = k_steps_cpu(K, T, iCp, [ops.interior_rect(nx, ny)])
    out = torch.full((ny, nx), -5.0, dtype=torch.float64, device=DEV)
    ops.stencilk_step(K, out, T.to(DEV), iCp.to(DEV), coef(),
                      tuning=ops.StencilTuning(chunk_rows=chunk, kernel="fast5", xcd_remap=xcd))
    o = out.cpu()
    assert torch.equal(o[0], ref[0]) and torch.equal(o[:, 0], ref[:, 0])
    torch.testing.assert_close(o, ref, rtol=1e-13, atol=1e-13)


def test_deep_k_needs_fast5():
    T = rand((40, 40), 17).to(DEV)
    with pytest.raises(ValueError):
        ops.stencilk_step(12, torch.empty_like(T), T, torch.ones_like(T), coef(),
                          tuning=ops.StencilTuning(chunk_rows=16, kernel="fast"))


@pytest.mark.parametrize("K", [4, 16])
def test_fast5_rect_lists(K):
    """Frame + interior rects as the executor issues them (thin column rects)."""
    ny, nx = 203, 900
    T, iCp = rand((ny, nx), 20), rand((ny, nx), 21) + 0.5
    w = K
    rects = [(w, nx - w, w, 2 * w), (w, nx - w, ny - 2 * w, ny - w), (w, 2 * w, 2 * w, ny - 2 * w),
             (nx - 2 * w, nx - w, 2 * w, ny - 2 * w)]
    interior = (2 * w, nx - 2 * w, 2 * w, ny - 2 * w)
    out = torch.full((ny, nx), -5.0, dtype=torch.float64, device=DEV)
    tn = ops.StencilTuning(chunk_rows=16, kernel="fast5", xcd_remap=1)
    Td, iCpd = T.to(DEV), iCp.to(DEV)
    ops.stencilk_step(K, out, Td, iCpd, coef(), rects, tn)
    ops.stencilk_step(K, out, Td, iCpd, coef(), [interior], tn)
    ref = k_steps_cpu(K, T, iCp, rects + [interior])
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("K,kern", [(8, "fast5p2"), (12, "fast5p2"), (16, "fast5p2"),
                                    (8, "fast5p4"), (12, "fast5p4"), (16, "fast5p4"),
                                    (8, "fast5p8"), (16, "fast5p8")])
@pytest.mark.parametrize("ny,nx", [(3, 3), (67, 131), (257, 1024), (300, 129), (41, 4097),
                                   (130, 515), (19, 2000)])
@pytest.mark.parametrize("chunk,xcd,vec", [(16, 1, 2), (1, 0, 2), (37, 1, 2), (16, 1, 4),
                                           (5, 0, 4)])
def test_pipelined_fast5_equals_fast5_bitwise(K, kern, ny, nx, chunk, xcd, vec):
    """The stage-pipelined kernels (levels of a strip split over 2 / 4 / 8 waves,
    hand-off rows through LDS; 2 or 4 cells per lane) compute exactly kernel
    fast5's operations."""
    T, iCp = rand((ny, nx), 18), rand((ny, nx), 19) + 0.5
    Td, iCpd = T.to(DEV), iCp.to(DEV)
    outs = []
    for kn, vv in (("fast5", 2), (kern, vec)):
        out = torch.full((ny, nx), -5.0, dtype=torch.float64, device=DEV)
        ops.stencilk_step(K, out, Td, iCpd, coef(),
                          tuning=ops.StencilTuning(chunk_rows=chunk, kernel=kn, xcd_remap=xcd,
                                                   vec=vv))
        outs.append(out.cpu())
    assert torch.equal(outs[0], outs[1])


@pytest.mark.slow
@pytest.mark.parametrize("K,kern,vec", [(16, "fast5p4", 4), (8, "lds_dpp", 2)])
def test_k_step_int64_indexing(K, kern, vec):
    """K-step kernels on a tile beyond 2^31 cells (64-bit row offsets, as at the
    288 GB bench tile): the last rows of the big tile equal the same kernel run
    on a small copy of those rows (a K-step result depends on K rows around it,
    so rows >= K away from the copy's top edge agree bitwise)."""
    free, _ = torch.cuda.mem_get_info()
    ny, nx = 33000, 65536  # 2.16e9 cells, 17.3 GB per array
    if free < 3 * ny * nx * 8 * 1.1:
        pytest.skip("not enough HBM")
    T = torch.empty((ny, nx), dtype=torch.float64, device=DEV)
    ops.init_random_(T, ops.TileGeometry(0, 0, nx, ny, 1.0, 1.0), seed=5)
    iCp = torch.empty_like(T)
    ops.init_random_(iCp, ops.TileGeometry(0, 0, nx, ny, 1.0, 1.0), seed=6)
    iCp.add_(0.5)
    out = torch.zeros_like(T)
    tn = ops.StencilTuning(chunk_rows=16, kernel=kern, xcd_remap=1, vec=vec)
    rows = 40
    ops.stencilk_step(K, out, T, iCp, coef(), [(1, nx - 1, ny - rows, ny - 1)], tn)
    got = out[ny - rows:ny - 1].cpu()
    del out
    h = rows + 2 * K  # the copy: K + rows + K rows, the last one the fixed boundary row
    Ts, Cs = T[ny - h:].clone(), iCp[ny - h:].clone()
    del T, iCp
    small = torch.zeros_like(Ts)
    ops.stencilk_step(K, small, Ts, Cs, coef(), [(1, nx - 1, h - rows, h - 1)], tn)
    assert torch.equal(got, small[h - rows:h - 1].cpu())
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def headline_width_tile():
    """A 101120-column tile (the headline's row width, nx % 4 == 0) of
    2.15e9 cells > 2^31, random T and 1/Cp; freed after the module."""
    free, _ = torch.cuda.mem_get_info()
    ny, nx = 21300, 101120
    if free < 3 * ny * nx * 8 * 1.1:
        pytest.skip("not enough HBM")
    T = torch.empty((ny, nx), dtype=torch.float64, device=DEV)
    ops.init_random_(T, ops.TileGeometry(0, 0, nx, ny, 1.0, 1.0), seed=7)
    iCp = torch.empty_like(T)
    ops.init_random_(iCp, ops.TileGeometry(0, 0, nx, ny, 1.0, 1.0), seed=8)
    iCp.mul_(0.5).add_(0.5)
    out = torch.zeros_like(T)
    yield T, iCp, out
    del T, iCp, out
    torch.cuda.empty_cache()


@pytest.mark.slow
@pytest.mark.parametrize("kern,K", [("piper", 20), ("piper", 24), ("pipe", 20), ("pipe", 24),
                                    ("pipec", 20), ("piper", 17)])
def test_headline_kernels_beyond_2e31_cells(headline_width_tile, kern, K):
    """the kernels the bench times (piper, kernel 12), the
    ring kernel (pipe, 9) and the canonical side number (pipec, 10) on a tile
    of > 2^31 cells with the headline's 101120-column rows: uniform 64-bit
    row bases + 32-bit lane byte offsets (stencil_pipe.h). Rows at the top,
    across the 2^31-cell boundary and at the bottom edge equal the C++ CPU
    twin of the same arithmetic run on a copy of the rows they depend on."""
    T, iCp, out = headline_width_tile
    ny, nx = T.shape
    rows = 24
    twin = "pipec" if kern == "pipec" else "pipe"
    if kern == "pipec":
        tn = ops.StencilTuning(chunk_rows=native().pipe_chunk_rows(K, ny, True) or 1024,
                               kernel="pipec", xcd_remap=1, vec=4)
    else:
        kid, vec, ch = native().fast_kernel_k(K, ny, tuple(coef()))
        tn = ops.StencilTuning(chunk_rows=ch, kernel=kern, xcd_remap=1, vec=4)
    cross = (2 ** 31) // nx  # the row holding cell 2^31
    for y0 in (1, cross - rows // 2, ny - 1 - rows):
        y1 = y0 + rows
        out.fill_(-7.0)
        ops.stencilk_step(K, out, T, iCp, coef(), [(1, nx - 1, y0, y1)], tn)
        got = out[y0:y1].cpu()
        # the CPU twin on the dependency rows [y0-K, y1+K) clipped to the tile
        a0, a1 = max(0, y0 - K), min(ny, y1 + K)
        Ts, Cs = T[a0:a1].cpu(), iCp[a0:a1].cpu()
        ref = torch.full_like(Ts, -7.0)
        ops.stencilk_step(K, ref, Ts, Cs, coef(), [(1, nx - 1, y0 - a0, y1 - a0)],
                          ops.StencilTuning(kernel=twin))
        want = ref[y0 - a0:y1 - a0]
        # columns 0 and nx-1 are boundary cells (not written): compare inner ones
        assert torch.equal(got[:, 1:nx - 1], want[:, 1:nx - 1]), (kern, K, y0)
        assert bool((got[:, 0] == -7.0).all()) and bool((got[:, nx - 1] == -7.0).all())


@pytest.mark.parametrize("kern", ["fast5p2", "fast5p4", "fast5p8"])
def test_pipelined_fast5_rect_lists(kern):
    K, ny, nx = 16, 203, 900
    T, iCp = rand((ny, nx), 20), rand((ny, nx), 21) + 0.5
    w = K
    rects = [(w, nx - w, w, 2 * w), (w, nx - w, ny - 2 * w, ny - w), (w, 2 * w, 2 * w, ny - 2 * w),
             (nx - 2 * w, nx - w, 2 * w, ny - 2 * w)]
    interior = (2 * w, nx - 2 * w, 2 * w, ny - 2 * w)
    Td, iCpd = T.to(DEV), iCp.to(DEV)
    outs = []
    for kn in ("fast5", kern):
        out = torch.full((ny, nx), -5.0, dtype=torch.float64, device=DEV)
        tn = ops.StencilTuning(chunk_rows=16, kernel=kn, xcd_remap=1)
        ops.stencilk_step(K, out, Td, iCpd, coef(), rects, tn)
        ops.stencilk_step(K, out, Td, iCpd, coef(), [interior], tn)
        outs.append(out.cpu())
    assert torch.equal(outs[0], outs[1])
