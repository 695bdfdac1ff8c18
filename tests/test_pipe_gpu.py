"""Any-K stage-pipelined kernels (csrc/kernels/stencil_pipe.h): ``pipe`` (fast5
arithmetic) and ``pipec`` (canonical) against the C++ CPU twins, bitwise, for
every pass depth K = 1..24, every cells-per-lane path (odd nx: 1, nx = 2 mod 4:
2, nx = 0 mod 4: 4), rect lists, alternative stage splits, and against the
fixed-K kernels they generalise (fast5 / fast5p4, lds_dpp). Guard bands catch
out-of-bounds writes."""
import pytest
import torch

from rocm_mpi_amd import ops
from rocm_mpi_amd._native import native

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def rand(shape, seed, lo=0.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return lo + (hi - lo) * torch.rand(shape, generator=g, dtype=torch.float64)


def coef():
    # dx != dy (ry != 1), stable explicit step for 1/Cp <= 1
    return ops.StencilCoef(-1.3, 1 / 0.037, 1 / 0.041, 0.00031)


def cpu_ref(K, T, iCp, rects, kernel, fill=-5.0):
    out = torch.full_like(T, fill)
    ops.stencilk_step(K, out, T, iCp, coef(), rects, ops.StencilTuning(kernel=kernel))
    return out


def gpu_run(K, T, iCp, rects, kernel, fill=-5.0, **kw):
    out = torch.full(T.shape, fill, dtype=torch.float64, device=DEV)
    tn = ops.StencilTuning(kernel=kernel, xcd_remap=kw.pop("xcd", 1),
                           chunk_rows=kw.pop("chunk", 16), vec=kw.pop("vec", 4),
                           stages=kw.pop("stages", 0), cols=kw.pop("cols", 0))
    ops.stencilk_step(K, out, T.to(DEV), iCp.to(DEV), coef(), rects, tn)
    return out.cpu()


@pytest.mark.parametrize("kernel", ["pipe", "pipec"])
@pytest.mark.parametrize("nx", [515, 518, 520])
@pytest.mark.parametrize("K", list(range(1, 25)))
def test_pipe_every_depth_bitwise_vs_cpu_twin(kernel, nx, K):
    ny = 131
    T, iCp = rand((ny, nx), 1), rand((ny, nx), 2, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    ref = cpu_ref(K, T, iCp, rects, kernel)
    out = gpu_run(K, T, iCp, rects, kernel, chunk=37)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("kernel", ["pipe", "pipec"])
@pytest.mark.parametrize("K", [3, 10, 16, 20, 24])
@pytest.mark.parametrize("xcd", [0, 1])
def test_pipe_rect_lists(kernel, K, xcd):
    """Frame + interior rects, as the multi-rank executor issues a pass."""
    ny, nx = 301, 1024
    T, iCp = rand((ny, nx), 3), rand((ny, nx), 4, 0.5, 1.0)
    w = K + 1
    frame = [(K, nx - K, K, K + w), (K, nx - K, ny - K - w, ny - K), (K, K + w, K + w, ny - K - w),
             (nx - K - w, nx - K, K + w, ny - K - w)]
    interior = (K + w, nx - K - w, K + w, ny - K - w)
    ref = cpu_ref(K, T, iCp, frame + [interior], kernel)
    out = torch.full((ny, nx), -5.0, dtype=torch.float64, device=DEV)
    Td, iCpd = T.to(DEV), iCp.to(DEV)
    ops.stencilk_step(K, out, Td, iCpd, coef(), frame,
                      ops.StencilTuning(kernel=kernel, chunk_rows=16, vec=2, xcd_remap=xcd))
    ops.stencilk_step(K, out, Td, iCpd, coef(), [interior],
                      ops.StencilTuning(kernel=kernel, chunk_rows=64, vec=4, xcd_remap=xcd))
    assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("nx", [516, 1028, 1500, 2052])
@pytest.mark.parametrize("K", [16, 20, 24])
def test_pipe_two_column_waves_bitwise(nx, K):
    """Blocks of 2 column waves per stage (8 waves over 500 columns, stage
    boundaries inside the block exchanged through LDS each row): bitwise equal
    to the CPU twin, also on rect lists whose strips end mid-block."""
    ny = 149
    T, iCp = rand((ny, nx), 11 + K), rand((ny, nx), 12, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    ref = cpu_ref(K, T, iCp, rects, "pipe")
    assert torch.equal(gpu_run(K, T, iCp, rects, "pipe", chunk=41, cols=2), ref)
    sub = [(K + 3, nx - K - 7, K + 2, ny - K - 5), (1, K + 3, 1, ny - 1)]
    ref = cpu_ref(K, T, iCp, sub, "pipe")
    assert torch.equal(gpu_run(K, T, iCp, sub, "pipe", chunk=23, cols=2, xcd=0), ref)


@pytest.mark.parametrize("nx", [516, 1028, 1500, 2052])
@pytest.mark.parametrize("K,kern", [(16, "piper"), (20, "piper"), (24, "piper"), (20, "piper_rot"),
                                    (24, "piper_rot")])
def test_piper_two_column_waves_bitwise(nx, K, kern):
    """piper (register factors, per-column LDS-DMA staging) with 2 column waves
    per stage: the block-wide T and factor hand-off rows are written by both
    column waves (each its [lo, hi) share); bitwise equal to the CPU twin on
    whole interiors, rect lists whose strips end mid-block, short chunks."""
    ny = 149
    T, iCp = rand((ny, nx), 101 + K), rand((ny, nx), 102, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    ref = cpu_ref(K, T, iCp, rects, "pipe")
    for chunk in (5, 41):
        assert torch.equal(gpu_run(K, T, iCp, rects, kern, chunk=chunk, cols=2), ref)
    sub = [(K + 3, nx - K - 7, K + 2, ny - K - 5), (1, K + 3, 1, ny - 1)]
    ref = cpu_ref(K, T, iCp, sub, "pipe")
    assert torch.equal(gpu_run(K, T, iCp, sub, kern, chunk=23, cols=2, xcd=0), ref)


def test_pipe_two_column_waves_need_vec4():
    """cols=2 on a tile that only allows 2 cells per lane runs the 1-column kernel."""
    ny, nx, K = 67, 518, 20
    T, iCp = rand((ny, nx), 13), rand((ny, nx), 14, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    assert torch.equal(gpu_run(K, T, iCp, rects, "pipe", cols=2), cpu_ref(K, T, iCp, rects, "pipe"))
    with pytest.raises(Exception):
        gpu_run(8, T, iCp, rects, "pipe", cols=2)  # instantiated for K = 16, 20, 24 only


@pytest.mark.parametrize("K,S", [(12, 3), (16, 8), (24, 8), (8, 4), (8, 1)])
def test_pipe_alternative_stage_splits(K, S):
    ny, nx = 257, 1028
    T, iCp = rand((ny, nx), 5), rand((ny, nx), 6, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    a = gpu_run(K, T, iCp, rects, "pipe", chunk=64)
    b = gpu_run(K, T, iCp, rects, "pipe", chunk=64, stages=S)
    assert torch.equal(a, b)
    assert torch.equal(a, cpu_ref(K, T, iCp, rects, "pipe"))


@pytest.mark.parametrize("K", [16, 20, 24])
def test_pipeb_lane_moves_by_bpermute_bitwise(K):
    ny, nx = 257, 1028
    T, iCp = rand((ny, nx), 18), rand((ny, nx), 19, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    assert torch.equal(gpu_run(K, T, iCp, rects, "pipeb", chunk=64),
                       cpu_ref(K, T, iCp, rects, "pipe"))


@pytest.mark.parametrize("K,old", [(8, "fast5"), (12, "fast5p2"), (16, "fast5p4"), (16, "fast5")])
def test_pipe_equals_fixed_k_fast5_kernels(K, old):
    ny, nx = 389, 2048
    T, iCp = rand((ny, nx), 7), rand((ny, nx), 8, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    vec = 4 if old.startswith("fast5p") else 2
    assert torch.equal(gpu_run(K, T, iCp, rects, "pipe", chunk=64),
                       gpu_run(K, T, iCp, rects, old, chunk=64, vec=vec))


@pytest.mark.parametrize("K", [3, 4, 6, 8])
def test_pipec_equals_canonical_kernel(K):
    ny, nx = 389, 2050
    T, iCp = rand((ny, nx), 9), rand((ny, nx), 10, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    assert torch.equal(gpu_run(K, T, iCp, rects, "pipec", chunk=64),
                       gpu_run(K, T, iCp, rects, "lds_dpp", chunk=64, vec=2))


def test_pipe_unaligned_view_and_tiny_tiles():
    base = rand(64 * 200 + 1, 11).to(DEV)
    T = base[1:].view(200, 64)  # 8-byte aligned only -> one cell per lane
    iCp = torch.ones((200, 64), dtype=torch.float64, device=DEV)
    for kernel in ("pipe", "pipec"):
        out = torch.zeros((200, 64), dtype=torch.float64, device=DEV)
        ops.stencilk_step(13, out, T, iCp, coef(), None, ops.StencilTuning(kernel=kernel))
        ref = cpu_ref(13, T.cpu(), iCp.cpu(), [ops.interior_rect(64, 200)], kernel, fill=0.0)
        assert torch.equal(out.cpu(), ref)
    for ny, nx in ((3, 3), (4, 5), (9, 260), (70, 4)):
        T, iCp = rand((ny, nx), 12), rand((ny, nx), 13, 0.5, 1.0)
        for K in (1, 7, 24):
            assert torch.equal(gpu_run(K, T, iCp, None, "pipe"),
                               cpu_ref(K, T, iCp, [ops.interior_rect(nx, ny)], "pipe"))


G = 4096
CANARY = -1.2345678901234567e300


@pytest.mark.parametrize("kernel,K,vec,nx", [(k, *c) for k in ("pipe", "pipec") for c in (
    (16, 4, 1024), (16, 2, 1026), (16, 4, 1027), (24, 4, 776), (20, 2, 514), (5, 4, 300))] + [
    ("piper", 24, 4, 776), ("piper", 20, 2, 514), ("piper", 17, 4, 1027), ("piper", 10, 4, 1024),
    ("piper", 14, 2, 1026)])
def test_pipe_guard_bands(kernel, K, vec, nx):
    """No write outside the output rects or the arrays (GPU ASan is not
    available on the pool): canaries around every array, untouched cells
    outside the rects compared bitwise."""
    ny = 197
    bufs, fields = [], []
    for seed in (14, 15, 16):
        b = torch.full((G + ny * nx + G,), CANARY, dtype=torch.float64, device=DEV)
        f = b[G:G + ny * nx].view(ny, nx)
        f.copy_(rand((ny, nx), seed, 0.5, 1.0))
        bufs.append(b)
        fields.append(f)
    T, iCp, out = fields
    before = out.clone()
    rects = [(K, nx - K, K, ny - K)]
    ops.stencilk_step(K, out, T, iCp, coef(), rects,
                      ops.StencilTuning(kernel=kernel, chunk_rows=29, vec=vec))
    torch.cuda.synchronize()
    for b in bufs:
        assert bool((b[:G] == CANARY).all()) and bool((b[-G:] == CANARY).all())
    mask = torch.ones((ny, nx), dtype=torch.bool, device=DEV)
    mask[K:ny - K, K:nx - K] = False
    assert torch.equal(out[mask], before[mask])


@pytest.mark.parametrize("K,nx", [(20, 1028), (24, 776), (16, 1500)])
def test_piper_two_column_waves_guard_bands(K, nx):
    """2-column piper: no write outside the output rect or the arrays."""
    ny = 197
    bufs, fields = [], []
    for seed in (17, 18, 19):
        b = torch.full((G + ny * nx + G,), CANARY, dtype=torch.float64, device=DEV)
        f = b[G:G + ny * nx].view(ny, nx)
        f.copy_(rand((ny, nx), seed, 0.5, 1.0))
        bufs.append(b)
        fields.append(f)
    T, iCp, out = fields
    before = out.clone()
    rects = [(K, nx - K, K, ny - K)]
    ops.stencilk_step(K, out, T, iCp, coef(), rects,
                      ops.StencilTuning(kernel="piper", chunk_rows=29, vec=4, cols=2))
    torch.cuda.synchronize()
    for b in bufs:
        assert bool((b[:G] == CANARY).all()) and bool((b[-G:] == CANARY).all())
    mask = torch.ones((ny, nx), dtype=torch.bool, device=DEV)
    mask[K:ny - K, K:nx - K] = False
    assert torch.equal(out[mask], before[mask])
    ref = cpu_ref(K, T.cpu(), iCp.cpu(), rects, "pipe")
    assert torch.equal(out.cpu()[~mask.cpu()], ref[~mask.cpu()])


def test_piper_tiny_tiles_and_short_chunks():
    """piper (register factors, LDS-DMA staging three rows ahead) where the
    prefetch runs past the last row, the tile is narrower than a strip, and
    chunks are shorter than the pipeline: clamped rows/columns, bitwise."""
    for ny, nx in ((9, 260), (70, 4), (41, 1028), (200, 64)):
        T, iCp = rand((ny, nx), 51), rand((ny, nx), 52, 0.5, 1.0)
        for K in (10, 17, 24):
            for chunk in (1, 5, 64):
                assert torch.equal(gpu_run(K, T, iCp, None, "piper", chunk=chunk),
                                   cpu_ref(K, T, iCp, [ops.interior_rect(nx, ny)], "pipe"))


def test_pipe_limits():
    T = rand((40, 300), 17).to(DEV)
    out = torch.empty_like(T)
    with pytest.raises(ValueError):
        ops.stencilk_step(25, out, T, T, coef(), None, ops.StencilTuning(kernel="pipe"))
    with pytest.raises(RuntimeError):  # no such stage split instantiated
        ops.stencilk_step(16, out, T, T, coef(), None, ops.StencilTuning(kernel="pipe", stages=5))
    assert native().pipe_max_k() == 24


def test_lab_kernels_fail_loudly_until_loaded():
    """The superseded / experimental K-step kernels live in librma_lab.so: in a
    fresh process that has not loaded it, asking the core for one is a loud
    error naming the library; after load_lab() the same launch runs."""
    import subprocess
    import sys

    code = r'''
import torch
from rocm_mpi_amd._native import native, load_lab, lab_loaded
from rocm_mpi_amd import ops
T = torch.rand(64, 256, dtype=torch.float64, device="cuda")
T2 = torch.zeros_like(T); iCp = torch.ones_like(T)
s = torch.cuda.current_stream().cuda_stream
args = (8, T2.data_ptr(), T.data_ptr(), iCp.data_ptr(), 256, 64, [(1, 255, 1, 63)],
        (-1.0, 10.0, 10.0, 1e-4), 16, 3, s, True, -1, 2, ops.kernel_id("fast5"), 0, 0)
assert not lab_loaded()
try:
    native().stencilk_rects(*args)
    raise SystemExit("no error")
except RuntimeError as e:
    assert "librma_lab.so" in str(e), str(e)
load_lab()
native().stencilk_rects(*args)
torch.cuda.synchronize()
print("OK")
'''
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr[-2000:]


@pytest.mark.parametrize("nx", [515, 520, 1285, 2050])
@pytest.mark.parametrize("K", [16, 17, 18, 19, 20])
def test_pipe_five_cells_per_lane_bitwise(nx, K):
    """5 cells per lane (320-column strips, v-major LDS rows, delayed factor
    ring, no-wrap immediate-offset path): bitwise equal to the CPU twin,
    also on rect lists whose strips end mid-window and on the x edges."""
    assert native().pipe_vec(K, 0, 0, nx, 5, True) == 5
    ny = 131
    T, iCp = rand((ny, nx), 21 + K), rand((ny, nx), 22, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    assert torch.equal(gpu_run(K, T, iCp, rects, "pipe", chunk=37, vec=5),
                       cpu_ref(K, T, iCp, rects, "pipe"))
    sub = [(K + 3, nx - K - 7, K + 2, ny - K - 5), (1, K + 3, 1, ny - 1)]
    assert torch.equal(gpu_run(K, T, iCp, sub, "pipe", chunk=23, vec=5, xcd=0),
                       cpu_ref(K, T, iCp, sub, "pipe"))


def test_pipe_five_cells_falls_back():
    """vec=5 where it does not apply (nx % 5 != 0, K outside 16..20, the
    canonical arithmetic) runs 4 / 2 / 1 cells per lane, still bitwise."""
    assert native().pipe_vec(20, 0, 0, 1028, 5, True) == 4
    assert native().pipe_vec(24, 0, 0, 1280, 5, True) == 4
    assert native().pipe_vec(20, 0, 1, 1280, 5, True) == 4
    assert native().pipe_vec(20, 0, 0, 1285, 5, False) == 5  # 8-B accesses only
    ny = 97
    for K, nx, kernel in ((20, 1028, "pipe"), (24, 1280, "pipe"), (20, 1280, "pipec")):
        T, iCp = rand((ny, nx), 23), rand((ny, nx), 24, 0.5, 1.0)
        rects = [ops.interior_rect(nx, ny)]
        assert torch.equal(gpu_run(K, T, iCp, rects, kernel, chunk=41, vec=5),
                           cpu_ref(K, T, iCp, rects, kernel))


@pytest.mark.parametrize("K,nx", [(20, 1285), (16, 520), (18, 2050)])
def test_pipe_five_cells_guard_bands(K, nx):
    ny = 197
    bufs, fields = [], []
    for seed in (25, 26, 27):
        b = torch.full((G + ny * nx + G,), CANARY, dtype=torch.float64, device=DEV)
        f = b[G:G + ny * nx].view(ny, nx)
        f.copy_(rand((ny, nx), seed, 0.5, 1.0))
        bufs.append(b)
        fields.append(f)
    T, iCp, out = fields
    before = out.clone()
    rects = [(K, nx - K, K, ny - K)]
    ops.stencilk_step(K, out, T, iCp, coef(), rects,
                      ops.StencilTuning(kernel="pipe", chunk_rows=29, vec=5))
    torch.cuda.synchronize()
    for b in bufs:
        assert bool((b[:G] == CANARY).all()) and bool((b[-G:] == CANARY).all())
    mask = torch.ones((ny, nx), dtype=torch.bool, device=DEV)
    mask[K:ny - K, K:nx - K] = False
    assert torch.equal(out[mask], before[mask])
    ref = cpu_ref(K, T.cpu(), iCp.cpu(), rects, "pipe")
    assert torch.equal(out.cpu()[~mask.cpu()], ref[~mask.cpu()])


@pytest.mark.parametrize("nx", [515, 518, 520, 1028])
@pytest.mark.parametrize("K", [10, 13, 16, 17, 20, 21, 24])
def test_piper_register_factors_bitwise(nx, K):
    """piper (factor rows in registers, shifted one level per row, one LDS
    hand-off row per stage boundary; at 2 and 4 cells per lane stage 0's T /
    1/Cp prefetch by LDS-DMA three rows ahead): bitwise equal to the CPU twin,
    also on rect lists and short chunks (1, 2 and 4 cells per lane)."""
    ny = 157
    T, iCp = rand((ny, nx), 31 + K), rand((ny, nx), 32, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    ref = cpu_ref(K, T, iCp, rects, "pipe")
    assert torch.equal(gpu_run(K, T, iCp, rects, "piper", chunk=43), ref)
    sub = [(K + 3, nx - K - 7, K + 2, ny - K - 5), (1, K + 3, 1, ny - 1)]
    assert torch.equal(gpu_run(K, T, iCp, sub, "piper", chunk=19, xcd=0),
                       cpu_ref(K, T, iCp, sub, "pipe"))


@pytest.mark.parametrize("kernel", ["piper6", "piper7"])
@pytest.mark.parametrize("nx", [515, 518, 1028])
@pytest.mark.parametrize("K", [20, 24])
def test_piper_split_form_bitwise(kernel, nx, K):
    """piper6 / piper7 (register factors, the split fast-math form for dx != dy:
    fma(g, fma(ry, fma(-2,c,U+D), fma(-2,c,L+R)), c), lab library): bitwise
    equal to their CPU twin (stencil6_rects_cpu), to each other, and within
    rounding of the 5-operation form."""
    ny = 157
    T, iCp = rand((ny, nx), 41 + K), rand((ny, nx), 42, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    ref = cpu_ref(K, T, iCp, rects, kernel)
    assert torch.equal(gpu_run(K, T, iCp, rects, kernel, chunk=43), ref)
    sub = [(K + 3, nx - K - 7, K + 2, ny - K - 5), (1, K + 3, 1, ny - 1)]
    assert torch.equal(gpu_run(K, T, iCp, sub, kernel, chunk=19, xcd=0),
                       cpu_ref(K, T, iCp, sub, kernel))
    f5 = cpu_ref(K, T, iCp, rects, "pipe")
    assert float((ref - f5).abs().max()) < 1e-13


@pytest.mark.parametrize("nx", [518, 1028])
@pytest.mark.parametrize("K", [17, 18, 19, 20])
def test_piper_unroll6_equals_unroll3(nx, K):
    """The core piper unrolls the row loop of its non-first stages by 6 at
    K = 17..20 (factor rows keep their registers across the back edge); the
    lab's piper_u3 is the round-3 unroll by 3: bitwise equal, and both equal
    the fast5 CPU twin."""
    ny = 203
    T, iCp = rand((ny, nx), 51 + K), rand((ny, nx), 52, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    ref = cpu_ref(K, T, iCp, rects, "pipe")
    for chunk in (7, 43):
        a = gpu_run(K, T, iCp, rects, "piper", chunk=chunk)
        b = gpu_run(K, T, iCp, rects, "piper_u3", chunk=chunk)
        assert torch.equal(a, ref) and torch.equal(b, ref)


@pytest.mark.parametrize("nx", [518, 1028])
@pytest.mark.parametrize("K", [20, 24])
def test_piper_iso_bitwise_and_refused_when_anisotropic(nx, K):
    """piper_iso (lab, kernel 17: the y-sum FMA by ry = 1 as an add) on an
    isotropic grid == piper == the fast5 CPU twin, bitwise; refused for
    ry != 1."""
    ny = 149
    T, iCp = rand((ny, nx), 61 + K), rand((ny, nx), 62, 0.5, 1.0)
    d = 0.039
    iso = ops.StencilCoef(-1.3, 1 / d, 1 / d, 0.00028)
    rects = [ops.interior_rect(nx, ny)]
    ref = torch.full_like(T, -5.0)
    ops.stencilk_step(K, ref, T, iCp, iso, rects, ops.StencilTuning(kernel="pipe"))
    for kern in ("piper", "piper_iso"):
        out = torch.full(T.shape, -5.0, dtype=torch.float64, device=DEV)
        ops.stencilk_step(K, out, T.to(DEV), iCp.to(DEV), iso, rects,
                          ops.StencilTuning(kernel=kern, xcd_remap=1, chunk_rows=37, vec=4))
        assert torch.equal(out.cpu(), ref), kern
    with pytest.raises(Exception, match="isotropic"):
        out = torch.zeros(T.shape, dtype=torch.float64, device=DEV)
        ops.stencilk_step(K, out, T.to(DEV), iCp.to(DEV), coef(), rects,
                          ops.StencilTuning(kernel="piper_iso", xcd_remap=1, chunk_rows=37, vec=4))


@pytest.mark.parametrize("nx", [518, 1028])
@pytest.mark.parametrize("K", [20, 24])
def test_piper_one_wave_per_simd_bitwise(nx, K):
    """piper_w1 (lab: one wave per SIMD, row loop unrolled by 6 at K = 20 and
    24) == the fast5 CPU twin, bitwise."""
    ny = 181
    T, iCp = rand((ny, nx), 71 + K), rand((ny, nx), 72, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    ref = cpu_ref(K, T, iCp, rects, "pipe")
    for chunk in (7, 43):
        assert torch.equal(gpu_run(K, T, iCp, rects, "piper_w1", chunk=chunk), ref)


@pytest.mark.parametrize("nx", [516, 1028])
@pytest.mark.parametrize("K", [20, 24])
def test_piper_masked_cone_bitwise(nx, K):
    """piper_mask (lab: lanes outside a level's valid cone skip the level under
    EXEC, the level's arithmetic in one asm statement) == the fast5 CPU twin,
    bitwise, on several rects (strip windows at both x edges of the array)."""
    ny = 167
    T, iCp = rand((ny, nx), 81 + K), rand((ny, nx), 82, 0.5, 1.0)
    for rects in ([ops.interior_rect(nx, ny)], [(1, nx // 2, 1, 100), (37, nx - 3, 100, ny - 1)]):
        ref = cpu_ref(K, T, iCp, rects, "pipe")
        for chunk in (7, 43):
            for kern in ("piper_mask", "piper_mask_ctl"):
                assert torch.equal(gpu_run(K, T, iCp, rects, kern, chunk=chunk), ref), kern


@pytest.mark.parametrize("K", [20, 24])
def test_piper_schedule_variants_bitwise(K):
    """piper_nosb (lab: no sched_barriers inside a level) == the fast5 CPU twin."""
    nx, ny = 1028, 149
    T, iCp = rand((ny, nx), 91 + K), rand((ny, nx), 92, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    ref = cpu_ref(K, T, iCp, rects, "pipe")
    for chunk in (11, 64):
        for kern in ("piper_nosb", "piper_rot", "piper_sp", "piper_sp2", "piper_prio",
                     "piper_prio_nr"):
            assert torch.equal(gpu_run(K, T, iCp, rects, kern, chunk=chunk), ref), kern


@pytest.mark.parametrize("K", [21, 24])
def test_piper_u6_spilling_bitwise(K):
    """piper_u6s (lab: unrolled by 6 at H = 6, with register spills) == the
    fast5 CPU twin."""
    nx, ny = 1028, 151
    T, iCp = rand((ny, nx), 95 + K, ), rand((ny, nx), 96, 0.5, 1.0)
    rects = [ops.interior_rect(nx, ny)]
    ref = cpu_ref(K, T, iCp, rects, "pipe")
    for chunk in (13, 64):
        assert torch.equal(gpu_run(K, T, iCp, rects, "piper_u6s", chunk=chunk), ref)
