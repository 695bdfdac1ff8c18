"""Single-GPU native executor (perf / perf_hide / kp, optional hipGraph) vs the
CPU reference loop: bitwise equal fields after many steps, including periodic
boundaries (self halo exchange on the device)."""
import pytest
import torch

from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig

pytestmark = pytest.mark.gpu


def run(variant, device, steps=37, **kw):
    cfg = DiffusionConfig(variant=variant, nx=kw.pop("nx", 301), ny=kw.pop("ny", 203), nt=steps,
                          device=device, quiet=True, init="random", **kw)
    m = Diffusion2D(cfg)
    if device != "cpu":
        assert m.executor is not None, "GPU run must use the native executor"
    m.step(steps)
    f = m.field.detach().cpu().clone()
    m.close()
    return f


@pytest.mark.parametrize("variant", ["perf", "perf_hide", "kp"])
@pytest.mark.parametrize("periods", [(0, 0, 0), (1, 1, 0), (1, 0, 0)])
def test_executor_matches_cpu(variant, periods):
    kw = dict(periods=periods, b_width=(7, 3))
    assert torch.equal(run(variant, "cuda:0", **kw), run(variant, "cpu", **kw))


@pytest.mark.parametrize("variant", ["perf", "perf_hide"])
def test_graph_replay_matches_eager(variant):
    a = run(variant, "cuda:0", steps=45, use_graph=True, graph_steps=10, nx=1030, ny=517)
    b = run(variant, "cuda:0", steps=45, nx=1030, ny=517)
    assert torch.equal(a, b)


def test_variants_agree_on_gpu():
    ref = run("perf", "cuda:0", nx=514, ny=260)
    for v in ("perf_hide", "kp"):
        assert torch.equal(run(v, "cuda:0", nx=514, ny=260), ref)


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("periods", [(0, 0, 0), (1, 1, 0)])
def test_ap_on_gpu_matches_cpu(graph, periods):
    """ap as torch ops on the GPU (eager, or replayed from a captured hipGraph in
    blocks of 7 steps + an eager remainder) == the CPU run, bitwise."""
    g = Diffusion2D(DiffusionConfig(variant="ap", nx=130, ny=131, nt=25, device="cuda:0",
                                    quiet=True, init="random", use_graph=graph, graph_steps=7,
                                    periods=periods))
    assert g.use_graph == graph
    g.step(11)
    g.step(14)
    assert g.steps_done == 25
    fg = g.field.cpu().clone()
    g.close()
    c = Diffusion2D(DiffusionConfig(variant="ap", nx=130, ny=131, nt=25, device="cpu",
                                    quiet=True, init="random", periods=periods))
    c.step(25)
    fc = c.field.clone()
    c.close()
    assert torch.equal(fg, fc)


def test_reference_protocol_run():
    m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=1024, ny=1024, nt=30, warmup=10,
                                    device="cuda:0", quiet=True))
    res = m.run()
    assert res.timed_steps == 20 and res.teff > 0
    assert torch.isfinite(m.field).all()
    m.close()
