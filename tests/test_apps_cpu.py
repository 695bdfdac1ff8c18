"""Entry points, launcher, checkpoint/resume, PNG output, C ABI (CPU side)."""
import ctypes
import json
import os
import subprocess
import sys

import pytest
import torch

from helpers import ROOT
from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
from rocm_mpi_amd.utils import checkpoint, vis


def run(cmd, timeout=300, env=None):
    e = dict(os.environ)
    e.update(env or {})
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=e)


def test_app_ap_cpu_writes_png_and_reference_line(tmp_path):
    r = run([sys.executable, "-m", "rocm_mpi_amd.apps.diffusion_2D_ap", "--device", "cpu",
             "--nt", "60", "--outdir", str(tmp_path), "--json"])
    assert r.returncode == 0, r.stderr
    assert "Executed 60 steps in = " in r.stdout and "GB/s" in r.stdout
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["variant"] == "ap" and rec["timed_steps"] == 50
    png = tmp_path / "Temp_ap_1_128_128.png"
    data = png.read_bytes()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"


def test_launcher_runs_four_ranks_and_matches_oracle(tmp_path):
    r = run([sys.executable, "-m", "rocm_mpi_amd.launch", "-n", "4", "-m",
             "rocm_mpi_amd.apps.diffusion_2D_perf", "--", "--nx", "128", "--ny", "128",
             "--device", "cpu", "--transport", "gloo", "--vis", "--outdir", str(tmp_path)],
            timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "maximum(T_v) = 0.39786473026690" in r.stdout
    assert (tmp_path / "Temp_perf_4_254_254.png").exists()


def test_launcher_kills_job_when_a_rank_fails():
    code = "import os,sys,time; r=int(os.environ['RANK']); time.sleep(0.2 if r==1 else 30); sys.exit(3 if r==1 else 0)"
    script = os.path.join(ROOT, "build", "fail_rank.py")
    os.makedirs(os.path.dirname(script), exist_ok=True)
    open(script, "w").write(code)
    r = run([sys.executable, "-m", "rocm_mpi_amd.launch", "-n", "3", script], timeout=60)
    assert r.returncode == 3
    assert "terminating the job" in r.stderr


def test_presets_and_cli_flags():
    from rocm_mpi_amd.apps import cli

    p = cli.build_parser("perf_hide")
    a = p.parse_args([])
    assert (a.nx, a.ny, a.nt) == (12288, 12288, 100)  # perf_hide.jl:37-43
    a = cli.build_parser("perf_hide_prof").parse_args([])
    assert (a.nx, a.nt, a.profile) == (8192, 300, True)
    assert set(cli.PRESETS) == {"ap256_cpu", "kp16k", "perf_2x1", "hide_2x2", "hide_4x2_288GB"}


def test_preset_supplies_defaults_flags_win(capsys):
    from rocm_mpi_amd.apps import cli

    assert cli.run_variant("ap", ["--preset", "ap256_cpu", "--nt", "20", "--nx", "40", "--ny",
                                  "36", "--quiet", "--no-vis", "--json"]) == 0
    rec = json.loads([l for l in capsys.readouterr().out.splitlines() if l.startswith("{")][-1])
    assert (rec["variant"], rec["nx"], rec["ny"], rec["nt"], rec["device"]) == \
        ("ap", 40, 36, 20, "cpu")
    with pytest.raises(SystemExit):  # a perf preset on the kp entry point
        cli.run_variant("kp", ["--preset", "perf_2x1"])


def test_checkpoint_resume_is_bitwise(tmp_path):
    cfg = dict(variant="perf", nx=40, ny=30, nt=10, quiet=True, init="random", device="cpu")
    m = Diffusion2D(DiffusionConfig(**cfg))
    m.step(10)
    checkpoint.save_checkpoint(m, str(tmp_path / "ck"))
    m.step(7)
    want = m.field.clone()
    m.close()
    m2 = Diffusion2D(DiffusionConfig(**cfg))
    meta = checkpoint.load_checkpoint(m2, str(tmp_path / "ck"))
    assert meta["steps_done"] == 10 and m2.steps_done == 10
    m2.step(7)
    assert torch.equal(m2.field, want)
    m2.close()
    m3 = Diffusion2D(DiffusionConfig(**dict(cfg, nx=42)))
    with pytest.raises(ValueError):
        checkpoint.load_checkpoint(m3, str(tmp_path / "ck"))
    m3.close()


def test_vis_png_roundtrip(tmp_path):
    f = torch.linspace(0, 1, 50 * 80, dtype=torch.float64).reshape(50, 80)
    info = vis.heatmap_png(f, str(tmp_path / "a.png"))
    raw = (tmp_path / "a.png").read_bytes()
    assert raw[12:16] == b"IHDR"
    w, h = int.from_bytes(raw[16:20], "big"), int.from_bytes(raw[20:24], "big")
    assert h == 50 and w > 80
    assert info["min"] == 0.0 and info["max"] == 1.0


def test_visualise_subsamples_large_tiles(tmp_path):
    """Above max_pixels per side every rank subsamples before the gather; the
    printed maximum stays the exact maximum over the full interior."""
    m = Diffusion2D(DiffusionConfig(variant="perf", nx=130, ny=70, nt=3, quiet=True,
                                    device="cpu", init="random", outdir=str(tmp_path)))
    m.step(3)
    exact = float(m.field[1:-1, 1:-1].max())
    full = m.visualise()
    sub = m.visualise(max_pixels=40)
    m.close()
    assert full["stride"] == 1 and sub["stride"] == 4
    assert full["max"] == exact and sub["max"] == exact
    raw = (tmp_path / "Temp_perf_1_130_70.png").read_bytes()
    assert int.from_bytes(raw[20:24], "big") == 17  # ceil(68 / 4) rows


def test_nan_guard_raises():
    m = Diffusion2D(DiffusionConfig(variant="perf", nx=20, ny=20, nt=5, quiet=True, device="cpu",
                                    check_every=2))
    m.field[5, 5] = float("nan")
    with pytest.raises(FloatingPointError):
        m._advance(4)
    m.close()


def test_c_abi_topology_and_geometry():
    """The C ABI of librma_core.so (what the Julia shim calls), single rank."""
    lib = ctypes.CDLL(os.path.join(ROOT, "rocm_mpi_amd", "librma_core.so"))
    assert lib is not None
    lib.rma_nx_g.restype = ctypes.c_int64
    lib.rma_x_g.restype = ctypes.c_double
    lib.rma_x_g.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_int64]
    lib.rma_last_error.restype = ctypes.c_char_p
    # init needs a device (hipSetDevice); on a CPU-only host it must fail cleanly
    g = ctypes.c_void_p()
    me = ctypes.c_int()
    dims = (ctypes.c_int * 3)()
    coords = (ctypes.c_int * 3)()
    rc = lib.rma_init_global_grid(10, 8, 1, None, None, None, None, 1, 0, None, 0,
                                  ctypes.byref(g), ctypes.byref(me), dims, coords)
    if torch.cuda.is_available():
        assert rc == 0
        assert lib.rma_nx_g(g) == 10 and list(dims) == [1, 1, 1]
        assert lib.rma_x_g(g, 3, 0.5, 10) == 1.5
        assert lib.rma_finalize_global_grid(g) == 0
    else:
        assert rc != 0 and b"HIP" in lib.rma_last_error()


def test_runme_and_startup_scripts(tmp_path):
    """scripts/startup.sh (toolchain check, in-tree build, import) and
    scripts/runme.sh N VARIANT (setenv.sh, launcher, one process per rank) —
    the counterparts of the reference's startup.sh and scripts/runme.sh."""
    r = run(["bash", "scripts/startup.sh"], timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ENV setup done" in r.stdout and "native core" in r.stdout and ": OK" in r.stdout
    r = run(["bash", "scripts/runme.sh", "2", "kp", "--nx", "66", "--ny", "34", "--nt", "30",
             "--device", "cpu", "--transport", "gloo", "--outdir", str(tmp_path), "--json",
             "--no-vis"], timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    # the launcher prefixes every line with "[rank] "
    rec = json.loads([l.split("] ", 1)[1] for l in r.stdout.splitlines()
                      if l.startswith("[0] {")][-1])
    assert rec["variant"] == "kp" and rec["nprocs"] == 2 and rec["nxg"] == 2 * (66 - 2) + 2


def test_preset_runs_the_bench_plan_and_kernel():
    """The BASELINE presets and --bench-plan run what bench.py measures (K <= 24
    steps per pass, fast-math) on GPU-sized tiles: `--preset hide_2x2` and
    `bench.py --dims 2,2` resolve the same configuration, hence the same pass
    plan and kernel; small tiles keep one step per pass and --canonical opts
    out of fast-math. Without them the reference-named entry points keep the
    reference's one-step canonical update."""
    import bench
    from rocm_mpi_amd import ops
    from rocm_mpi_amd._native import native
    from rocm_mpi_amd.apps import cli

    cfg, _ = cli.resolve("perf_hide", ["--preset", "hide_2x2"])
    a = bench.parse(["--dims", "2,2", "--nx", "16384", "--gpus", "4"])
    bcfg = bench.make_config(a, 16384, 16384, "cpu", (2, 2, 0))
    keys = ("variant", "nx", "ny", "dims", "temporal", "fast_math", "chunk2", "vec")
    assert {k: getattr(cfg, k) for k in keys} == {k: getattr(bcfg, k) for k in keys}
    assert (cfg.temporal, cfg.fast_math) == (24, True)
    N = native()
    cells = float(cfg.nx) * cfg.ny
    for steps in (20, 1000):
        plans = [list(N.plan_passes(steps, N.default_pass_costs(c.temporal, c.fast_math, cells)))
                 for c in (cfg, bcfg)]
        assert plans[0] == plans[1] and sum(plans[0]) == steps
        coef = ops.StencilCoef.from_physics(1.0, 10 / 32674, 10 / 32674, (10 / 32674) ** 2 / 4.1)
        assert (N.fast_kernel_k(max(plans[0]), cfg.ny, tuple(coef))
                == N.fast_kernel_k(max(plans[1]), bcfg.ny, tuple(coef)))
    # the reference's own perf default (12288^2): its one-step canonical update
    cfg, _ = cli.resolve("perf", [])
    assert (cfg.nx, cfg.temporal, cfg.fast_math) == (12288, 1, False)
    cfg, _ = cli.resolve("perf", ["--bench-plan"])
    assert (cfg.nx, cfg.temporal, cfg.fast_math) == (12288, 24, True)
    cfg, _ = cli.resolve("perf", ["--bench-plan", "--canonical"])
    assert (cfg.temporal, cfg.fast_math) == (24, False)
    cfg, _ = cli.resolve("perf", ["--temporal", "1"])
    assert (cfg.temporal, cfg.fast_math) == (1, False)
    cfg, _ = cli.resolve("perf", ["--nx", "128", "--ny", "128"])  # below ~1.5M cells
    assert (cfg.temporal, cfg.fast_math) == (1, False)
    cfg, _ = cli.resolve("kp", ["--preset", "kp16k"])
    assert (cfg.temporal, cfg.fast_math) == (1, False)


def test_perf_entry_point_prints_its_plan(capsys):
    """The perf scripts print the pass plan and arithmetic next to the
    reference's T_eff line."""
    from rocm_mpi_amd.apps import cli

    assert cli.run_variant("perf_hide", ["--nx", "1300", "--ny", "1200", "--nt", "60",
                                         "--device", "cpu", "--no-vis", "--init", "random",
                                         "--bench-plan"]) == 0
    out = capsys.readouterr().out
    assert "Executed 60 steps in = " in out
    line = [l for l in out.splitlines() if l.startswith("[plan]")][-1]
    assert "50 timed steps" in line and "fast-math" in line and "24" in line


def test_perf_entry_point_keeps_the_reference_global_grid():
    """`diffusion_2D_perf --dims 2,1 --nx 12288` solves IGG's
    overlap-2 grid, nx_g = 2*(12288-2)+2 = 24574 (diffusion_2D_perf.jl:22,26,28),
    by default and with --temporal 1; the bench plan (overlap 2K = 48) differs
    and says so."""
    from rocm_mpi_amd.apps import cli

    for argv in (["--dims", "2,1"], ["--dims", "2,1", "--temporal", "1"]):
        cfg, _ = cli.resolve("perf", argv)
        assert (cfg.temporal, cfg.fast_math) == (1, False)
        run, ref = cli.global_sizes(cfg.nx, cfg.ny, cfg.dims, cfg.periods, 2, cfg.temporal)
        assert run == ref == (24574, 12288)
    cfg, _ = cli.resolve("perf", ["--dims", "2,1", "--bench-plan"])
    run, ref = cli.global_sizes(cfg.nx, cfg.ny, cfg.dims, cfg.periods, 2, cfg.temporal)
    assert cfg.temporal == 24 and run == (2 * (12288 - 48) + 48, 12288) and ref[0] == 24574


def test_bench_plan_on_multi_rank_grid_prints_the_changed_grid(capsys):
    """A K-step run on 2 ranks (loopback threads, CPU) prints both global grids
    and records the overlaps; the one-step default prints nothing of the kind."""
    from helpers import run_loopback
    from rocm_mpi_amd.apps import cli
    from rocm_mpi_amd.models import Diffusion2D
    from rocm_mpi_amd.parallel import implicit_grid as gg

    def rank(r, hub, argv):
        cfg, _ = cli.resolve("perf", argv)
        K = cfg.temporal
        gg.init_global_grid(cfg.nx, cfg.ny, 1, dimx=2, dimy=1, quiet=True, loopback=(hub, r),
                            device="cpu", overlaps=(2 * K if K > 1 else 2,) * 2 + (2,),
                            halowidths=(max(1, K),) * 2 + (1,))
        m = Diffusion2D(cfg)
        line = cli.grid_line(m)
        m.close()
        gg.finalize_global_grid()
        return line

    base = ["--nx", "40", "--ny", "30", "--dims", "2,1", "--device", "cpu"]
    assert run_loopback(2, rank, base) == [None, None]
    lines = run_loopback(2, rank, base + ["--temporal", "4", "--canonical"])
    assert lines[0] and "global grid 72x30 (overlap 8 for 4-step passes)" in lines[0]
    assert "overlap 2 gives 78x30" in lines[0]
