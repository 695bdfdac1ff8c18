"""The measurement tools behind profiles/: the planner's cost tables in
csrc/runtime/plan.cpp are exactly what scripts/fit_pass_costs.py derives from
the committed pass sweeps, and the overlap analysis of the committed kernel
traces (scripts/overlap_timeline.py) reproduces profiles/overlap_r2.md."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")


def load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "scripts", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("tile", [101376, 16384, 8192, 4096])
def test_planner_tables_come_from_the_committed_sweeps(tile):
    native = pytest.importorskip("rocm_mpi_amd._native").native
    try:
        N = native()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native core not built: {e}")
    fpc = load("fit_pass_costs")
    n, fast, can = fpc.tables(os.path.join(P, f"pass_sweep_{tile}_r2_final.json"))
    assert n == tile
    if tile == 101376:  # round 3: piper from K = 10, scaled by its measured ratios to pipe
        fast = fpc.apply_ratios(fast, fpc.piper_ratios(
            [os.path.join(P, q) for q in fpc.PIPER_SWEEPS_101376]), 10)
    # round 4: K = 17..20 scaled by the unroll-by-6 / unroll-by-3 ratios
    fast = fpc.apply_u6(fast, fpc.u6_ratios(os.path.join(P, fpc.U6_SWEEPS[tile])))
    # round 6: the K = 20 / K = 24 kernels under the iterative-ILP scheduler
    fast = fpc.apply_r6(fast, fpc.r6_ratios(tile, P))
    cells = float(tile) * tile
    got_f = list(N.default_pass_costs(24, True, cells))[1:]
    got_c = list(N.default_pass_costs(24, False, cells))[1:]
    assert got_f == pytest.approx(fast, abs=6e-4)
    assert got_c == pytest.approx(can, abs=6e-4)


def test_overlap_analysis_of_committed_traces(capsys):
    ot = load("overlap_timeline")
    tr = os.path.join(P, "traces_r2", "loopback2_k24_kernel_trace.csv")
    assert ot.main([tr, "--from-pass", "4"]) == 0
    out = capsys.readouterr().out
    first = out.splitlines()[0]
    frac = float(first.split("(")[-1].split("%")[0]) / 100
    assert frac > 0.9, first
    md = open(os.path.join(P, "overlap_r2.md")).read()
    assert first in md


def test_plan_app_predicts_the_measured_headline(capsys):
    """apps/plan.py: the planner's pass plan and predicted time for the driver's
    command on the 288 GB tile (one 20-step pass, ~70 ms: measured 68-71 ms), run by
    the register-factor pipelined kernel."""
    pytest.importorskip("rocm_mpi_amd._native")
    from rocm_mpi_amd.apps import plan as app

    try:
        d = app.describe(101376, 101376, 20)
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native core not built: {e}")
    assert d["passes"] == {20: 1} and d["kernels"][20]["kernel"] == "piper"
    assert 60.0 < d["pred_ms"] < 80.0
    c = app.describe(4096, 4096, 45, fast_math=False)
    assert sum(K * n for K, n in c["passes"].items()) == 45
    assert app.main(["--nx", "8192", "--steps", "100"]) == 0
    assert '"pred_teff_GBps"' in capsys.readouterr().out


def test_pipe_chunk_rows_by_tile_class():
    """Rows per task of the pipelined passes (csrc/runtime/plan.cpp), the
    measured best per tile class (profiles/chunk_sweep_r2.json)."""
    nat = pytest.importorskip("rocm_mpi_amd._native")
    try:
        N = nat.native()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native core not built: {e}")
    assert [N.pipe_chunk_rows(24, n) for n in (2048, 4096, 8192, 16384, 24576)] == \
        [48, 192, 256, 512, 768]
    assert N.pipe_chunk_rows(24, 101376) == 0 and N.pipe_chunk_rows(4, 512) == 0  # r1 rule
    assert N.pipe_chunk_rows(12, 4096, True) == 64 and N.pipe_chunk_rows(16, 8192, True) == 256
    # the executor's tuning uses them (fast and canonical pipelined kernels)
    coef = (-1.0, 10.0, 10.0, 1e-3)
    assert N.fast_kernel_k(24, 4096, coef)[2] == 192
    assert N.canonical_kernel_k(16, 8192)[2] == 256


def test_fast_kernel_choice_by_depth():
    """The executor's fast-math kernel per pass depth: the register-factor
    pipelined kernel ("piper", 12) from K = 14 (from K = 10 on tiles of >= 65536
    rows), at K = 24 its variant without in-level sched_barriers ("piper_nosb",
    22, round 6), the ring kernel ("pipe", 9) below; cells per lane as the kernel will run them (pipe_vec: 5 only for the
    lab's fast5 K = 16..20 on nx % 5 == 0, else 4 / 2 / 1 by alignment)."""
    nat = pytest.importorskip("rocm_mpi_amd._native")
    try:
        N = nat.native()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native core not built: {e}")
    coef = (-1.0, 10.0, 10.0, 1e-3)
    kern = {K: N.fast_kernel_k(K, 101376, coef)[0] for K in range(3, 25)}
    assert all(kern[K] == 12 for K in range(10, 24)) and kern[24] == 22, kern
    assert all(kern[K] == 9 for K in range(3, 10)), kern
    small = {K: N.fast_kernel_k(K, 16384, coef)[0] for K in range(3, 25)}
    assert all(small[K] == 12 for K in range(14, 24)) and small[24] == 22, small
    assert all(small[K] == 9 for K in range(3, 14)), small
    assert N.pipe_vec(20, 0, 0, 101120, 5, True) == 5
    assert N.pipe_vec(20, 0, 0, 101376, 5, True) == 4      # nx % 5 != 0
    assert N.pipe_vec(24, 0, 0, 101120, 5, True) == 4      # K > 20
    assert N.pipe_vec(20, 0, 3, 101120, 5, True) == 4      # piper: 4 cells
    assert N.pipe_vec(20, 0, 0, 1026, 4, True) == 2        # nx % 4 != 0
    assert N.pipe_vec(20, 0, 0, 1024, 4, False) == 1       # not 16-B aligned
