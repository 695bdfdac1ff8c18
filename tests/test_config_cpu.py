"""One configuration surface: documented tuning
variables validated where they are read, and every diagnostic in ONE variable,
RMA_DIAG, parsed identically by the Python side (rocm_mpi_amd/config.py) and
the native core (csrc/runtime/config.cpp)."""
import pytest

from rocm_mpi_amd import config
from rocm_mpi_amd._native import native


def test_diag_parsing_python(monkeypatch):
    monkeypatch.setenv("RMA_DIAG", "no_lag,exec_streams=hifirst,pass_costs=20:1.9/24:2.2")
    assert config.diag_flag("no_lag") and not config.diag_flag("no_prime")
    assert config.diag_value("exec_streams") == "hifirst"
    assert config.diag_value("pass_costs") == "20:1.9/24:2.2"
    assert config.diag_value("frame_bands", "x") == "x"
    monkeypatch.setenv("RMA_DIAG", "no_lag=0")
    assert not config.diag_flag("no_lag")
    monkeypatch.setenv("RMA_DIAG", "no_such_key")
    with pytest.raises(ValueError, match="unknown key 'no_such_key'"):
        config.diag_flag("no_lag")


def test_diag_with_merges():
    s = config.diag_with("no_lag,hostname=a", hostname="b", bench_check_corrupt=True)
    assert config.diag_entries(s) == {"no_lag": "1", "hostname": "b", "bench_check_corrupt": "1"}
    assert config.diag_entries(config.diag_with(s, no_lag=None)) == {
        "hostname": "b", "bench_check_corrupt": "1"}
    with pytest.raises(ValueError):
        config.diag_with("", nope=1)


def test_diag_parsing_native_agrees(monkeypatch):
    n = native()
    monkeypatch.setenv("RMA_DIAG", "frame_bands=ol,no_halo_batch")
    assert n.diag_string() == "frame_bands=ol,no_halo_batch"
    assert n.diag_value("frame_bands") == "ol" and n.diag_value("no_halo_batch") == "1"
    assert n.diag_value("frame_sides") == ""
    monkeypatch.setenv("RMA_DIAG", "frame_bands=ol,bogus=1")
    with pytest.raises(Exception, match="RMA_DIAG: unknown key"):
        n.diag_string()


def test_tuning_variables_are_validated(monkeypatch):
    n = native()
    monkeypatch.delenv("RMA_EXEC_FUSED_TIMEOUT", raising=False)
    assert n.env_double("RMA_EXEC_FUSED_TIMEOUT", 60.0, 1e-9, 1e6) == 60.0
    monkeypatch.setenv("RMA_EXEC_FUSED_TIMEOUT", "2.5")
    assert n.env_double("RMA_EXEC_FUSED_TIMEOUT", 60.0, 1e-9, 1e6) == 2.5
    for bad in ("0", "-1", "abc", "1e7", "nan", "3s"):
        monkeypatch.setenv("RMA_EXEC_FUSED_TIMEOUT", bad)
        with pytest.raises(Exception, match="RMA_EXEC_FUSED_TIMEOUT: bad value"):
            n.env_double("RMA_EXEC_FUSED_TIMEOUT", 60.0, 1e-9, 1e6)
    monkeypatch.setenv("RMA_EXEC_FUSED", "1")
    assert n.env_choice("RMA_EXEC_FUSED", "auto|0|1", "auto") == "1"
    monkeypatch.setenv("RMA_EXEC_FUSED", "yes")
    with pytest.raises(Exception, match="RMA_EXEC_FUSED: bad value"):
        n.env_choice("RMA_EXEC_FUSED", "auto|0|1", "auto")
