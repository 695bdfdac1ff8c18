"""Host code of the native core under AddressSanitizer + UBSan.

GPU-side sanitizers are not available on the MI355X pool; the host parts
(topology and the C ABI grid description, CPU twins, pack/unpack, reductions,
the executor's pass geometry and planner, the halo exchange plan run for fake
ranks on host memory, parallel_for, validation) are compiled with
g++ -fsanitize=address,undefined and run here."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_selftest_asan_ubsan(tmp_path):
    exe = tmp_path / "host_selftest"
    srcs = [os.path.join(ROOT, "tests", "native", "host_selftest.cpp"),
            os.path.join(ROOT, "csrc", "runtime", "topology.cpp"),
            os.path.join(ROOT, "csrc", "runtime", "errors.cpp"),
            os.path.join(ROOT, "csrc", "runtime", "plan.cpp"),
            os.path.join(ROOT, "csrc", "runtime", "config.cpp"),
            os.path.join(ROOT, "csrc", "runtime", "halo_plan.cpp"),
            os.path.join(ROOT, "csrc", "kernels", "cpu_kernels.cpp")]
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-ffp-contract=off", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-I", os.path.join(ROOT, "csrc", "include"), *srcs, "-o", str(exe), "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ,
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host selftest OK" in r.stdout
