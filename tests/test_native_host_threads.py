"""The threaded native path under host sanitizers (VERDICT r4
next-step 2).

tests/native/threaded_selftest.cpp drives the real loopback transport
(csrc/runtime/loopback.cpp) and halo engine (csrc/runtime/halo.cpp) from
2..8 rank threads against a host stand-in of the HIP runtime
(tests/native/hip_stub): post / take / consume, plan-cache misses with pack
buffer reallocation (per-dimension, cross and merged groups), and endpoint
teardown while peers finish; and the HIP IPC transport (csrc/runtime/ipc.cpp)
between rank threads standing in for processes, in host and stream mode
(shared-memory flags, mailbox overflow of a later peer, bounded wait
timeout); and the executor's time loop on rank threads
(tests/native/executor_selftest.cpp, kernels as CPU twins, bitwise against
one rank). Built with clang's ThreadSanitizer (its runtime
intercepts pthread_cond_clockwait, which g++ 11's libtsan does not) and with
AddressSanitizer + UBSan.

The regression half rebuilds the same driver against the loopback transport
as it was before the fix (commit 5704426, round 4: events owned by the
endpoint) and requires both sanitizers to report the heap-use-after-free of
the receiver's "consumed" event -- the round-4 GPU-suite SIGSEGV.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
PRE_FIX = "5704426"
SRCS = ["tests/native/threaded_selftest.cpp", "csrc/runtime/loopback.cpp", "csrc/runtime/halo.cpp",
        "csrc/runtime/halo_plan.cpp", "csrc/runtime/topology.cpp", "csrc/runtime/errors.cpp",
        "csrc/runtime/ipc.cpp", "csrc/runtime/config.cpp", "csrc/kernels/cpu_kernels.cpp"]
# the executor's time loop (csrc/runtime/executor.cpp) with the kernels' CPU twins
EXEC_SRCS = ["tests/native/executor_selftest.cpp", "csrc/runtime/executor.cpp",
             "csrc/runtime/plan.cpp", "csrc/runtime/loopback.cpp", "csrc/runtime/halo.cpp",
             "csrc/runtime/halo_plan.cpp", "csrc/runtime/topology.cpp", "csrc/runtime/errors.cpp",
             "csrc/runtime/trace.cpp", "csrc/runtime/config.cpp", "csrc/kernels/cpu_kernels.cpp",
             "csrc/kernels/kernel_select.cpp"]
SAN = {"tsan": ["-fsanitize=thread"],
       "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]}
ENV = {"tsan": {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"},
       "asan": {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:verify_asan_link_order=0"}}

needs_clang = pytest.mark.skipif(not os.path.exists(CLANG), reason="needs ROCm's clang++")


def _build(kind, out, srcs, extra_inc=()):
    cmd = [CLANG, "-std=c++17", "-O1", "-g", "-ffp-contract=off", "-fno-omit-frame-pointer",
           *SAN[kind], "-I", os.path.join(ROOT, "tests", "native", "hip_stub"),
           *[a for d in extra_inc for a in ("-I", d)], "-I", os.path.join(ROOT, "csrc", "include"),
           *srcs, "-o", str(out), "-lpthread", "-ldl"]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]


def _run(kind, exe):
    return subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                          env=dict(os.environ, **ENV[kind]))


@needs_clang
@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_threaded_loopback_and_halo_clean(kind, tmp_path):
    exe = tmp_path / f"threaded_{kind}"
    _build(kind, exe, [os.path.join(ROOT, s) for s in SRCS])
    r = _run(kind, exe)
    assert r.returncode == 0, (r.stdout + r.stderr)[-6000:]
    assert "threaded selftest OK" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr


@needs_clang
@pytest.mark.skipif(shutil.which("git") is None, reason="needs git")
@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_pre_fix_loopback_teardown_race_is_reported(kind, tmp_path):
    """The same driver against the round-4 loopback.{h,cpp} must fail with the
    use-after-free of the event a destroyed endpoint recorded."""
    inc = tmp_path / "old" / "include"
    (inc / "rma").mkdir(parents=True)
    old_cpp = tmp_path / "old" / "loopback.cpp"
    for rev_path, dst in (("csrc/include/rma/loopback.h", inc / "rma" / "loopback.h"),
                          ("csrc/runtime/loopback.cpp", old_cpp)):
        r = subprocess.run(["git", "show", f"{PRE_FIX}:{rev_path}"], capture_output=True,
                           text=True, cwd=ROOT)
        if r.returncode != 0:
            pytest.skip(f"git history without {PRE_FIX}")
        dst.write_text(r.stdout)
    srcs = [os.path.join(ROOT, s) if s != "csrc/runtime/loopback.cpp" else str(old_cpp)
            for s in SRCS]
    exe = tmp_path / f"threaded_{kind}_prefix"
    _build(kind, exe, srcs, extra_inc=[str(inc)])
    r = _run(kind, exe)
    assert r.returncode != 0
    # the sanitizer's report, or -- when the stub's own liveness check on the
    # event reads the freed word first (timing) -- the stub's abort naming it
    if "heap-use-after-free" in r.stderr:
        assert "hipStreamWaitEvent" in r.stderr
        assert "LoopbackEndpoint::~LoopbackEndpoint" in r.stderr
    else:
        assert "hipStreamWaitEvent on a destroyed event" in r.stderr, r.stderr[-3000:]


@needs_clang
def test_ipc_slot_reuse_without_the_done_wait_is_reported(tmp_path):
    """Mutation check of the IPC half: with the sender's "receive done" wait
    removed (host mode reuses mailbox slot g % 2 before the peer's receive of
    g - 2 has copied it out), the build must fail: ThreadSanitizer reports the
    mailbox race, or -- when a sender two groups ahead overwrites the slot
    before the receiver copies it out -- the selftest's bitwise check of the
    received data fails first (which of the two comes first is timing)."""
    src = open(os.path.join(ROOT, "csrc", "runtime", "ipc.cpp")).read()
    needle = "} else if (g > 2) {  // slot g % 2"
    assert src.count(needle) == 1
    mut = tmp_path / "ipc.cpp"
    mut.write_text(src.replace(needle, "} else if (false && g > 2) {  // slot g % 2"))
    srcs = [os.path.join(ROOT, s) if s != "csrc/runtime/ipc.cpp" else str(mut) for s in SRCS]
    exe = tmp_path / "threaded_tsan_ipc_mut"
    _build("tsan", exe, srcs)
    r = _run("tsan", exe)
    assert r.returncode != 0
    race = "ThreadSanitizer: data race" in r.stderr and "IpcTransport::enqueue_group" in r.stderr
    corrupt = "ipc mode 0 rank" in r.stderr  # threaded_selftest.cpp ipc_ring's data check
    assert race or corrupt, r.stderr[-3000:]


@needs_clang
@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_executor_time_loop_on_rank_threads_clean_and_bitwise(kind, tmp_path):
    """tests/native/executor_selftest.cpp: DiffusionExecutor on 2-4 rank
    threads over the loopback transport (perf / perf_hide, canonical K = 1 and
    fast-math K = 4 / 8 / 24, open and periodic grids, split launches and the
    frame-first fused pass) == the same grid on one rank, bitwise, with the
    kernels as their CPU twins; clean under TSan and under ASan + UBSan (the
    process-wide stream pool's streams are kept for the process lifetime by
    design and suppressed by name)."""
    exe = tmp_path / f"executor_{kind}"
    _build(kind, exe, [os.path.join(ROOT, s) for s in EXEC_SRCS])
    r = _run(kind, exe)
    assert r.returncode == 0, (r.stdout + r.stderr)[-6000:]
    assert "executor selftest OK" in r.stdout
    assert "fused)" in r.stdout and "perf_hide K=24 2x2 auto OK" in r.stdout
    # direct-store halos between the rank threads (DiffusionExecutor::set_direct)
    for name in ("direct perf_hide K=8 2x2 open split OK", "direct perf_hide K=8 2x2 periodic fused OK",
                 "direct perf_hide K=24 3x1 periodic-x OK", "direct perf K=4 2x2 periodic-y OK",
                 "direct perf_hide K=6 1x1 periodic self OK"):
        assert name in r.stdout, name
    assert "WARNING: ThreadSanitizer" not in r.stderr
