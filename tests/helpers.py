"""Multi-rank test drivers: loopback threads and real processes over gloo."""
import os
import socket
import sys
import threading
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_loopback(n, fn, *args, timeout=120, **kw):
    """Run fn(rank, hub, *args) on n threads sharing one LoopbackHub."""
    from rocm_mpi_amd.parallel.comm import LoopbackHub

    try:
        from conftest import breadcrumb
    except ImportError:  # helpers used outside pytest
        def breadcrumb(msg):
            pass
    # logged before any rank thread starts: a native crash inside the threads
    # still names the case (seed-derived arguments included)
    breadcrumb(f"run_loopback n={n} fn={getattr(fn, '__name__', fn)} args={args!r} kw={kw!r}")
    hub = LoopbackHub(n, timeout_s=timeout)
    out = [None] * n
    err = []

    def body(r):
        try:
            out[r] = fn(r, hub, *args, **kw)
        except BaseException as e:  # noqa: BLE001
            err.append((r, e, traceback.format_exc()))
            hub._barrier.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout + 60)
    if err:
        r, e, tb = err[0]
        raise AssertionError(f"rank {r} failed: {e}\n{tb}")
    return out


def _proc_entry(rank, world, port, target, args, env):
    os.environ.update(env)
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import importlib

    mod, fn = target.rsplit(":", 1)
    getattr(importlib.import_module(mod), fn)(rank, world, *args)


def run_procs(world, target, *args, env=None, timeout=300):
    """Spawn `world` processes running module:function(rank, world, *args)."""
    import torch.multiprocessing as mp

    env = dict(env or {})
    env.setdefault("RMA_TRANSPORT", "gloo")
    env.setdefault("RMA_AUTOBUILD", "0")
    ctx = mp.get_context("spawn")
    port = free_port()
    procs = [ctx.Process(target=_proc_entry, args=(r, world, port, target, args, env))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout)
    bad = [(i, p.exitcode) for i, p in enumerate(procs) if p.exitcode != 0]
    for p in procs:
        if p.is_alive():
            p.kill()
    if bad:
        raise AssertionError(f"ranks failed (rank, exitcode): {bad}")
