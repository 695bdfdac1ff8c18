"""Local launcher: N ranks on one node, one process per GPU (``srun -n N`` analogue).

The reference launches with ``srun -n 4 --mpi=pmix ./runme.sh`` (README.md:18).
This spawns N child processes with the torch.distributed env contract
(RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1,
MASTER_PORT), prefixes their output with the rank, and — failure detection —
terminates the whole job as soon as one rank exits non-zero (a dead rank can
otherwise leave its peers blocked in a halo exchange).

    python -m rocm_mpi_amd.launch -n 4 -m rocm_mpi_amd.apps.diffusion_2D_perf -- --nx 16384
    python -m rocm_mpi_amd.launch -n 2 path/to/script.py arg1 arg2

``torchrun --nproc-per-node N --master-addr 127.0.0.1 ...`` works just as well.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import threading
import time


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(nprocs: int, cmd: list[str], env: dict | None = None, timeout: float | None = None,
           prefix: bool = True) -> int:
    port = int(os.environ.get("MASTER_PORT", 0)) or _free_port()
    base = dict(os.environ)
    base.update(env or {})
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = []
    for r in range(nprocs):
        e = dict(base)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nprocs),
                  "LOCAL_WORLD_SIZE": str(nprocs), "MASTER_ADDR": "127.0.0.1",
                  "MASTER_PORT": str(port)})
        procs.append(subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True,
                                      start_new_session=True))

    def pump(r, p):
        for line in p.stdout:
            sys.stdout.write(f"[{r}] {line}" if prefix else line)
            sys.stdout.flush()

    threads = [threading.Thread(target=pump, args=(r, p), daemon=True) for r, p in enumerate(procs)]
    for t in threads:
        t.start()
    t0 = time.time()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                sys.stderr.write(f"[launch] a rank exited with code {rc}; terminating the job\n")
                break
            if all(c == 0 for c in codes):
                break
            if timeout and time.time() - t0 > timeout:
                rc = 124
                sys.stderr.write("[launch] timeout; terminating the job\n")
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        deadline = time.time() + 10
        for p in procs:
            try:
                p.wait(max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
        for t in threads:
            t.join(1)
    return rc


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("-n", "--nprocs", type=int, required=True)
    ap.add_argument("-m", "--module", help="run `python -m MODULE`")
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("--no-prefix", action="store_true")
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    rest = [x for x in a.rest if x != "--"] if a.rest[:1] == ["--"] else list(a.rest)
    if a.module:
        cmd = [sys.executable, "-m", a.module, *rest]
    elif rest and rest[0].endswith(".py"):
        cmd = [sys.executable, *rest]
    elif rest:  # a native executable (e.g. build/examples/diffusion_2D_perf_hide)
        cmd = list(rest)
    else:
        ap.error("give -m MODULE or a script")
    return launch(a.nprocs, cmd, timeout=a.timeout, prefix=not a.no_prefix)


if __name__ == "__main__":
    sys.exit(main())
