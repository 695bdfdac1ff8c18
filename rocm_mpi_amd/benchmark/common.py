"""Shared plumbing of the headline benchmark (bench.py): logging, bounded
collectives over the gloo group, the failure protocol (every rank exits
non-zero, rank 0 still prints the record) and the per-phase watchdog."""
from __future__ import annotations

import datetime
import os
import sys
import threading

def log(rank: int, msg: str) -> None:
    print(f"bench.py rank {rank}: {msg}", file=sys.stderr, flush=True)


class CheckFailed(RuntimeError):
    """A correctness check failed (on this or another rank)."""


# ---------------------------------------------------------------------------
# bounded collectives over the gloo group (metadata only)
# ---------------------------------------------------------------------------
def gather_obj(obj, world: int):
    """All-gather a small picklable object over the gloo group (main phase:
    every rank reaches it; torchrun ends the job if one rank dies)."""
    if world == 1:
        return [obj]
    import torch.distributed as dist

    from rocm_mpi_amd.parallel import comm as C

    out: list = [None] * world
    dist.all_gather_object(out, obj, group=C._gloo_group())
    return out


def _wait(work, timeout_s: float, what: str) -> None:
    try:
        work.wait(timeout=datetime.timedelta(seconds=timeout_s))
    except Exception as e:  # noqa: BLE001 - a peer is gone or stuck
        raise CheckFailed(f"{what}: no answer from every rank within {timeout_s:.0f} s ({e})") \
            from None


def bounded_status(ok: bool, msg: str, world: int, timeout_s: float) -> list:
    """All-gather (ok, message) from every rank, bounded: every rank learns
    whether any rank failed and why, and nobody blocks longer than timeout_s."""
    if world == 1:
        return [(ok, msg)]
    import torch
    import torch.distributed as dist

    from rocm_mpi_amd.parallel import comm as C

    raw = msg.encode("utf-8", "replace")[:480]
    buf = torch.zeros(512, dtype=torch.uint8)
    buf[0] = 1 if ok else 0
    buf[1] = len(raw) >> 8
    buf[2] = len(raw) & 0xFF
    if raw:
        buf[3:3 + len(raw)] = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
    out = [torch.empty_like(buf) for _ in range(world)]
    _wait(dist.all_gather(out, buf, group=C._gloo_group(), async_op=True), timeout_s,
          "status exchange")
    res = []
    for b in out:
        n = (int(b[1]) << 8) | int(b[2])
        res.append((bool(b[0]), bytes(b[3:3 + n].tolist()).decode("utf-8", "replace")))
    return res


def agree(ok: bool, msg: str, world: int, timeout_s: float, what: str) -> None:
    """Raise CheckFailed on EVERY rank if any rank failed (bounded)."""
    st = bounded_status(ok, msg, world, timeout_s)
    bad = [(r, m) for r, (o, m) in enumerate(st) if not o]
    if bad:
        raise CheckFailed(f"{what} failed on rank(s) " +
                          "; ".join(f"{r}: {m}" for r, m in bad))


def bounded_gather_tiles(field, world: int, timeout_s: float):
    """The equal-shape tiles of every rank on rank 0 (host copies), bounded."""
    host = field.detach().cpu().contiguous()
    if world == 1:
        return [host]
    import torch
    import torch.distributed as dist

    from rocm_mpi_amd.parallel import comm as C

    lst = [torch.empty_like(host) for _ in range(world)] if dist.get_rank() == 0 else None
    _wait(dist.gather(host, lst, dst=0, group=C._gloo_group(), async_op=True), timeout_s,
          "tile gather")
    return lst


_DONE_KEY = "rma/bench/rank0_reported"


def signal_reported(world: int) -> None:
    """Rank 0 has printed its record (or is about to exit without one)."""
    if world > 1:
        try:
            import torch.distributed as dist

            dist.distributed_c10d._get_default_store().set(_DONE_KEY, "1")
        except Exception:  # noqa: BLE001 - best effort on an error path
            pass


def wait_reported(world: int, timeout_s: float) -> None:
    """A failing rank > 0 waits (bounded) for rank 0's record before it exits:
    torchrun ends the whole job as soon as one rank exits non-zero."""
    if world > 1:
        try:
            import torch.distributed as dist

            dist.distributed_c10d._get_default_store().wait(
                [_DONE_KEY], datetime.timedelta(seconds=timeout_s))
        except Exception:  # noqa: BLE001
            pass


class Watchdog:
    """Ends this rank if a phase outlives its deadline (a rank stuck inside
    the GPU runtime, RCCL or a gloo receive cannot be interrupted from
    Python): rank 0 first prints the record it has, with the failure, so the
    run still reports; the other ranks give it time to do so."""

    def __init__(self, rank: int, world: int, seconds: float, what: str, on_fire=None):
        self.rank, self.world, self.what, self.on_fire = rank, world, what, on_fire
        self._t = threading.Timer(seconds, self._fire)
        self._t.daemon = True
        self._t.start()

    def _fire(self) -> None:
        msg = f"watchdog: {self.what} did not finish in time"
        log(self.rank, msg + "; exiting")
        try:
            if self.rank == 0 and self.on_fire is not None:
                self.on_fire(msg)
        finally:
            finish_failed(self.rank, self.world, 6, 30.0)

    def cancel(self) -> None:
        self._t.cancel()


def finish_failed(rank: int, world: int, rc: int, wait_s: float) -> None:
    """Exit a failed run on this rank without touching the (possibly broken)
    process groups: rank 0 after its record, the others after rank 0's."""
    if rank == 0:
        signal_reported(world)
    else:
        wait_reported(world, wait_s)
    hard_exit(rank, rc)


def hard_exit(rank: int, rc: int) -> None:
    record_rc(rank, rc)
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(rc)


def record_rc(rank: int, rc: int) -> None:
    """RMA_DIAG bench_rc_dir=<dir>: every rank writes its exit status (tests)."""
    from rocm_mpi_amd.config import diag_value

    d = diag_value("bench_rc_dir")
    if d:  # atomically: torchrun may end this rank right after (a half-written file)
        # one temp file per thread: the check-phase watchdog thread and the main
        # thread can both be exiting the rank at once; with one shared temp
        # name one thread renamed the other's still-empty file into place
        tmp = os.path.join(d, f".rc{rank}.{threading.get_ident()}.tmp")
        with open(tmp, "w") as f:
            f.write(str(rc))
            f.flush()
        os.replace(tmp, os.path.join(d, f"rc{rank}"))
