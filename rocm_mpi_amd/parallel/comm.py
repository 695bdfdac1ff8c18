"""Communicators: bootstrap, device selection, P2P groups, tiny collectives.

The reference's communication layer is MPI.jl over ROCm-aware OpenMPI/UCX or
plain OpenMPI (``scripts/setenv.sh:11-18``, ``README.md:25-35``), selected by
``IGG_ROCMAWARE_MPI``. Here one process drives one MI355X and the transports
are:

* ``rccl``     GPU-direct RCCL point-to-point over xGMI (native
  :class:`rocm_mpi_amd._C.RcclComm`); default whenever a GPU is present.
* ``staged``   host-staged: device planes are copied to pinned host memory and
  exchanged with torch.distributed/gloo (parity with ``IGG_ROCMAWARE_MPI=0``;
  validation only, never on the perf path).
* ``gloo``     CPU tensors over torch.distributed/gloo (CPU-only runs, CI).
* ``loopback`` N logical ranks as threads of ONE process exchanging through
  in-memory mailboxes (multi-rank tests without a
  cluster or a GPU).
* ``self``     a single rank (no communication).

Bootstrap is MPI-free: ``torch.distributed`` env:// rendezvous (RANK,
WORLD_SIZE, MASTER_ADDR, MASTER_PORT — torchrun or our launcher), its store
carries the RCCL unique id. The node-local rank (``MPI.Comm_split_type(
COMM_TYPE_SHARED)`` in ``scripts/rocmaware_test_selectdevice.jl:7-9``) comes
from LOCAL_RANK or, failing that, from a hostname exchange through the store.
"""
from __future__ import annotations

import os
import queue
import socket
import threading
import time
from dataclasses import dataclass
from typing import Sequence

import torch
import torch.distributed as dist

DEFAULT_TIMEOUT_S = float(os.environ.get("RMA_COMM_TIMEOUT", "300"))


@dataclass
class P2P:
    """One point-to-point operation of a group: send ``tensor`` to / receive it
    from ``peer``. ``tag`` disambiguates several messages between one pair."""

    kind: str  # "send" | "recv"
    tensor: torch.Tensor
    peer: int
    tag: int = 0


class Communicator:
    name = "abstract"
    rank: int = 0
    size: int = 1

    # --- collectives -----------------------------------------------------
    def barrier(self) -> None:
        raise NotImplementedError

    def allreduce(self, value: float, op: str = "sum") -> float:
        raise NotImplementedError

    def gather(self, t: torch.Tensor, root: int = 0) -> list[torch.Tensor] | None:
        """Every rank contributes ``t`` (same shape everywhere); root gets the
        list in rank order, others None."""
        raise NotImplementedError

    # --- point to point ---------------------------------------------------
    def exchange(self, ops: Sequence[P2P]) -> None:
        """Run all sends and receives as one group; returns when received data
        is usable in stream order (GPU) or in memory (CPU)."""
        raise NotImplementedError

    def sendrecv(self, send: torch.Tensor, dst: int, recv: torch.Tensor, src: int,
                 tag: int = 0) -> None:
        self.exchange([P2P("send", send, dst, tag), P2P("recv", recv, src, tag)])

    def supports(self, t: torch.Tensor) -> bool:
        return True

    def finalize(self) -> None:
        pass


class SelfComm(Communicator):
    name = "self"

    def barrier(self) -> None:
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()

    def allreduce(self, value: float, op: str = "sum") -> float:
        return float(value)

    def gather(self, t, root=0):
        return [t.clone()]

    def exchange(self, ops):
        sends = [o for o in ops if o.kind == "send"]
        recvs = [o for o in ops if o.kind == "recv"]
        for r in recvs:
            match = [s for s in sends if s.tag == r.tag]
            if not match:
                raise RuntimeError("self exchange: unmatched receive")
            s = match[0]
            sends.remove(s)
            r.tensor.copy_(s.tensor)


_REDUCE = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}


class TorchDistComm(Communicator):
    """torch.distributed (gloo) transport; GPU tensors are host-staged."""

    def __init__(self, staged: bool = False):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialized")
        self.rank = dist.get_rank()
        self.size = dist.get_world_size()
        self.staged = staged
        self.name = "staged" if staged else "gloo"
        self._pg = _gloo_group()

    def barrier(self) -> None:
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        dist.barrier(group=self._pg)

    def allreduce(self, value: float, op: str = "sum") -> float:
        t = torch.tensor([float(value)], dtype=torch.float64)
        dist.all_reduce(t, op=_REDUCE[op], group=self._pg)
        return float(t.item())

    def gather(self, t, root=0):
        host = t.detach().to("cpu").contiguous()
        lst = [torch.empty_like(host) for _ in range(self.size)] if self.rank == root else None
        dist.gather(host, lst, dst=root, group=self._pg)
        return lst

    def exchange(self, ops):
        if not ops:
            return
        staged = []
        p2p = []
        for o in ops:
            t = o.tensor
            if t.is_cuda:
                h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                if o.kind == "send":
                    h.copy_(t)
                staged.append((o, h))
                t = h
            fn = dist.isend if o.kind == "send" else dist.irecv
            p2p.append(dist.P2POp(fn, t, o.peer, group=self._pg, tag=o.tag))
        if any(o.tensor.is_cuda for o in ops):
            torch.cuda.current_stream().synchronize()  # D2H of send planes complete
        for w in dist.batch_isend_irecv(p2p):
            w.wait()
        for o, h in staged:
            if o.kind == "recv":
                o.tensor.copy_(h, non_blocking=False)


_gloo_pg = None


def _gloo_group():
    """A gloo group for host-side metadata even when the default PG is nccl."""
    global _gloo_pg
    if _gloo_pg is None:
        backend = dist.get_backend()
        _gloo_pg = dist.group.WORLD if "gloo" in str(backend) else dist.new_group(backend="gloo")
    return _gloo_pg


def shutdown_distributed(barrier: bool = True, timeout_s: float | None = None) -> None:
    """Destroy the default process group once every rank has reached teardown.

    Without the barrier a rank that finishes first closes its gloo pairs while
    a peer's last collective is still draining them; the peer's gloo thread
    then aborts the process ("terminate called without an active exception",
    seen at 4 and 8 ranks), turning a finished run into a failed one.

    The barrier is bounded (``RMA_TEARDOWN_TIMEOUT``, default 30 s): if a peer
    died or is stuck in another collective, the others give up waiting and
    destroy their group instead of blocking for the full communication
    timeout. Error paths pass ``barrier=False`` (or run inside an exception
    handler, detected here) and destroy directly.
    """
    global _gloo_pg
    if not dist.is_initialized():
        return
    import datetime
    import sys

    if timeout_s is None:
        timeout_s = float(os.environ.get("RMA_TEARDOWN_TIMEOUT", "30"))
    if sys.exc_info()[0] is not None:  # called from an error path (finally / except)
        barrier = False
    try:
        if barrier:
            # a CPU all-reduce is a barrier on the gloo side of a "cpu:gloo,cuda:nccl"
            # group (dist.barrier there would create a torch RCCL communicator)
            work = dist.all_reduce(torch.zeros(1), group=_gloo_group(), async_op=True)
            work.wait(timeout=datetime.timedelta(seconds=timeout_s))
    except Exception:  # noqa: BLE001 - a dead peer must not block teardown
        pass
    finally:
        dist.destroy_process_group()
        _gloo_pg = None


_rccl_generation = 0


def shared_gpu_rccl(rank: int, size: int) -> bool:
    """RMA_RCCL_SHARED_GPU=1: let RCCL ranks of ONE node share a GPU, for
    functional tests of the real multi-process RCCL path on a 1-GPU machine.

    RCCL refuses two ranks on one device ("Duplicate GPU detected") only when
    they report the same host; a per-rank NCCL_HOSTID makes each rank its own
    "host", so RCCL connects them with its network transport (sockets over
    NCCL_SOCKET_IFNAME, lo here) instead of xGMI P2P. Same communicator
    bootstrap, groups, send/recv matching and stream semantics as between
    GPUs; the wire is host memory. Never a performance path. Must run before
    the process's first RCCL call (RCCL reads the host id at init)."""
    if os.environ.get("RMA_RCCL_SHARED_GPU", "0") != "1" or size <= 1:
        return False
    os.environ.setdefault("NCCL_HOSTID", f"rma-shared-gpu-rank-{rank}")
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    return True


class RcclComm(Communicator):
    """GPU-direct RCCL communicator (native), bootstrapped through the store.

    Every rank creates its communicators in the same order, so a per-process
    generation counter gives all ranks the same store key for the unique id
    of the n-th communicator (re-initialising a grid never reads a stale id).
    """

    name = "rccl"

    def __init__(self, device: torch.device, timeout_s: float = DEFAULT_TIMEOUT_S,
                 store=None, rank: int | None = None, size: int | None = None,
                 key: str | None = None):
        from .._native import native

        global _rccl_generation
        if key is None:
            key = f"rma/rccl_uid/{_rccl_generation}"
            _rccl_generation += 1

        n = native()
        standalone = not dist.is_initialized()
        self.rank = (0 if standalone else dist.get_rank()) if rank is None else rank
        self.size = (1 if standalone else dist.get_world_size()) if size is None else size
        self.device = torch.device(device)
        self.timeout_s = timeout_s
        shared_gpu_rccl(self.rank, self.size)  # before this process's first RCCL call
        if self.size == 1 and store is None:
            uid = n.RcclComm.unique_id()  # single rank: nothing to distribute
        else:
            if store is None:
                store = dist.distributed_c10d._get_default_store()
            if self.rank == 0:
                uid = n.RcclComm.unique_id()
                store.set(key, uid)
            else:
                uid = store.get(key)
        n.set_rank_for_errors(self.rank)
        # non-blocking init + timeout unless RMA_RCCL_BLOCKING=1
        nb = os.environ.get("RMA_RCCL_BLOCKING", "0") != "1"
        self._c = n.RcclComm(self.size, self.rank, bytes(uid), self.device.index or 0,
                             init_timeout_s=timeout_s if nb else 0.0)
        self._scratch = torch.zeros(2, dtype=torch.float64, device=self.device)

    @property
    def native(self):
        return self._c

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def supports(self, t):
        return t.is_cuda

    def barrier(self) -> None:
        self._c.barrier(self._stream(), self.timeout_s)

    def wait(self) -> None:
        self._c.wait(self._stream(), self.timeout_s)

    def allreduce(self, value: float, op: str = "sum") -> float:
        from .._native import native

        n = native()
        self._scratch[0] = float(value)
        ptr = self._scratch.data_ptr()
        self._c.allreduce(ptr, ptr + 8, 1, n.DType.float64, getattr(n.RedOp, op), self._stream())
        self.wait()
        return float(self._scratch[1].item())

    def allreduce_tensor(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        from .._native import native

        n = native()
        if t.dtype != torch.float64 or not t.is_contiguous():
            raise TypeError("allreduce_tensor expects a contiguous float64 device tensor")
        self._c.allreduce(t.data_ptr(), t.data_ptr(), t.numel(), n.DType.float64,
                          getattr(n.RedOp, op), self._stream())
        return t

    def gather(self, t, root=0):
        src = t.detach().to(self.device).contiguous()
        nbytes = src.numel() * src.element_size()
        out = torch.empty((self.size,) + tuple(src.shape), dtype=src.dtype, device=self.device) \
            if self.rank == root else torch.empty(1, dtype=src.dtype, device=self.device)
        self._c.gather(src.data_ptr(), out.data_ptr(), nbytes, root, self._stream())
        self.wait()
        return list(out.unbind(0)) if self.rank == root else None

    def exchange(self, ops):
        if not ops:
            return
        s = self._stream()
        self._c.group_start()
        try:
            for o in ops:
                t = o.tensor
                if not t.is_cuda or not t.is_contiguous():
                    raise ValueError("rccl exchange needs contiguous device tensors")
                nb = t.numel() * t.element_size()
                if o.kind == "send":
                    self._c.send(t.data_ptr(), nb, o.peer, s)
                else:
                    self._c.recv(t.data_ptr(), nb, o.peer, s)
        finally:
            self._c.group_end()

    def finalize(self) -> None:
        if self._c is not None:
            try:
                self.wait()
            finally:
                self._c = None


_ipc_generation = 0


class IpcComm(TorchDistComm):
    """Device-direct halo transport between the processes of ONE node over HIP
    IPC (``csrc/include/rma/ipc.h``): every receiver owns a double-buffered
    device mailbox per sender, which the sender maps and fills with one
    device-to-device copy per message (over xGMI between GPUs, on-device when
    ranks share a GPU). Ordering (``RMA_IPC_MODE``): ``stream`` -- per-slot
    full/empty flags in POSIX shared memory that bounded one-wave flag
    kernels (``csrc/kernels/flags.hip``: system-scope acquire / release,
    timeout with an error word) wait on and write on the streams, nothing
    blocks the host (the default when every rank shares one GPU, the only
    case it has run on); ``host`` -- the host waits for its own copies and
    polls the peers' generation flags (the default across GPUs, see
    :meth:`_auto_mode`). The reference's intra-node
    ROCm-aware MPI path (``scripts/rocmaware_test_selectdevice.jl:16-22``) without
    MPI or RCCL. Collectives and gather stay on gloo (host-staged), as in
    ``staged``. ``peers``: the halo peers (Cartesian neighbours and diagonals).
    Mailbox size per slot: ``RMA_IPC_MAILBOX_MB`` (default 64 MiB).
    """

    def __init__(self, device: torch.device, peers, timeout_s: float = DEFAULT_TIMEOUT_S,
                 mailbox_mb: float | None = None, store=None, mode: str | None = None):
        super().__init__(staged=True)
        self.name = "ipc"
        from .._native import native

        global _ipc_generation
        key = f"rma/ipc/{_ipc_generation}"
        _ipc_generation += 1
        store = store if store is not None else dist.distributed_c10d._get_default_store()
        if self.rank == 0:
            import secrets

            store.set(f"{key}/token", f"{os.getpid():x}{secrets.token_hex(4)}")
        token = store.get(f"{key}/token").decode()
        mb = float(mailbox_mb if mailbox_mb is not None
                   else os.environ.get("RMA_IPC_MAILBOX_MB", "64"))
        cap = max(8, int(mb * (1 << 20)))
        self.device = torch.device(device)
        self.peers = sorted({int(p) for p in peers if int(p) >= 0})
        mode = mode or os.environ.get("RMA_IPC_MODE", "") or self._auto_mode()
        if mode not in ("stream", "host"):
            raise ValueError(f"IPC mode must be stream or host, got {mode!r}")
        self.mode = mode
        self._c = native().IpcTransport(self.rank, self.size, self.device.index or 0, self.peers,
                                        cap, token, timeout_s, 1 if mode == "stream" else 0)
        others = [p for p in self.peers if p != self.rank]
        for p in others:  # what p needs from me (my mailbox)
            store.set(f"{key}/{self.rank}/{p}", self._c.export_for(p))
        for p in others:  # p's shared-memory block exists: it published after creating it
            self._c.connect(p, store.get(f"{key}/{p}/{self.rank}"))
        # every peer has mapped every block: drop the names, so that nothing
        # stays in /dev/shm even if the job dies
        dist.barrier(group=self._pg)
        self._c.unlink_shm()

    def _auto_mode(self) -> str:
        """Stream mode (flag kernels, nothing blocks the host) is verified only
        with every rank on ONE GPU: whether a peer GPU's xGMI writes into this
        GPU's mailbox are visible to the copy-out under the flag kernels'
        system-scope acquire has not run on a multi-GPU node. So
        stream mode is the default only when every rank of the job shares one
        physical GPU; ranks on different GPUs default to host mode (the host
        waits on its own copies' events and polls the peers' generation flags,
        which needs no cross-GPU memory-scope argument). RMA_IPC_MODE overrides."""
        try:
            from .._native import native

            bus = native().device_pci_bus_id(self.device.index or 0)
        except Exception:  # noqa: BLE001 - unknown: the conservative mode
            bus = f"unknown-{self.rank}"
        buses: list = [None] * self.size
        dist.all_gather_object(buses, bus, group=self._pg)
        return "stream" if len(set(buses)) == 1 else "host"

    @property
    def native(self):
        return self._c

    def exchange(self, ops):
        """Device tensors to / from connected peers: device-to-device through
        the mailboxes, stream-ordered on the current stream; anything else
        host-staged over gloo."""
        if not ops:
            return
        if not all(o.tensor.is_cuda and o.tensor.is_contiguous() and o.peer in self.peers
                   for o in ops):
            return super().exchange(ops)
        s = torch.cuda.current_stream(self.device).cuda_stream
        self._c.group_start()
        try:
            for o in ops:
                t = o.tensor
                nb = t.numel() * t.element_size()
                if o.kind == "send":
                    self._c.send(t.data_ptr(), nb, o.peer, s)
                else:
                    self._c.recv(t.data_ptr(), nb, o.peer, s)
        finally:
            self._c.group_end()

    def finalize(self) -> None:
        if self._c is not None:
            import datetime

            # every peer reached teardown (so every group it owes me is
            # enqueued); a peer that died instead leaves my stream-mode waits
            # unsatisfiable: release them from the host before draining
            # long: a live peer may be late (rank 0 gathering, checkpointing),
            # and releasing the waits under it corrupts its receives
            tmo = max(float(os.environ.get("RMA_TEARDOWN_TIMEOUT", "30")), DEFAULT_TIMEOUT_S)
            aborted = None
            try:
                work = dist.barrier(group=self._pg, async_op=True)
                work.wait(timeout=datetime.timedelta(seconds=tmo))
            except Exception as e:  # noqa: BLE001 - a dead peer must not hang teardown
                aborted = e
                self._c.abort_waits()
            if torch.cuda.is_available() and torch.cuda.is_initialized():
                torch.cuda.synchronize(self.device)
            timed_out = None
            if not self._c.poisoned:
                try:
                    self._c.check_error()  # a stream-mode wait that gave up
                except RuntimeError as e:
                    timed_out = e
            # every rank is done with every mailbox before any rank unmaps its own
            try:
                work = dist.barrier(group=self._pg, async_op=True)
                work.wait(timeout=datetime.timedelta(seconds=tmo))
            except Exception:  # noqa: BLE001
                pass
            self._c = None
            if aborted is not None:
                # the released waits let pending receives copy stale mailbox
                # data: never a normal return
                raise RuntimeError(
                    f"IPC teardown (rank {self.rank}): the peers' barrier did not complete "
                    f"within {tmo:.0f} s ({type(aborted).__name__}: {aborted}); pending "
                    f"stream waits were released, received halos may be incomplete")
            if timed_out is not None:
                raise timed_out


# ---------------------------------------------------------------------------
# loopback: N logical ranks = N threads of one process
# ---------------------------------------------------------------------------
class LoopbackHub:
    """Shared mailboxes/barrier for :class:`LoopbackComm` ranks."""

    def __init__(self, size: int, timeout_s: float = 60.0):
        self.size = size
        self.timeout_s = timeout_s
        self._boxes: dict = {}
        self._lock = threading.Lock()
        self._barrier = threading.Barrier(size)
        self._slots: list = [None] * size
        self._native = None

    def native_hub(self):
        """Shared native hub for the device loopback transport (GPU halo path)."""
        with self._lock:
            if self._native is None:
                from .._native import native

                self._native = native().LoopbackHub(self.size, self.timeout_s)
            return self._native

    def box(self, src: int, dst: int, tag: int) -> queue.Queue:
        k = (src, dst, tag)
        with self._lock:
            q = self._boxes.get(k)
            if q is None:
                q = self._boxes[k] = queue.Queue()
            return q

    def collect(self, rank: int, value):
        """All ranks deposit a value; every rank gets the full list."""
        self._slots[rank] = value
        self._barrier.wait(self.timeout_s)
        out = list(self._slots)
        self._barrier.wait(self.timeout_s)
        return out


class LoopbackComm(Communicator):
    name = "loopback"

    def __init__(self, hub: LoopbackHub, rank: int):
        self.hub = hub
        self.rank = rank
        self.size = hub.size

    def barrier(self) -> None:
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        self.hub._barrier.wait(self.hub.timeout_s)

    def allreduce(self, value: float, op: str = "sum") -> float:
        vals = self.hub.collect(self.rank, float(value))
        return {"sum": sum, "max": max, "min": min}[op](vals)

    def gather(self, t, root=0):
        c = t.detach().clone()
        if c.is_cuda:
            # the root reads this copy from ITS thread and stream: the clone
            # (and the steps before it on this rank's stream) must have run
            # (without this the root intermittently read a rank's tile one
            # step stale in the loopback GPU tests)
            torch.cuda.current_stream(c.device).synchronize()
        vals = self.hub.collect(self.rank, c)
        return vals if self.rank == root else None

    def exchange(self, ops):
        cuda = bool(ops) and any(o.tensor.is_cuda for o in ops)
        sends = [(o, o.tensor.detach().clone()) for o in ops if o.kind == "send"]
        if cuda:
            # the send copies (and the producers before them) must have run
            # before a peer thread reads them on its own stream
            torch.cuda.current_stream().synchronize()
        for o, c in sends:
            self.hub.box(self.rank, o.peer, o.tag).put(c)
        for o in ops:
            if o.kind == "recv":
                try:
                    v = self.hub.box(o.peer, self.rank, o.tag).get(timeout=self.hub.timeout_s)
                except queue.Empty:
                    raise RuntimeError(
                        f"loopback rank {self.rank}: no message from {o.peer} tag {o.tag} "
                        f"within {self.hub.timeout_s}s") from None
                if v.is_cuda:
                    # the clone was allocated on the peer's stream and is read
                    # on this one: keep its block from the caching allocator
                    # until this stream's copy has run
                    v.record_stream(torch.cuda.current_stream(v.device))
                o.tensor.copy_(v)

    def finalize(self) -> None:
        """Teardown barrier (the reference brackets its device exchange with
        ``MPI.Barrier``, ``scripts/rocmaware_test_selectdevice.jl:20,24``):
        every rank's queued work has drained before ANY rank releases its halo
        buffers, streams and native endpoint, which peers' copies and event
        waits may still reference. A broken barrier (a peer already failed)
        does not mask that peer's error."""
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        try:
            self.hub._barrier.wait(self.hub.timeout_s)
        except threading.BrokenBarrierError:
            pass


# ---------------------------------------------------------------------------
# bootstrap helpers
# ---------------------------------------------------------------------------
def env_world() -> tuple[int, int, int | None]:
    """(rank, world_size, local_rank or None) from torchrun/SLURM/OpenMPI env."""
    def first(*names):
        for n in names:
            v = os.environ.get(n)
            if v not in (None, ""):
                return int(v)
        return None

    rank = first("RANK", "SLURM_PROCID", "OMPI_COMM_WORLD_RANK", "PMI_RANK")
    size = first("WORLD_SIZE", "SLURM_NTASKS", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE")
    local = first("LOCAL_RANK", "SLURM_LOCALID", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID")
    return (rank or 0), (size or 1), local


def init_distributed(backend: str | None = None, timeout_s: float = DEFAULT_TIMEOUT_S) -> None:
    """Initialise torch.distributed from the environment if needed (env://)."""
    if dist.is_initialized():
        return
    rank, size, _ = env_world()
    os.environ.setdefault("RANK", str(rank))
    os.environ.setdefault("WORLD_SIZE", str(size))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    import datetime

    if backend is None:
        backend = "cpu:gloo,cuda:nccl" if torch.cuda.is_available() else "gloo"
    dist.init_process_group(backend=backend, rank=rank, world_size=size,
                            timeout=datetime.timedelta(seconds=timeout_s))


def node_local_rank(comm_rank: int, comm_size: int) -> tuple[int, int]:
    """(local rank, ranks on this node). LOCAL_RANK if set, else a hostname
    exchange over the store (MPI.Comm_split_type(COMM_TYPE_SHARED) analogue)."""
    _, _, local = env_world()
    lsize = os.environ.get("LOCAL_WORLD_SIZE")
    if local is not None and lsize:
        return local, int(lsize)
    if comm_size == 1 or not dist.is_initialized():
        return (local or 0), 1
    from ..config import diag_value

    host = diag_value("hostname") or socket.gethostname()
    names: list = [None] * comm_size
    dist.all_gather_object(names, host, group=_gloo_group())
    same = [r for r, h in enumerate(names) if h == host]
    return same.index(comm_rank), len(same)


def visible_devices() -> int:
    """Number of visible GPUs. torch.cuda.device_count() goes through amdsmi on
    ROCm and was observed to return 0 from worker threads on the GPU box while
    the HIP runtime sees the device; fall back to the runtime's own count."""
    n = torch.cuda.device_count()
    if n <= 0 and torch.cuda.is_available():
        n = torch._C._cuda_getDeviceCount()
    return n


def shared_gpu_allowed() -> bool:
    """May several ranks of a node share one GPU? Only in the functional test
    modes: ``RMA_SHARED_GPU=1`` (multi-process tests and rehearsals on a
    1-GPU box) or ``RMA_RCCL_SHARED_GPU=1`` (which implies it)."""
    return (os.environ.get("RMA_SHARED_GPU", "0") == "1"
            or os.environ.get("RMA_RCCL_SHARED_GPU", "0") == "1")


def select_device(local_rank: int) -> torch.device:
    """One GPU per process: device = the node-local rank (the reference's
    ``AMDGPU.device!(rank_l+1)``, ``scripts/rocmaware_test_selectdevice.jl:9``).

    More local ranks than visible GPUs is an error (two ranks would silently
    share a device and every timing would be wrong), unless a shared-GPU test
    mode is on (:func:`shared_gpu_allowed`): then device = local_rank mod
    visible devices."""
    if not torch.cuda.is_available():
        return torch.device("cpu")
    n = visible_devices()
    if n <= 0:
        raise RuntimeError("torch reports a GPU but no visible device")
    if local_rank < 0:
        raise ValueError(f"local rank {local_rank} < 0")
    if local_rank >= n and not shared_gpu_allowed():
        raise RuntimeError(
            f"node-local rank {local_rank} but only {n} visible GPU(s): one process per GPU "
            f"(launch at most {n} ranks per node, or set RMA_SHARED_GPU=1 for a functional "
            f"test that shares a GPU)")
    dev = torch.device("cuda", local_rank % n)
    torch.cuda.set_device(dev)
    return dev


def wait_all(comm: Communicator) -> None:
    if isinstance(comm, RcclComm):
        comm.wait()
    elif torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


def now() -> float:
    return time.perf_counter()
