"""GPU-direct point-to-point smoke test with node-local device selection.

Reference: scripts/rocmaware_test_selectdevice.jl:1-25 — MPI.Init, node-local
rank via Comm_split_type(COMM_TYPE_SHARED), AMDGPU.device!(rank_l+1), a
4-element Float64 device buffer filled with the rank, ring Sendrecv! on the
DEVICE buffers between barriers. Here: torch.distributed bootstrap, RCCL
send/recv on device tensors over xGMI (gloo on CPU-only hosts); ``--transport
ipc``: HIP IPC device-to-device copies between the processes of one node
(which also runs with every rank on one GPU, where RCCL refuses).

Fixes the reference quirk (:12-13) of computing ring neighbours from the
node-local rank modulo the GLOBAL size (only correct on one node): the ring
uses global ranks.

    python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 \
        -m rocm_mpi_amd.apps.rocmaware_test_selectdevice
"""
from __future__ import annotations

import argparse
import sys

import torch


def run(n: int = 4, transport: str = "auto", verbose: bool = True,
        self_ring: bool = False, info: dict | None = None) -> list[float]:
    """The ring exchange; returns what this rank received. ``self_ring``: with
    one rank, still send/recv through the transport (RCCL send/recv to itself
    on one GPU: the device-buffer P2P path without a second GPU). ``info``
    (optional dict) receives the transport and, for RCCL, the communicator's
    own rank count (ncclCommCount)."""
    from ..parallel import comm as C
    from ..parallel.implicit_grid import _choose_transport

    rank, size, _ = C.env_world()
    if size > 1:
        C.init_distributed()
    local, lsize = C.node_local_rank(rank, size)
    dev = C.select_device(local)
    t = _choose_transport(transport, size, dev, lsize)
    dst, src = (rank + 1) % size, (rank - 1) % size
    if t == "rccl":
        comm = C.RcclComm(dev)
        if info is not None:
            info["rccl_nranks"] = comm.native.count()
    elif t == "ipc":  # device-to-device between processes of one node, no RCCL
        comm = C.IpcComm(dev, [dst, src])
    elif t == "self":
        comm = C.SelfComm()
    else:
        comm = C.TorchDistComm(staged=(t == "staged"))
    if info is not None:
        info["transport"] = t
    if verbose:
        name = torch.cuda.get_device_name(dev) if dev.type == "cuda" else "cpu"
        print(f"rank={rank} local_rank={local}/{lsize} (device={dev} {name}), size={size}, "
              f"dst={dst}, src={src}, transport={t}", flush=True)
    send = torch.full((n,), float(rank), dtype=torch.float64, device=dev)
    recv = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
    comm.barrier()
    if rank == 0 and verbose:
        print("start sending...", flush=True)
    if size == 1 and not self_ring:
        recv.copy_(send)
    else:
        comm.sendrecv(send, dst, recv, src)
    comm.barrier()
    vals = recv.cpu().tolist()
    if verbose:
        print(f"recv_mesg on proc {rank}: {vals}", flush=True)
    comm.barrier()
    if rank == 0 and verbose:
        print("done.", flush=True)
    comm.finalize()
    return vals


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("-n", type=int, default=4)
    ap.add_argument("--transport", default="auto")
    ap.add_argument("--self-ring", action="store_true",
                    help="one rank: send/recv to itself through the transport")
    a = ap.parse_args(argv)
    from ..parallel import comm as C

    rank, size, _ = C.env_world()
    vals = run(a.n, a.transport, self_ring=a.self_ring)
    ok = all(v == float((rank - 1) % size) for v in vals)
    C.shutdown_distributed()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
