"""Probe: can two processes on ONE GPU form an RCCL communicator (send/recv)?
RCCL normally refuses duplicate GPUs; this checks what the bundled RCCL does.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        scripts/probe_rccl_shared_gpu.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rocm_mpi_amd.parallel import comm as C  # noqa: E402


def main() -> int:
    rank, size, _ = C.env_world()
    C.init_distributed("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    try:
        comm = C.RcclComm(dev)
    except Exception as e:  # noqa: BLE001
        print(f"rank {rank}: RCCL init failed: {type(e).__name__}: {str(e)[:300]}", flush=True)
        return 3
    send = torch.full((4,), float(rank), dtype=torch.float64, device=dev)
    recv = torch.full((4,), -1.0, dtype=torch.float64, device=dev)
    comm.sendrecv(send, (rank + 1) % size, recv, (rank - 1) % size)
    torch.cuda.synchronize()
    print(f"rank {rank}: received {recv.tolist()}", flush=True)
    comm.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
