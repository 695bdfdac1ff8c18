"""Host cost of one RCCL send/recv group (the halo exchange's per-dimension
group) on one GPU, RCCL send/recv to self:

* idle: the GPU has no other work;
* busy_other: a long kernel runs on another stream (perf_hide: the exchange
  on the high-priority stream while the interior runs);
* busy_same: the long kernel is ahead of the group on the same stream (perf).

If the enqueue cost depends on the GPU being busy, RCCL is waiting on the
device inside ncclGroupEnd; if not, it is pure host work.

    python bench/rccl_enqueue_probe.py --mb 3 --groups 50 --out gpurun_out/enq.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rocm_mpi_amd import ops  # noqa: E402
from rocm_mpi_amd.parallel import comm as C  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--mb", type=float, default=3.0, help="message size per send (MB)")
    ap.add_argument("--msgs", type=int, default=2, help="sends (and receives) per group")
    ap.add_argument("--groups", type=int, default=50)
    ap.add_argument("--busy-n", type=int, default=16384, help="tile of the busy kernel")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = C.RcclComm(dev)
    n = int(a.mb * 1e6 / 8)
    send = [torch.ones(n, dtype=torch.float64, device=dev) for _ in range(a.msgs)]
    recv = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(a.msgs)]
    nb = a.busy_n
    T = torch.rand((nb, nb), dtype=torch.float64, device=dev)
    T2 = torch.empty_like(T)
    iCp = torch.ones_like(T)
    coef = ops.StencilCoef(-1.0, 1.0, 1.0, 1e-3)

    def busy(stream):
        with torch.cuda.stream(stream):
            for _ in range(40):  # ~40 one-step kernels, tens of ms
                ops.stencil_step(T2, T, iCp, coef)

    def group(stream):
        c = comm.native
        s = stream.cuda_stream
        c.group_start()
        for i in range(a.msgs):
            c.send(send[i].data_ptr(), n * 8, 0, s)
            c.recv(recv[i].data_ptr(), n * 8, 0, s)
        c.group_end()

    main_s = torch.cuda.Stream(dev)
    other = torch.cuda.Stream(dev)
    res = {"mb": a.mb, "msgs_per_group": a.msgs, "env": {k: v for k, v in os.environ.items()
                                                       if k.startswith(("NCCL_", "RCCL_"))}}
    for mode in ("idle", "busy_other", "busy_same", "idle"):
        group(main_s)  # warm (connections)
        torch.cuda.synchronize()
        if mode == "busy_other":
            busy(other)
        elif mode == "busy_same":
            busy(main_s)
        ts = []
        for _ in range(a.groups):
            t0 = time.perf_counter()
            group(main_s)
            ts.append(time.perf_counter() - t0)
        t_enq = time.perf_counter()
        torch.cuda.synchronize()
        drain = time.perf_counter() - t_enq
        ts.sort()
        key = mode if mode not in res else mode + "_again"
        res[key] = {"median_us": round(ts[len(ts) // 2] * 1e6, 1),
                    "min_us": round(ts[0] * 1e6, 1), "max_us": round(ts[-1] * 1e6, 1),
                    "drain_after_enqueue_ms": round(drain * 1e3, 2)}
        print(key, json.dumps(res[key]), flush=True)
    comm.finalize()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
