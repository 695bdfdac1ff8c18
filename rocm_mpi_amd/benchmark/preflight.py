"""Preflight of a bench.py run, before the HBM-sized tile is allocated: the
reference smoke test's ring send/recv over the halo transport, a tiny halo
check, and which RCCL carries the traffic."""
from __future__ import annotations

import os
import re
import time

from .checks import halo_check
from .common import agree


def preflight(dims, K: int, dev: str, world: int, rank: int, gpu: bool, n: int,
              timeout_s: float, link_sizes: dict | None = None) -> dict:
    """Before the HBM-sized tile: the ring send/recv of the reference's smoke
    test over the halo transport, the halo check on a tiny grid, and (with
    ``link_sizes``) one timed exchange per halo neighbour at the timed tile's
    message sizes plus the transport RCCL chose for each connection."""
    from rocm_mpi_amd.apps import rocmaware_test_selectdevice as smoke

    t0 = time.perf_counter()
    err = ""
    transport = "rccl" if gpu and world == 1 else "auto"
    ring: dict = {}
    try:
        vals = smoke.run(4, transport=transport, verbose=False, self_ring=world == 1, info=ring)
        if any(v != float((rank - 1) % world) for v in vals):
            err = f"ring received {vals}, expected {(rank - 1) % world}"
    except Exception as e:  # noqa: BLE001
        err = f"ring send/recv: {type(e).__name__}: {e}"
    agree(not err, err, world, timeout_s, "preflight ring")
    info = {"ring_ok": True, "ring_ranks": world, "ring_transport": ring.get("transport"),
            "rccl_nranks": ring.get("rccl_nranks")}
    info["halo"] = halo_check(n, dims, K, dev, world, rank, timeout_s,
                              self_rccl=gpu and world == 1, inject=False)
    if link_sizes:
        info["links"] = links(dims, dev, world, rank, gpu, link_sizes, timeout_s)
    info["seconds"] = round(time.perf_counter() - t0, 3)
    return info


def links(dims, dev: str, world: int, rank: int, gpu: bool, sizes: dict,
          timeout_s: float) -> dict:
    """config.preflight.links: per rank, its Cartesian halo peers, one timed
    exchange per peer and message size (RCCL between GPUs, RCCL to itself on
    one GPU, gloo on the CPU driver), and the transport RCCL logged for each
    connection (NCCL_DEBUG_FILE, set by bench.py before the first RCCL call).
    verdict: 'p2p' (every connection GPU-direct), 'socket' / 'net' / 'shm' /
    'other' (a connection is not: never a scaling point), 'unknown' (no log)."""
    from rocm_mpi_amd.parallel import comm as C
    from rocm_mpi_amd.parallel.topology import CartTopology, dims_create

    from .common import gather_obj

    d = dims_create(world, [int(dims[0]), int(dims[1]), 1])
    topo = CartTopology(world, d, [0, 0, 0])
    peers = sorted({p for side in topo.neighbors(rank)[:2] for p in side if p >= 0})
    err, rows, conns, cls = "", [], {}, None
    comm = None
    try:
        halo_t = os.environ.get("RMA_TRANSPORT", "rccl")
        if gpu and (world == 1 or halo_t in ("rccl", "auto", "")):
            comm = C.RcclComm(dev)  # world 1: send/recv to itself over RCCL
            if world == 1:
                peers = [0]
        elif gpu and halo_t == "ipc":  # shared-GPU functional modes: their own transport
            comm = C.IpcComm(dev, peers)
        elif gpu:
            comm = C.TorchDistComm(staged=True)
        else:
            comm = C.TorchDistComm() if world > 1 else C.SelfComm()
        rows = link_probe(comm, peers if world > 1 or gpu else [], sizes, dev)
        if any(not r["data_ok"] for r in rows):
            err = "link probe received wrong data"
        logf = os.environ.get("NCCL_DEBUG_FILE", "")
        if gpu and logf and isinstance(comm, C.RcclComm):
            conns = parse_rccl_connections(read_own_rccl_log(logf), rank)
            cls = classify_links(conns, [p for p in peers if p != rank])
    except Exception as e:  # noqa: BLE001 - reported to every rank below
        err = f"{type(e).__name__}: {e}"
    finally:
        if comm is not None:
            try:
                comm.finalize()
            except Exception:  # noqa: BLE001
                pass
    agree(not err, err, world, timeout_s, "preflight links")
    mine = {"rank": rank, "peers": peers, "timed": rows,
            "rccl_connections": {str(k): v for k, v in conns.items()},
            "transport": ((cls or {}).get("verdict") or "unknown") if gpu else "gloo (CPU driver)",
            "transport_kinds": (cls or {}).get("kinds")}
    if gpu and world == 1:
        mine["transport"] = "self (RCCL send/recv to itself, one GPU)"
    elif gpu and not isinstance(comm, C.RcclComm):
        mine["transport"] = f"{os.environ.get('RMA_TRANSPORT')} (shared-GPU functional mode)"
    allr = gather_obj(mine, world)
    verdicts = {r["transport"] for r in allr}
    p2p = verdicts == {"p2p"} if gpu and world > 1 else None
    return {"ranks": allr, "sizes": sizes, "all_p2p": p2p,
            "note": ("one exchange (send + receive with the peer as one group) per halo peer "
                     "and message size, median of 5; GBps per direction; transport from "
                     "RCCL's own connection log")}


def _rccl_info() -> dict | None:
    """Which RCCL carries the halo traffic (RMA_RCCL_LIB may swap it)."""
    try:
        from rocm_mpi_amd._native import native

        return {"library": native().rccl_library(), "version": native().rccl_version()}
    except Exception:  # noqa: BLE001 - informational
        return None


def _rccl_nranks(g, pre: dict | None):
    """ncclCommCount of the halo communicator (or of the preflight ring's RCCL
    communicator on the single-GPU RCCL-self path); None without RCCL."""
    try:
        from rocm_mpi_amd.parallel.comm import RcclComm

        if isinstance(g.comm, RcclComm) and g.comm.native is not None:
            return int(g.comm.native.count())
    except Exception:  # noqa: BLE001 - informational
        return None
    return (pre or {}).get("rccl_nranks")


# --- per-link timing and RCCL transport -----------------
# RCCL / NCCL INFO connection lines, e.g.
#   host:123:456 [0] NCCL INFO Channel 00/1 : 0[0] -> 1[1] [send] via P2P/IPC/read
#   host:123:456 [1] NCCL INFO Channel 00/0 : 1[1] -> 0[0] [receive] via NET/Socket/0
#   host:123:456 [0] NCCL INFO Channel 01/0 : 0[3e000] -> 1[4e000] via P2P/IPC comm 0x55 nRanks 02
_CONN = re.compile(r"NCCL INFO Channel \d+/\d+ : (\d+)\[[^\]]*\] -> (\d+)\[[^\]]*\]"
                   r"(?: \[(send|receive)\])? via (\S+)")
# transports that move the bytes GPU to GPU without the host (xGMI on an
# MI355X node): P2P (IPC / direct pointer) and RCCL's own intra-process path
DIRECT = ("P2P",)


def rccl_debug_env(out_dir: str) -> dict:
    """The RCCL logging a bench run sets before its first RCCL call: INFO on
    the INIT / P2P / NET subsystems into one file per process (%h host, %p pid),
    never on stdout (rank 0's stdout carries the JSON record)."""
    return {"NCCL_DEBUG": "INFO", "NCCL_DEBUG_SUBSYS": "INIT,P2P,NET",
            "NCCL_DEBUG_FILE": os.path.join(out_dir, "rccl.%h.%p.log")}


def parse_rccl_connections(text: str, rank: int | None = None) -> dict:
    """{peer: sorted transports} of the connections RCCL logged (optionally
    only those of `rank`, as sender or receiver). A transport is the first
    component of the "via" field: P2P, SHM, NET/Socket, NET/IB, COLLNET..."""
    out: dict = {}
    for m in _CONN.finditer(text):
        a, b, _dir, via = int(m.group(1)), int(m.group(2)), m.group(3), m.group(4)
        if rank is not None and rank not in (a, b):
            continue
        peer = b if rank is None or a == rank else a
        parts = via.split("/")
        kind = parts[0] if parts[0] != "NET" else "/".join(parts[:2])
        out.setdefault(peer, set()).add(kind)
    return {p: sorted(v) for p, v in sorted(out.items())}


def classify_links(conns: dict, peers: list[int]) -> dict:
    """Summary over this rank's halo peers: 'p2p' if every peer connection
    RCCL logged is direct, 'socket' / 'net' / 'shm' if any is not, 'unknown'
    if a peer has no logged connection (logging off, or not yet connected)."""
    kinds = set()
    missing = [p for p in peers if p not in conns]
    for p in peers:
        kinds.update(conns.get(p, []))
    if missing or not kinds:
        verdict = "unknown"
    elif all(k in DIRECT for k in kinds):
        verdict = "p2p"
    elif "NET/Socket" in kinds:
        verdict = "socket"
    elif any(k.startswith("NET") for k in kinds):
        verdict = "net"
    elif "SHM" in kinds:
        verdict = "shm"
    else:
        verdict = "other"
    return {"verdict": verdict, "kinds": sorted(kinds), "peers_without_log": missing}


def read_own_rccl_log(pattern: str) -> str:
    """This process's RCCL log (NCCL_DEBUG_FILE with %h / %p substituted)."""
    import socket

    path = pattern.replace("%h", socket.gethostname()).replace("%p", str(os.getpid()))
    try:
        with open(path, errors="replace") as f:
            return f.read()
    except OSError:
        return ""


def link_probe(comm, peers: list[int], sizes: dict, dev: str, reps: int = 5) -> list[dict]:
    """Time one exchange (send to and receive from the peer as one group) per
    halo peer and message size, in the global edge order (each rank visits its
    peers in increasing rank: deadlock-free pairwise rendezvous). Median of
    `reps` timed exchanges after one warm-up; GB/s is per direction."""
    import statistics

    import torch

    from rocm_mpi_amd.parallel import comm as C

    out = []
    for p in sorted(set(q for q in peers if q >= 0)):
        for label, nbytes in sizes.items():
            n = max(1, int(nbytes) // 8)
            s = torch.full((n,), float(comm.rank), dtype=torch.float64, device=dev)
            r = torch.empty_like(s)
            ts = []
            for it in range(reps + 1):
                C.wait_all(comm)
                t0 = time.perf_counter()
                comm.sendrecv(s, p, r, p)
                C.wait_all(comm)
                if it:
                    ts.append(time.perf_counter() - t0)
            ok = bool((r == float(p)).all())
            t = statistics.median(ts)
            out.append({"peer": p, "message": label, "bytes": n * 8, "us": round(t * 1e6, 2),
                        "GBps": round(n * 8 / t / 1e9, 3), "data_ok": ok})
            del s, r
    return out
