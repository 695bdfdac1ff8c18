"""2D heat diffusion (explicit Euler, 5-point stencil, fp64) — all variants.

Physics and numerics are those of the reference scripts
(``scripts/diffusion_2D_{ap,kp,perf,perf_hide,perf_hide_prof}.jl``):
``lx=ly=10, lam=1, Cp0=1``, ``dx=lx/nx_g()``, ``dt=min(dx^2,dy^2)*Cp0/lam/4.1``,
initial Gaussian ``exp(-(x-lx/2)^2-(y-ly/2)^2)`` on cell centres (ap.jl:11-28).

Variants:

``ap``         array programming: torch tensor expressions (CPU or GPU), like
               the reference's broadcasts (ap.jl:37-43) but with preallocated
               temporaries (the reference allocates every step, §7.4 item 4).
``kp``         three hand-written kernels Flux/Residual/Update (kp.jl:16-54).
``perf``       one fused kernel, double-buffered (perf.jl:3-13,47-52).
``perf_hide``  boundary frame on a high-priority stream, halo exchange right
               behind it, interior on a low-priority stream — the reference's
               intended-but-unfinished overlap (perf_hide.jl:94-101).

All variants compute the same canonical per-cell expression, so their fields
agree bitwise, across variants and across decompositions.

On a GPU with the native halo engine the time loop runs inside the native
executor (no per-step Python, no host waits). Elsewhere (CPU, host-staged or
loopback transports) the same steps are issued from Python.
"""
from __future__ import annotations

import socket
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from .._native import native
from ..parallel import implicit_grid as gg
from ..parallel.halo import gather_, update_halo_
from ..utils import metrics
from ..utils import profiling as prof

TEMPORAL = tuple(range(1, 25))  # max steps per kernel pass (csrc kPipeMaxK)


def default_chunk2(K: int, ny: int) -> int:
    """Rows per wave-task of the K-step kernels: the native executor's measured
    table (csrc/runtime/executor.cpp default_tune_k; 16 for the two-step kernel,
    16..1024 growing with the tile height for K >= 3)."""
    from .._native import has_native, native

    if has_native():
        return int(native().default_chunk_k(int(K), int(ny)))
    if K <= 2:
        return 16
    for lim, c in ((3072, 16), (6144, 32), (12288, 64)):
        if ny < lim:
            return c
    if ny < 32768:
        return 128 if K == 8 else 256
    if K == 16 and ny >= 98304:
        return 1536
    return 1024 if K >= 8 else 512


VARIANTS = ("ap", "kp", "perf", "perf_hide")
_MODE = {"perf": 0, "perf_hide": 1, "kp": 2}


@dataclass
class DiffusionConfig:
    variant: str = "perf"
    nx: int = 128
    ny: int = 128
    nt: int = 1000
    warmup: int = 10  # timer starts at it == warmup+1 (reference: it==11)
    lx: float = 10.0
    ly: float = 10.0
    lam: float = 1.0
    Cp0: float = 1.0
    b_width: tuple = (1, 1)  # perf_hide frame widths (the send planes need 1)
    init: str = "gaussian"  # gaussian | random
    init_on: str = "auto"  # auto | device | host
    seed: int = 1234
    dims: tuple = (0, 0, 0)
    periods: tuple = (0, 0, 0)
    transport: str = "auto"
    device: str | None = None
    chunk_rows: int = 4
    nontemporal: int = 3  # bit 0: NT T2 stores, bit 1: NT 1/Cp loads, bit 2: NT T loads
    kernel: str = "march"
    unroll: int = 4
    vec: int = 2
    use_graph: bool = False
    graph_steps: int = 0
    executor: str = "auto"  # auto | native | python
    do_vis: bool = False
    outdir: str = "output"
    profile: bool = False
    check_every: int = 0  # NaN/Inf guard period (0 = off)
    quiet: bool = False
    # temporal blocking (perf / perf_hide): at most K = temporal steps per
    # kernel pass (1..24) and one width-K halo exchange per pass (grid overlap
    # 2K); step(n) plans passes of 1..K steps (native plan_passes: e.g. 20
    # steps = one 20-step pass). Canonical passes are bitwise identical to
    # single steps.
    temporal: int = 1
    chunk2: int = 0  # K-step kernel rows per wave-task (0: per pass depth, default_chunk2)
    unroll2: int = 2
    # fast-math fp64 arithmetic in every pass (5-point sum with one folded
    # per-cell factor, FMAs; kernels fast5/pipe): same scheme, not bitwise
    # equal to the canonical expression, bitwise equal to its C++ CPU twin
    # (which the CPU path then runs)
    fast_math: bool = False
    # direct-store halos (native executor, fast-math K-step passes): the frame
    # tasks store the neighbours' halo cells straight into their fields --
    # periodic images of this rank, other ranks' tiles in this process
    # (loopback); the halo exchange is not run (DiffusionExecutor::set_direct)
    halo_direct: bool = False
    # (dx, dy) instead of (lx/nx_g, ly/ny_g): probes that compare decompositions
    # at equal coefficients (the pass energy, hence the power-capped clock,
    # depends on them: ry = (dx/dy)^2 = 1 makes two of the three fast-math
    # multipliers trivial; profiles/SUMMARY_r3.md)
    spacing: tuple | None = None

    def validate(self) -> None:
        if self.variant not in VARIANTS:
            raise ValueError(f"variant must be one of {VARIANTS}")
        if self.nt < 1 or self.warmup < 0:
            raise ValueError("nt >= 1 and warmup >= 0 required")
        if self.init not in ("gaussian", "random"):
            raise ValueError("init must be gaussian or random")
        if self.nx < 3 or self.ny < 3:
            raise ValueError("nx, ny >= 3 required")
        if self.temporal not in TEMPORAL:
            raise ValueError(f"temporal must be one of {TEMPORAL}")
        if self.temporal > 1 and self.variant not in ("perf", "perf_hide"):
            raise ValueError("temporal blocking applies to the perf and perf_hide variants")
        if self.fast_math and self.variant not in ("perf", "perf_hide"):
            raise ValueError("fast_math applies to the perf and perf_hide variants")


class Diffusion2D:
    """One rank's share of the distributed diffusion problem."""

    def __init__(self, cfg: DiffusionConfig, grid_kwargs: dict | None = None):
        cfg.validate()
        self.cfg = cfg
        self.chunk2 = cfg.chunk2 or default_chunk2(cfg.temporal, cfg.ny)
        kw = dict(grid_kwargs or {})
        if not gg.grid_is_initialized():
            kw.setdefault("quiet", cfg.quiet)
            if cfg.temporal > 1:  # width-K halos need overlap 2K (IGG: ol >= 2*hw)
                K = cfg.temporal
                kw.setdefault("overlaps", (2 * K, 2 * K, 2))
                kw.setdefault("halowidths", (K, K, 1))
            gg.init_global_grid(cfg.nx, cfg.ny, 1, dimx=cfg.dims[0], dimy=cfg.dims[1],
                                periodx=cfg.periods[0], periody=cfg.periods[1],
                                transport=cfg.transport, device=cfg.device, **kw)
            self._owns_grid = True
        else:
            self._owns_grid = False
        g = self.g = gg.global_grid()
        if (g.nx, g.ny) != (cfg.nx, cfg.ny):
            raise ValueError(f"global grid local size {g.nxyz} != config {(cfg.nx, cfg.ny)}")
        self.device = g.device
        nx, ny = cfg.nx, cfg.ny
        self.dx = cfg.lx / gg.nx_g() if cfg.spacing is None else float(cfg.spacing[0])
        self.dy = cfg.ly / gg.ny_g() if cfg.spacing is None else float(cfg.spacing[1])
        self.dt = min(self.dx * self.dx, self.dy * self.dy) * cfg.Cp0 / cfg.lam / 4.1
        self.coef = ops.StencilCoef.from_physics(cfg.lam, self.dx, self.dy, self.dt)
        dev = self.device
        f64 = dict(dtype=torch.float64, device=dev)
        # 1/Cp (the reference's Cp0.*ones; stored inverted, see rma/common.h)
        self.iCp = torch.empty((ny, nx), **f64)
        ops.fill_(self.iCp, 1.0 / cfg.Cp0)
        self.T = torch.empty((ny, nx), **f64)
        self.init_field(self.T)
        self.T2 = None
        if cfg.variant in ("perf", "perf_hide"):
            self.T2 = self.T.clone()  # perf.jl:36 T2 = copy(T)
        if cfg.variant == "ap":  # the reference's arrays (ap.jl:22-24), preallocated
            self.qx = torch.zeros((ny - 2, nx - 1), **f64)
            self.qy = torch.zeros((ny - 1, nx - 2), **f64)
            self.dTdt = torch.zeros((ny - 2, nx - 2), **f64)
            self._tmp = torch.zeros((ny - 2, nx - 2), **f64)
        elif cfg.variant == "kp":  # T-indexed flux/residual buffers (csrc/kernels/kp.hip)
            self.QX = torch.zeros((ny, nx), **f64)
            self.QY = torch.zeros((ny, nx), **f64)
            self.D = torch.zeros((ny, nx), **f64)
            self.qx, self.qy, self.dTdt = ops.kp_views(self.QX, self.QY, self.D)
        self.parity = 0
        self.steps_done = 0
        self._solo = False
        self._timing = False
        self._ptimes: list = []
        self.executor = None
        self.use_graph = False
        use_native = cfg.executor == "native" or (
            cfg.executor == "auto" and dev.type == "cuda" and g.halo is not None)
        if use_native and cfg.variant != "ap":
            if dev.type != "cuda" or g.halo is None:
                raise RuntimeError("native executor needs a GPU and the rccl/self transport")
            use_graph = bool(cfg.use_graph)
            if use_graph and not g.halo.capturable():
                import warnings

                warnings.warn(f"hipGraph replay disabled: the {g.transport} halo transport cannot "
                              "be stream-captured (RMA_DIAG=rccl_graph forces it for RCCL)",
                              RuntimeWarning, stacklevel=2)
                use_graph = False
            self.use_graph = use_graph
            self.executor = self._build_executor()
            self._setup_direct()
        elif cfg.halo_direct:
            raise ValueError("halo_direct needs the native GPU executor (fast-math perf / "
                             "perf_hide on a GPU); the CPU and torch paths exchange halos")
        self._ap_graph = None
        if cfg.variant == "ap" and cfg.use_graph:
            # ap on a GPU is ~11 small torch launches per step: replay them from
            # a captured hipGraph (torch.cuda.CUDAGraph) when the halo exchange
            # is capturable (1 rank or self copies; RCCL/staged are not)
            self.use_graph = dev.type == "cuda" and g.halo is not None and g.halo.capturable()
            if not self.use_graph:
                import warnings

                warnings.warn(f"hipGraph replay disabled for ap ({dev.type}, {g.transport} "
                              "transport)", RuntimeWarning, stacklevel=2)
        if cfg.temporal > 1 and nx * ny < 1_500_000 and not cfg.quiet:
            import warnings

            warnings.warn(f"temporal={cfg.temporal} on a {nx}x{ny} tile: too few wave-tasks to "
                          "fill the GPU (measured slower than one step per pass below ~1.5M "
                          "cells, e.g. 1024^2: 1.2 vs 1.6 TB/s)", RuntimeWarning, stacklevel=2)
        if cfg.temporal > 1:
            K = cfg.temporal
            nb = g.neighbors
            if any(max(nb[d]) >= 0 and g.overlaps[d] < 2 * K for d in (0, 1)):
                raise ValueError(f"temporal={K} needs grid overlaps >= {2 * K} "
                                 f"(init_global_grid(overlaps=({2 * K},{2 * K},2), "
                                 f"halowidths=({K},{K},1)))")
            self.out2 = self.owned_rect(K)
        if cfg.variant == "perf_hide":
            # the frame holds the send planes [ol-hw, ol): at least ol-1 wide
            bw = (max(cfg.b_width[0], g.overlaps[0] - 1), max(cfg.b_width[1], g.overlaps[1] - 1))
            self.frame_rects, self.interior = ops.hide_rects(nx, ny, *bw, vec=cfg.vec)
        self.tuning = ops.StencilTuning(cfg.chunk_rows, int(cfg.nontemporal), cfg.kernel,
                                        cfg.unroll, cfg.vec)

    def owned_rect(self, k: int) -> tuple:
        """Cells a k-step pass writes: next to a neighbour the k cells [0,k)
        are halo (refreshed by the exchange), elsewhere boundary cell 0 stays
        (csrc/runtime/plan.cpp owned_rect)."""
        nb, nx, ny = self.g.neighbors, self.cfg.nx, self.cfg.ny
        return (k if nb[0][0] >= 0 else 1, nx - (k if nb[0][1] >= 0 else 1),
                k if nb[1][0] >= 0 else 1, ny - (k if nb[1][1] >= 0 else 1))

    def plan(self, n: int) -> list:
        """Passes step(n) runs (deepest first): the native executor's plan, or
        the same planner for the Python loop (csrc/runtime/plan.cpp)."""
        if self.executor is not None:
            return list(self.executor.plan(int(n)))
        cfg = self.cfg
        if cfg.variant not in ("perf", "perf_hide") or (cfg.temporal == 1 and not cfg.fast_math):
            return [1] * int(n)
        from .._native import has_native

        if has_native():
            fast = cfg.fast_math and ops.fast5_ok(self.coef)
            costs = native().default_pass_costs(cfg.temporal, fast, float(cfg.nx) * cfg.ny)
            return list(native().plan_passes(int(n), costs))
        K = cfg.temporal
        return [K] * (int(n) // K) + ([int(n) % K] if int(n) % K else [])

    def _build_executor(self):
        cfg, g = self.cfg, self.g
        nx, ny = cfg.nx, cfg.ny
        bwx, bwy = cfg.b_width
        if cfg.kernel != "march" and self.T.is_cuda:  # the LDS-tiled one-step kernel: librma_lab.so
            from .._native import load_lab

            load_lab()
        return native().Executor(
            self.T.data_ptr(), self.T2.data_ptr() if self.T2 is not None else 0,
            self.iCp.data_ptr(), nx, ny, _MODE[cfg.variant], tuple(self.coef),
            cfg.chunk_rows, int(cfg.nontemporal), ops.kernel_id(cfg.kernel), int(bwx), int(bwy),
            int(self.use_graph), int(cfg.graph_steps), g.halo,
            self.QX.data_ptr() if cfg.variant == "kp" else 0,
            self.QY.data_ptr() if cfg.variant == "kp" else 0,
            self.D.data_ptr() if cfg.variant == "kp" else 0, int(cfg.unroll),
            int(cfg.vec), int(cfg.temporal), int(g.overlaps[0]), int(g.overlaps[1]),
            int(cfg.chunk2), int(cfg.unroll2), int(bool(cfg.fast_math)))

    def _direct_ranks(self) -> list:
        """Rank of each of the 8 directions (native executor order
        ``Executor.direct_dirs``): the Cartesian neighbours, the diagonals
        where both axis neighbours exist, -1 elsewhere."""
        g = self.g
        nb = g.neighbors
        diag = list(g.topo.diagonals(g.me))
        out = []
        for i, j in native().Executor.direct_dirs:
            if j == 0:
                out.append(nb[0][i > 0])
            elif i == 0:
                out.append(nb[1][j > 0])
            elif nb[0][i > 0] >= 0 and nb[1][j > 0] >= 0:
                out.append(diag[(j > 0) * 2 + (i > 0)])
            else:
                out.append(-1)
        return out

    def _setup_direct(self) -> None:
        """Collective: hand the executor its direct-store peers (cfg.halo_direct).
        Every rank's fields and pass-count words are exchanged -- in-process
        through the loopback hub; between processes of one node as IPC
        exports (``IpcMap``: the peers' T / T2 / count words mapped into this
        process) gathered over the gloo group -- and the counts zeroed while
        every rank is quiescent."""
        if not self.cfg.halo_direct or self.executor is None:
            return
        g, cfg = self.g, self.cfg
        if not (cfg.fast_math and cfg.variant in ("perf", "perf_hide")):
            raise ValueError("halo_direct needs fast-math perf / perf_hide passes")
        ranks = self._direct_ranks()
        remote = any(r >= 0 and r != g.me for r in ranks)
        procs = remote and g.transport != "loopback"
        if procs and not (dist.is_available() and dist.is_initialized()):
            raise ValueError(f"halo_direct with other ranks needs their fields mapped in this "
                             f"process (loopback) or IPC between processes, not {g.transport!r}")
        # the words the neighbours count our passes in: device memory between
        # processes (wait kernels); pinned host memory for ranks of this
        # process, whose host threads wait (DiffusionExecutor::direct_wait)
        host_wait = remote and not procs
        if getattr(self, "_dflags", None) is None or self._dflags.is_cuda == host_wait:
            self._dflags = (torch.zeros(8, dtype=torch.int64, pin_memory=True) if host_wait
                            else torch.zeros(8, dtype=torch.int64, device=self.T.device))
        mine = (self.T.data_ptr(), self.T2.data_ptr(), self._dflags.data_ptr())
        torch.cuda.synchronize(self.T.device)
        if remote:
            g.comm.barrier()  # every rank's previous executor drained
        self._dflags.zero_()
        torch.cuda.synchronize(self.T.device)
        if procs:
            table = self._direct_ipc_table(ranks, mine)
        else:
            table = g.comm.hub.collect(g.me, mine) if remote else {g.me: mine}
        peers = []
        for d, r in enumerate(ranks):
            if r < 0:
                peers.append((-1, 0, 0, 0))
                continue
            T, T2, fl = table[r]
            # the peer's count of OUR passes: from its side we are direction 7 - d
            peers.append((r, T, T2, 0 if r == g.me else fl + 8 * (7 - d)))
        self.executor.set_direct(peers, self._dflags.data_ptr() if remote else 0, host_wait)
        if remote:
            g.comm.barrier()  # nobody stores before every rank has zeroed its counts

    def _direct_ipc_table(self, ranks: list, mine: tuple) -> dict:
        """IPC exports of every rank's (T, T2, count words), gathered over the
        gloo group; the direct-store peers' opened in this process. Every peer
        must be a process of this node (its handle opens here)."""
        from ..parallel.comm import _gloo_group

        n = native()
        host = socket.gethostname()
        exp = (host, tuple(n.IpcMap.export_ptr(p) for p in mine))
        allx: list = [None] * dist.get_world_size()
        dist.all_gather_object(allx, exp, group=_gloo_group())
        me = self.g.me
        others = sorted({r for r in ranks if r >= 0 and r != me})
        far = [r for r in others if allx[r][0] != host]
        if far:
            raise ValueError(f"halo_direct: ranks {far} run on other nodes ({allx[far[0]][0]}); "
                             f"IPC maps device memory of this node only")
        if getattr(self, "_ipc_map", None) is None:
            self._ipc_map = n.IpcMap()
        table = {me: mine}
        for r in others:
            table[r] = tuple(self._ipc_map.open(b) for b in allx[r][1])
        return table

    def set_temporal(self, K: int, fast_math: bool | None = None) -> None:
        """Switch the steps per kernel pass (e.g. to time the one-step kernel on
        the same tile) and optionally the fast-math arithmetic. The grid
        overlap must allow it (2K <= overlap)."""
        cfg, g = self.cfg, self.g
        if K not in TEMPORAL or (K > 1 and cfg.variant not in ("perf", "perf_hide")):
            raise ValueError(f"temporal={K} not available for {cfg.variant}")
        nb = g.neighbors
        if any(max(nb[d]) >= 0 and g.overlaps[d] < 2 * K for d in (0, 1)):
            raise ValueError(f"temporal={K} needs grid overlaps >= {2 * K}")
        self.synchronize()
        if self.parity:  # make T the current field, then rebuild from parity 0
            self.T, self.T2 = self.T2, self.T
            self.parity = 0
        cfg.temporal = K
        if fast_math is not None:
            cfg.fast_math = bool(fast_math)
        self.chunk2 = cfg.chunk2 or default_chunk2(K, cfg.ny)
        if K > 1:
            self.out2 = self.owned_rect(K)
        self._rebuild_executor()

    def set_spacing(self, spacing: tuple | None) -> None:
        """Switch the grid spacing (dx, dy) the coefficients derive from (None:
        the physical lx/nx_g, ly/ny_g) -- dt, the stencil coefficients and the
        executor follow. For timing probes: bench.py re-times each rank at
        isotropic coefficients to split a weak-scaling loss into halo,
        coefficient and GPU parts (the fast-math pass energy depends on
        ry = (dx/dy)^2, profiles/SUMMARY_r3.md section 1). Changes the physics
        of the run."""
        cfg, g = self.cfg, self.g
        self.synchronize()
        cfg.spacing = None if spacing is None else (float(spacing[0]), float(spacing[1]))
        self.dx = cfg.lx / g.nxyz_g[0] if cfg.spacing is None else cfg.spacing[0]
        self.dy = cfg.ly / g.nxyz_g[1] if cfg.spacing is None else cfg.spacing[1]
        self.dt = min(self.dx * self.dx, self.dy * self.dy) * cfg.Cp0 / cfg.lam / 4.1
        self.coef = ops.StencilCoef.from_physics(cfg.lam, self.dx, self.dy, self.dt)
        self._rebuild_executor()

    def _rebuild_executor(self) -> None:
        """A new native executor for the current config / coefficients (field
        parity folded into T first; solo mode carried over)."""
        if self.executor is None:
            return
        self.synchronize()
        if self.parity:
            self.T, self.T2 = self.T2, self.T
            self.parity = 0
        self.executor = self._build_executor()
        self._setup_direct()
        if self._solo:
            self.executor.set_solo(True)

    # ------------------------------------------------------------------
    def geometry(self, A_shape=None) -> ops.TileGeometry:
        g = self.g
        ny_a, nx_a = A_shape or (g.ny, g.nx)
        return ops.TileGeometry(
            gx0=g.coords[0] * (g.nx - g.overlaps[0]), gy0=g.coords[1] * (g.ny - g.overlaps[1]),
            nxg=g.nxyz_g[0], nyg=g.nxyz_g[1], dx=self.dx, dy=self.dy,
            xoff=0.5 * (g.nx - nx_a) * self.dx, yoff=0.5 * (g.ny - ny_a) * self.dy,
            periodx=g.periods[0], periody=g.periods[1])

    def init_field(self, T: torch.Tensor) -> None:
        cfg = self.cfg
        geom = self.geometry(tuple(T.shape))
        if cfg.init == "random":
            ops.init_random_(T, geom, seed=cfg.seed)
            return
        where = cfg.init_on
        if where == "auto":
            where = "device"
        if where == "host":  # the reference's host comprehension + copy (ap.jl:28)
            ny, nx = T.shape
            from ..parallel.geometry import coords_1d

            x = coords_1d(geom.gx0, nx, self.dx, geom.xoff, geom.nxg, geom.periodx).numpy()
            y = coords_1d(geom.gy0, ny, self.dy, geom.yoff, geom.nyg, geom.periody).numpy()
            a = (x + self.dx / 2) - cfg.lx / 2
            b = (y + self.dy / 2) - cfg.ly / 2
            T.copy_(torch.from_numpy(np.exp(-(a * a)[None, :] - (b * b)[:, None])))
        else:
            ops.init_gaussian_(T, geom, cfg.lx, cfg.ly)

    @property
    def field(self) -> torch.Tensor:
        """The current temperature field (after the last completed step)."""
        if self.T2 is None:
            return self.T
        return self.T2 if self.parity else self.T

    # ------------------------------------------------------------------
    def step(self, n: int = 1) -> None:
        """Advance n time steps (asynchronous on GPU)."""
        if n <= 0:
            return
        if self.executor is not None:
            self.executor.run(int(n), torch.cuda.current_stream(self.device).cuda_stream)
            self.parity = self.executor.parity
            self.steps_done += n
            return
        v = self.cfg.variant
        if v == "ap" and getattr(self, "use_graph", False):
            k = self._ap_graph_len()
            for _ in range(n // k):
                self._ap_graph.replay()
            self.steps_done += n - n % k
            n %= k
        if v in ("perf", "perf_hide"):
            # the passes of the native planner (one-step passes when
            # temporal=1 without fast_math). The executor splits frame /
            # interior over two streams; this loop runs them in sequence:
            # frame -> exchange -> interior.
            for K in self.plan(n):
                self._pass(K)
            return
        for _ in range(n):
            if v == "ap":
                self._step_ap()
            else:  # kp
                ops.flux(self.QX, self.QY, self.T, self.coef.mlam, self.coef.rdx, self.coef.rdy)
                ops.residual(self.D, self.QX, self.QY, self.iCp, self.coef.rdx, self.coef.rdy)
                ops.update(self.T, self.D, self.coef.dt)
                update_halo_(self.T)
            self.steps_done += 1

    def _pass(self, K: int) -> None:
        """One pass of K steps outside the native executor (CPU twins, or the
        GPU kernels with the loopback / staged transports)."""
        cfg = self.cfg
        Tin, Tout = (self.T2, self.T) if self.parity else (self.T, self.T2)
        fast = cfg.fast_math and ops.fast5_ok(self.coef)
        solo = self._solo
        timing = self._timing
        if timing:
            self.synchronize()
            t0 = metrics.now()
        t_frame = t_halo = None
        if K == 1 and not fast:  # one canonical step
            if cfg.variant == "perf" or solo:
                ops.stencil_step(Tout, Tin, self.iCp, self.coef, tuning=self.tuning)
            else:  # perf_hide, sequential emulation: frame -> halo -> interior
                ops.stencil_step(Tout, Tin, self.iCp, self.coef, self.frame_rects, self.tuning)
                if timing:
                    self.synchronize()
                    t_frame = metrics.now()
                update_halo_(Tout)
                if timing:
                    self.synchronize()
                    t_halo = metrics.now()
                if self.interior is not None:
                    ops.stencil_step(Tout, Tin, self.iCp, self.coef, [self.interior], self.tuning)
        else:
            rect = ops.interior_rect(cfg.nx, cfg.ny) if solo else self.owned_rect(K)
            if Tin.is_cuda:  # the executor's kernel for this pass depth
                fn = native().fast_kernel_k if fast else None
                kern, vec, ch = (fn(K, cfg.ny, tuple(self.coef)) if fn
                                 else native().canonical_kernel_k(K, cfg.ny))
                name = ops.kernel_name(kern)
                tn = ops.StencilTuning(chunk_rows=cfg.chunk2 or ch, xcd_remap=1, kernel=name,
                                       vec=vec)
            else:  # the C++ twin of the pass arithmetic
                tn = ops.StencilTuning(kernel="pipe" if fast else "pipec")
            if K == 2 and not fast and Tin.is_cuda:
                ops.stencil2_step(Tout, Tin, self.iCp, self.coef, [rect])
            else:
                ops.stencilk_step(K, Tout, Tin, self.iCp, self.coef, [rect], tn)
        if t_halo is None and not solo:
            if timing:
                self.synchronize()
                t_frame = metrics.now()
            update_halo_(Tout)
            if timing:
                self.synchronize()
                t_halo = metrics.now()
        if timing:
            self.synchronize()
            t1 = metrics.now()
            tf = t_frame if t_frame is not None else t1
            th = t_halo if t_halo is not None else tf
            # sequential: the exchange is never hidden (frame_ms = compute
            # before the exchange, interior_ms = compute after it)
            self._ptimes.append({"K": K, "frame_ms": (tf - t0) * 1e3,
                                 "halo_ms": (th - tf) * 1e3, "interior_ms": (t1 - th) * 1e3,
                                 "pass_ms": (t1 - t0) * 1e3, "exposed_halo_ms": (th - tf) * 1e3})
        self.parity ^= 1
        self.steps_done += K

    # ------------------------------------------------------------------
    def enable_pass_timing(self, on: bool = True) -> None:
        """Record per-pass timings from now on (native executor: HIP events on
        both streams; Python loop: synchronised wall clock)."""
        self._timing = bool(on)
        self._ptimes = []
        if self.executor is not None:
            self.executor.set_timing(bool(on))

    def pass_timings(self) -> list:
        """One dict per pass since enable_pass_timing: K, frame_ms, halo_ms
        (pack + exchange + unpack), interior_ms, pass_ms, exposed_halo_ms (how
        long the exchange outlasted the interior; == halo_ms without overlap)."""
        if self.executor is not None:
            return [dict(t) for t in self.executor.timings()]
        return list(self._ptimes)

    def set_solo(self, on: bool) -> None:
        """Run this tile as if it had no neighbour (no exchange, one launch per
        pass): the same-run single-GPU reference of a weak-scaling measurement.
        The field is then not the multi-rank solution."""
        self.synchronize()
        self._solo = bool(on)
        if self.executor is not None:
            self.executor.set_solo(bool(on))

    def _ap_graph_len(self) -> int:
        """Capture graph_steps ap steps once (capture does not execute them)."""
        if self._ap_graph is None:
            k = max(1, int(self.cfg.graph_steps) or 20)
            cur = torch.cuda.current_stream(self.device)
            side = torch.cuda.Stream(self.device)
            side.wait_stream(cur)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.stream(side):
                graph.capture_begin()
                try:
                    for _ in range(k):
                        self._step_ap()
                finally:
                    graph.capture_end()
            cur.wait_stream(side)
            self._ap_graph, self._ap_graph_steps = graph, k
        return self._ap_graph_steps

    def _step_ap(self) -> None:
        """ap.jl:38-42 as torch expressions (canonical operation order)."""
        c = self.coef
        T, qx, qy, d, tmp = self.T, self.qx, self.qy, self.dTdt, self._tmp
        torch.sub(T[1:-1, 1:], T[1:-1, :-1], out=qx)
        qx.mul_(c.mlam).mul_(c.rdx)  # qx = -lam*d_xi(T)*_dx
        torch.sub(T[1:, 1:-1], T[:-1, 1:-1], out=qy)
        qy.mul_(c.mlam).mul_(c.rdy)  # qy = -lam*d_yi(T)*_dy
        torch.sub(qx[:, 1:], qx[:, :-1], out=d)
        d.mul_(c.rdx)
        torch.sub(qy[1:, :], qy[:-1, :], out=tmp)
        tmp.mul_(c.rdy)
        d.add_(tmp).neg_().mul_(self.iCp[1:-1, 1:-1])  # dTdt = 1/Cp*(-(dqx+dqy))
        d.mul_(c.dt)
        T[1:-1, 1:-1].add_(d)  # T = T + dt*dTdt
        update_halo_(T)

    def synchronize(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        if self.executor is not None and hasattr(self.executor, "check_error"):
            self.executor.check_error()  # a fused pass's timed-out frame wait, if any

    def check_finite(self) -> None:
        bad = float(ops.reduce(self.field, "nonfinite"))
        if bad:
            raise FloatingPointError(
                f"rank {self.g.me}: {int(bad)} non-finite cells after step {self.steps_done}")

    # ------------------------------------------------------------------
    def run(self) -> metrics.RunResult:
        """The reference protocol: nt steps, timer from step warmup+1, T_eff."""
        cfg = self.cfg
        g = self.g
        if g.me == 0 and not cfg.quiet:
            print("Starting the time loop 🚀...", end="", flush=True)
        warm = min(cfg.warmup, cfg.nt)
        timed = cfg.nt - warm
        if warm:
            self._advance(warm)
        profiler = prof.LoopProfiler(enabled=cfg.profile, rank=g.me)
        gg.tic()
        with profiler:
            self._advance(timed)
            wtime = gg.toc()
        if g.me == 0 and not cfg.quiet:
            print("done", flush=True)
        teff = metrics.t_eff(cfg.nx, cfg.ny, wtime, timed)
        tmin = g.comm.allreduce(teff, "min")
        tmax = g.comm.allreduce(teff, "max")
        ttot = g.comm.allreduce(teff, "sum")
        res = metrics.RunResult(
            variant=cfg.variant, nprocs=g.nprocs, dims=g.dims, nx=cfg.nx, ny=cfg.ny,
            nxg=g.nxyz_g[0], nyg=g.nxyz_g[1], nt=cfg.nt, timed_steps=timed, wtime=wtime,
            t_it=wtime / timed if timed else float("nan"), teff=teff, teff_min=tmin,
            teff_max=tmax, teff_total=ttot, transport=g.transport, device=str(self.device))
        if g.me == 0 and not cfg.quiet:
            print(metrics.reference_line(cfg.nt, wtime, teff), flush=True)
        if cfg.profile:
            profiler.write("prof.txt")
        if cfg.do_vis:
            res.extra["vis"] = self.visualise()
        return res

    def _advance(self, n: int) -> None:
        k = self.cfg.check_every
        if k <= 0:
            self.step(n)
            return
        done = 0
        while done < n:
            m = min(k, n - done)
            self.step(m)
            done += m
            self.check_finite()

    # ------------------------------------------------------------------
    def gather_interior(self, root: int = 0, max_bytes: int | None = None):
        """T_v: the halo-stripped fields of all ranks assembled on root
        (ap.jl:45-46: T_nh .= Array(T[2:end-1,2:end-1]); gather!(T_nh, T_v)).

        The gather lands on the root's device (RCCL) or host: refused above
        ``max_bytes`` (default ``RMA_GATHER_MAX_BYTES`` or 8 GiB) -- a 288 GB
        tile per rank would need N x 80 GB there; ``visualise`` subsamples."""
        import os

        limit = int(max_bytes if max_bytes is not None
                    else os.environ.get("RMA_GATHER_MAX_BYTES", 8 << 30))
        inner = self.field[1:-1, 1:-1]
        total = inner.numel() * inner.element_size() * self.g.nprocs
        if total > limit:
            raise ValueError(f"gather_interior would assemble {total / 2**30:.1f} GiB on rank "
                             f"{root} (limit {limit / 2**30:.1f} GiB): subsample first "
                             "(visualise(max_pixels=...)) or raise max_bytes")
        T_nh = inner.contiguous()
        return gather_(T_nh, None, root)

    def visualise(self, max_pixels: int = 2048) -> dict | None:
        """Gather + heatmap PNG on rank 0 (ap.jl:45-47). Above ``max_pixels``
        per side (e.g. the 288 GB tiles: ~80 GB of interior per rank) every
        rank subsamples its interior with the same stride before the gather
        (SURVEY.md §2.5); maximum(T_v) stays exact (a device reduction)."""
        from ..utils import vis

        g = self.g
        inner = self.field[1:-1, 1:-1]
        extent = max(inner.shape[1] * g.dims[0], inner.shape[0] * g.dims[1])
        stride = max(1, -(-extent // max_pixels))
        if stride == 1:
            T_v = self.gather_interior()
            tmax = None
        else:
            T_v = gather_(inner[::stride, ::stride].contiguous(), None, 0)
            tmax = g.comm.allreduce(float(inner.amax()), "max")
        if g.me != 0:
            return None
        name = {"perf_hide": "hide"}.get(self.cfg.variant, self.cfg.variant)
        path = vis.output_name(name, self.g.nprocs, gg.nx_g(), gg.ny_g(), self.cfg.outdir)
        info = vis.heatmap_png(T_v, path)
        info["stride"] = stride
        if tmax is not None:
            info["max"] = tmax
        if not self.cfg.quiet:
            print(f"maximum(T_v) = {info['max']}", flush=True)  # perf_hide.jl:115
        return info

    def close(self) -> None:
        try:
            self.synchronize()  # raises a pending executor error; resources go either way
        finally:
            self.executor = None
            if getattr(self, "_ipc_map", None) is not None:
                # every rank's kernels are done storing into the mapped peers
                # (its synchronize above) before any rank unmaps or frees. Our
                # own run already waited for every neighbour's last stores into
                # us, so a dead peer only costs this bounded wait
                import datetime
                import os
                import warnings

                from ..parallel.comm import _gloo_group

                tmo = float(os.environ.get("RMA_TEARDOWN_TIMEOUT", "30"))
                try:
                    dist.barrier(group=_gloo_group(), async_op=True).wait(
                        timeout=datetime.timedelta(seconds=tmo))
                except Exception as e:  # noqa: BLE001 - a dead peer must not hang close()
                    warnings.warn(f"halo_direct teardown: the peers' barrier did not complete "
                                  f"within {tmo:.0f} s ({e}); unmapping anyway",
                                  RuntimeWarning, stacklevel=2)
                finally:
                    self._ipc_map.close_all()
                    self._ipc_map = None
            self._ap_graph = None
            if self._owns_grid:
                gg.finalize_global_grid()
