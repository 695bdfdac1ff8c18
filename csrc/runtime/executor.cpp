#include "rma/executor.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <array>
#include <utility>

#include "rma/hip_check.h"
#include "rma/trace.h"

namespace rma {

namespace {
hipStream_t S(void* p) { return reinterpret_cast<hipStream_t>(p); }
hipEvent_t E(void* p) { return reinterpret_cast<hipEvent_t>(p); }
}  // namespace

StencilTuning default_tune_k(int K, int64_t ny) {
  StencilTuning t;
  t.nontemporal = 3;
  if (K <= 2) {
    t.chunk_rows = 16;
    t.unroll = 2;
    return t;
  }
  t.kernel = 3;  // LDS 1/Cp ring + DPP lane shifts (sweep_tbk_dpp_*: +6% over bpermute)
  t.xcd_remap = 1;
  // rows per wave-task: long chunks amortise the 2K-1 rows a chunk recomputes,
  // short ones give small tiles enough waves (sweeps at 2048^2..101376^2,
  // profiles/SUMMARY_r1.md)
  if (ny < 3072) t.chunk_rows = 16;
  else if (ny < 6144) t.chunk_rows = 32;
  else if (ny < 12288) t.chunk_rows = 64;
  else if (ny < 32768) t.chunk_rows = K == 8 ? 128 : 256;  // K=12/16: c256 (profiles/sweep_deepk_16k)
  else if (K == 16 && ny >= 98304) t.chunk_rows = 1536;  // 288 GB tile: 63.8 vs 64.5 ms (c1024)
  else t.chunk_rows = K >= 8 ? 1024 : 512;
  return t;
}

StencilTuning fast_tune_k(int K, int64_t ny, const StencilCoef& c) {
  StencilTuning t = default_tune_k(K, ny);
  if (K <= 1) return t;
  t.xcd_remap = 1;
  if (!fast5_ok(c)) {
    t.kernel = 4;
    return t;
  }
  t.kernel = K == 16 ? 7 : K == 12 ? 6 : 5;
  t.vec = K >= 12 ? 4 : 2;
  return t;
}

DiffusionExecutor::DiffusionExecutor(double* T, double* T2, const double* iCp, int64_t nx,
                                     int64_t ny, const ExecParams& p, HaloExchanger* halo,
                                     double* qx, double* qy, double* dTdt)
    : T_(T), T2_(T2), iCp_(iCp), nx_(nx), ny_(ny), p_(p), halo_(halo), qx_(qx), qy_(qy),
      dTdt_(dTdt) {
  RMA_CHECK_ARG(nx >= 3 && ny >= 3, "grid too small: " << nx << "x" << ny);
  RMA_CHECK_ARG(T && iCp, "null field");
  RMA_CHECK_ARG(p.mode == Mode::kKp || T2 != nullptr, "T2 required");
  RMA_CHECK_ARG(p.mode != Mode::kKp || (qx && qy && dTdt), "kp needs qx, qy, dTdt");
  RMA_CHECK_ARG(!p.use_graph || !halo || halo->capturable(),
                "hipGraph replay needs a capturable halo transport (RCCL or none); the loopback "
                "transport synchronises on the host");
  RMA_CHECK_ARG(p.temporal == 1 || p.temporal == 2 || p.temporal == 3 || p.temporal == 4 ||
                    p.temporal == 6 || p.temporal == 8 || p.temporal == 12 || p.temporal == 16,
                "temporal (steps per pass) must be 1, 2, 3, 4, 6, 8, 12 or 16, got "
                    << p.temporal);
  RMA_CHECK_ARG(p.temporal <= 8 || (p.fast_math && fast5_ok(p.coef)),
                "12 or 16 steps per pass run on the fast5 kernel only: needs fast_math and "
                "lam != 0");
  RMA_CHECK_ARG(p.temporal == 1 || p.mode != Mode::kKp,
                "temporal blocking applies to perf / perf_hide, not kp");
  RMA_CHECK_ARG(p.olx >= 2 && p.oly >= 2, "overlaps must be >= 2");
  hwx_ = hwy_ = p.temporal;  // halo width = steps per exchange
  // fast_math: the 5-point-sum kernels (5 fp64 ops per cell update) unless the
  // coefficients cannot be folded (lam == 0), then the reassociated-flux one
  if (p_.fast_math && p.temporal > 1) {
    const StencilTuning f = fast_tune_k(p.temporal, ny, p.coef);
    p_.tune2.kernel = f.kernel;
    p_.tune2.vec = f.vec;
    p_.tune2.xcd_remap = f.xcd_remap;
  }
  std::array<std::array<int, 2>, 3> nbr{{{-1, -1}, {-1, -1}, {-1, -1}}};
  if (halo) nbr = halo->neighbors();
  const int64_t ol[2] = {p.olx, p.oly};
  for (int d = 0; d < 2; ++d)
    RMA_CHECK_ARG((nbr[d][0] < 0 && nbr[d][1] < 0) || ol[d] >= 2 * p.temporal,
                  "temporal=" << p.temporal << " needs a grid overlap >= " << 2 * p.temporal
                              << " along dim " << d << " (init_global_grid overlaps=2K, "
                              << "halowidths=K), got " << ol[d]);
  full_ = {1, nx - 1, 1, ny - 1};
  // perf_hide: the frame must contain the send planes [ol-hw, ol) of every
  // side, so it is at least ol-1 cells wide (the reference's b_width >= overlap
  // invariant); minimal frames otherwise (width 1 for ol=2:
  // thin x-frames run in the kernel's column mode, profiles/).
  if (p.mode == Mode::kHide) {
    RMA_CHECK_ARG(p.bwx >= 1 && p.bwy >= 1,
                  "b_width must be >= 1 so the send planes belong to the boundary kernel");
    split(full_, std::max(p.bwx, p.olx - 1), std::max(p.bwy, p.oly - 1), frame_, interior_);
  } else {
    interior_ = full_;
  }
  if (p.temporal > 1) {
    // owned rect of a K-step pass: next to a neighbour the K cells [0,K) are
    // halo and only the exchange refreshes them (level j is valid from
    // column j on, so the pass outputs from column K)
    const int64_t K = p.temporal;
    out2_ = {nbr[0][0] >= 0 ? K : 1, nx - (nbr[0][1] >= 0 ? K : 1),
             nbr[1][0] >= 0 ? K : 1, ny - (nbr[1][1] >= 0 ? K : 1)};
    RMA_CHECK_ARG(!out2_.empty(), "tile too small for temporal blocking: " << nx << "x" << ny);
    // perf_hide with no neighbour at all has nothing to overlap: the frame
    // launch would only compete with the interior (measured ~1% of a K=16 pass
    // at the 288 GB tile, rocprofv3 trace), so one launch covers the owned rect
    const bool any_nbr = nbr[0][0] >= 0 || nbr[0][1] >= 0 || nbr[1][0] >= 0 || nbr[1][1] >= 0;
    if (p.mode == Mode::kHide && any_nbr)
      split(out2_, std::max(p.bwx, p.olx - out2_.x0), std::max(p.bwy, p.oly - out2_.y0),
            frame2_, interior2_);
    else
      interior2_ = out2_;
  }
  int least = 0, greatest = 0;
  RMA_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t hi, lo;
  // Create the low-priority (interior) stream FIRST. Measured on MI355X /
  // ROCm 7 (bench/probe_set_temporal.py, profiles/SUMMARY_r1.md): creating the
  // high-priority stream first left every second executor of a process with
  // a low-priority stream running the stencil ~25% slower (4.6 vs 6.2 TB/s);
  // low-first (or unprioritised streams) is fast for every instance.
  // RMA_EXEC_STREAMS=plain|hifirst selects the alternatives for diagnostics.
  const char* sm = std::getenv("RMA_EXEC_STREAMS");
  const std::string mode = sm ? sm : "lofirst";
  if (mode == "plain") {
    RMA_HIP_CHECK(hipStreamCreateWithFlags(&lo, hipStreamNonBlocking));
    RMA_HIP_CHECK(hipStreamCreateWithFlags(&hi, hipStreamNonBlocking));
  } else if (mode == "hifirst") {
    RMA_HIP_CHECK(hipStreamCreateWithPriority(&hi, hipStreamNonBlocking, greatest));
    RMA_HIP_CHECK(hipStreamCreateWithPriority(&lo, hipStreamNonBlocking, least));
  } else {
    RMA_HIP_CHECK(hipStreamCreateWithPriority(&lo, hipStreamNonBlocking, least));
    RMA_HIP_CHECK(hipStreamCreateWithPriority(&hi, hipStreamNonBlocking, greatest));
  }
  if (std::getenv("RMA_EXEC_VERBOSE"))
    fprintf(stderr, "[executor] priority range least=%d greatest=%d mode=%s hi=%p lo=%p\n", least,
            greatest, mode.c_str(), (void*)hi, (void*)lo);
  s_hi_ = hi;
  s_lo_ = lo;
  hipEvent_t a, b, c;
  RMA_HIP_CHECK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
  RMA_HIP_CHECK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
  RMA_HIP_CHECK(hipEventCreateWithFlags(&c, hipEventDisableTiming));
  e_hi_ = a;
  e_lo_ = b;
  e_in_ = c;
}

DiffusionExecutor::~DiffusionExecutor() {
  if (graph_exec_) (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(graph_exec_));
  if (e_hi_) (void)hipEventDestroy(E(e_hi_));
  if (e_lo_) (void)hipEventDestroy(E(e_lo_));
  if (e_in_) (void)hipEventDestroy(E(e_in_));
  if (s_hi_) (void)hipStreamDestroy(S(s_hi_));
  if (s_lo_) (void)hipStreamDestroy(S(s_lo_));
}

void DiffusionExecutor::split(const Rect& out, int64_t bwx, int64_t bwy,
                              std::vector<Rect>& frame, Rect& interior) const {
  const int64_t xi0 = out.x0 + bwx, xi1 = out.x1 - bwx;
  const int64_t yi0 = out.y0 + bwy, yi1 = out.y1 - bwy;
  if (xi0 >= xi1 || yi0 >= yi1) {
    interior = {0, 0, 0, 0};
    frame = {out};
  } else {
    interior = {xi0, xi1, yi0, yi1};
    frame = {{out.x0, out.x1, out.y0, yi0},
             {out.x0, out.x1, yi1, out.y1},
             {out.x0, xi0, yi0, yi1},
             {xi1, out.x1, yi0, yi1}};
  }
}

namespace {
HaloField field_of(double* A, int64_t nx, int64_t ny, int64_t olx, int64_t oly, int64_t hwx,
                   int64_t hwy) {
  HaloField f;
  f.ptr = A;
  f.size = {nx, ny, 1};
  f.elem_bytes = 8;
  f.ol = {olx, oly, 2};
  f.hw = {hwx, hwy, 1};
  return f;
}
}  // namespace

void DiffusionExecutor::exchange(double* A, stream_t s) {
  if (!halo_) return;
  halo_->exchange({field_of(A, nx_, ny_, p_.olx, p_.oly, hwx_, hwy_)}, s, 3);
}

void DiffusionExecutor::enqueue_step(double* Tin, double* Tout) {
  const StencilCoef& c = p_.coef;
  switch (p_.mode) {
    case Mode::kPerf: {
      TraceRange tr("rma.step.perf");
      stencil_rects_gpu(Tout, Tin, iCp_, nx_, ny_, &full_, 1, c, p_.tune, s_lo_);
      exchange(Tout, s_lo_);
      break;
    }
    case Mode::kKp: {
      TraceRange tr("rma.step.kp");
      flux_gpu(qx_, qy_, Tin, nx_, ny_, c.mlam, c.rdx, c.rdy, s_lo_);
      residual_gpu(dTdt_, qx_, qy_, iCp_, nx_, ny_, c.rdx, c.rdy, s_lo_);
      update_gpu(Tin, dTdt_, nx_, ny_, c.dt, s_lo_);
      exchange(Tin, s_lo_);
      break;
    }
    case Mode::kHide: {
      TraceRange tr("rma.step.hide");
      // previous step fully done on both streams before this one touches T/T2
      RMA_HIP_CHECK(hipStreamWaitEvent(S(s_hi_), E(e_lo_), 0));
      RMA_HIP_CHECK(hipStreamWaitEvent(S(s_lo_), E(e_hi_), 0));
      StencilTuning ft = p_.tune;
      ft.chunk_rows = std::min(ft.chunk_rows, 16);
      {
        TraceRange tb("rma.boundary");
        stencil_rects_gpu(Tout, Tin, iCp_, nx_, ny_, frame_.data(), (int)frame_.size(), c, ft,
                          s_hi_);
      }
      {
        TraceRange th("rma.halo");
        exchange(Tout, s_hi_);
      }
      RMA_HIP_CHECK(hipEventRecord(E(e_hi_), S(s_hi_)));
      if (!interior_.empty()) {
        TraceRange ti("rma.interior");
        stencil_rects_gpu(Tout, Tin, iCp_, nx_, ny_, &interior_, 1, c, p_.tune, s_lo_);
      }
      RMA_HIP_CHECK(hipEventRecord(E(e_lo_), S(s_lo_)));
      break;
    }
  }
}

void DiffusionExecutor::multi_step(double* Tin, double* Tout, const Rect* rects, int n,
                                   const StencilTuning& tn, void* stream) {
  if (p_.temporal == 2 && !p_.fast_math)  // dedicated two-step kernel: faster at K=2
    stencil2_rects_gpu(Tout, Tin, iCp_, nx_, ny_, rects, n, p_.coef, tn, stream);
  else
    stencilk_rects_gpu(p_.temporal, Tout, Tin, iCp_, nx_, ny_, rects, n, p_.coef, tn, stream);
}

void DiffusionExecutor::enqueue_step2(double* Tin, double* Tout) {
  if (p_.mode == Mode::kPerf) {
    TraceRange tr("rma.stepK.perf");
    multi_step(Tin, Tout, &out2_, 1, p_.tune2, s_lo_);
    exchange(Tout, s_lo_);
    return;
  }
  TraceRange tr("rma.stepK.hide");
  RMA_HIP_CHECK(hipStreamWaitEvent(S(s_hi_), E(e_lo_), 0));
  RMA_HIP_CHECK(hipStreamWaitEvent(S(s_lo_), E(e_hi_), 0));
  // frame tuning: the x-frames are ~2K columns wide, so the narrowest strip
  // (2 cells per lane: 128 columns) wastes the least recomputation, and the
  // interior's long row chunks keep the launch small; the frame still ends
  // long before the interior (1.6 of ~64 ms per pass at the 288 GB tile)
  StencilTuning ft = p_.tune2;
  ft.chunk_rows = std::min(ft.chunk_rows, 64);
  if (ft.kernel >= 6) ft.vec = std::min(ft.vec, 2);
  {
    TraceRange tb("rma.boundary");
    multi_step(Tin, Tout, frame2_.data(), (int)frame2_.size(), ft, s_hi_);
  }
  {
    TraceRange th("rma.halo");
    exchange(Tout, s_hi_);
  }
  RMA_HIP_CHECK(hipEventRecord(E(e_hi_), S(s_hi_)));
  if (!interior2_.empty()) {
    TraceRange ti("rma.interior");
    multi_step(Tin, Tout, &interior2_, 1, p_.tune2, s_lo_);
  }
  RMA_HIP_CHECK(hipEventRecord(E(e_lo_), S(s_lo_)));
}

void DiffusionExecutor::run_eager(int64_t nsteps) {
  for (int64_t i = 0; i < nsteps;) {
    if (p_.mode == Mode::kKp) {
      enqueue_step(T_, nullptr);
      ++steps_;
      ++i;
      continue;
    }
    double* Tin = parity_ ? T2_ : T_;
    double* Tout = parity_ ? T_ : T2_;
    const int64_t left = nsteps - i;
    if (p_.temporal > 1 && left >= p_.temporal) {
      enqueue_step2(Tin, Tout);
      steps_ += p_.temporal;
      i += p_.temporal;
    } else if (p_.temporal > 1 && left >= 2) {
      // remainder: one shorter pass (K' < K steps; the width-K exchange then
      // rewrites [K', K) with the identical values the neighbour owns)
      const int kr = left >= 12 ? 12 : left >= 8 ? 8 : left >= 6 ? 6 : left >= 4 ? 4
                     : left >= 3 ? 3 : 2;
      TraceRange tr("rma.stepK.rest");
      if (p_.mode == Mode::kHide) {  // previous pass done on both streams
        RMA_HIP_CHECK(hipStreamWaitEvent(S(s_lo_), E(e_hi_), 0));
      }
      Rect out = out2_;
      const auto& nb = halo_ ? halo_->neighbors() : std::array<std::array<int, 2>, 3>{};
      if (halo_) {
        out = {nb[0][0] >= 0 ? kr : 1, nx_ - (nb[0][1] >= 0 ? kr : 1), nb[1][0] >= 0 ? kr : 1,
               ny_ - (nb[1][1] >= 0 ? kr : 1)};
      }
      StencilTuning tn = p_.tune2;
      if (kr == 2 && !p_.fast_math) {
        tn.chunk_rows = 16;
        tn.xcd_remap = -1;
        stencil2_rects_gpu(Tout, Tin, iCp_, nx_, ny_, &out, 1, p_.coef, tn, s_lo_);
      } else {
        tn.xcd_remap = 1;
        tn.kernel = 3;
        if (p_.fast_math) {
          const StencilTuning f = fast_tune_k(kr, ny_, p_.coef);
          tn.kernel = f.kernel;
          tn.vec = f.vec;
        }
        stencilk_rects_gpu(kr, Tout, Tin, iCp_, nx_, ny_, &out, 1, p_.coef, tn, s_lo_);
      }
      exchange(Tout, s_lo_);
      if (p_.mode == Mode::kHide) {
        RMA_HIP_CHECK(hipEventRecord(E(e_lo_), S(s_lo_)));
        RMA_HIP_CHECK(hipStreamWaitEvent(S(s_hi_), E(e_lo_), 0));
        RMA_HIP_CHECK(hipEventRecord(E(e_hi_), S(s_hi_)));
      }
      steps_ += kr;
      i += kr;
    } else {
      // one step (also the remainder of a temporal run: with overlap 2K and
      // halo width K the single-step update + exchange stays consistent)
      enqueue_step(Tin, Tout);
      ++steps_;
      ++i;
    }
    parity_ ^= 1;
  }
}

void DiffusionExecutor::build_graph(int64_t steps) {
  if (graph_exec_) {
    (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(graph_exec_));
    graph_exec_ = nullptr;
  }
  if (halo_)  // pack buffers must exist before capture (no hipMalloc inside)
    halo_->prepare({field_of(T_, nx_, ny_, p_.olx, p_.oly, hwx_, hwy_)}, 3);
  hipStream_t lo = S(s_lo_), hi = S(s_hi_);
  const int saved_parity = parity_;
  const int64_t saved_steps = steps_;
  RMA_HIP_CHECK(hipStreamBeginCapture(lo, hipStreamCaptureModeThreadLocal));
  hipGraph_t g = nullptr;
  try {
    // fork hi into the capture
    RMA_HIP_CHECK(hipEventRecord(E(e_in_), lo));
    RMA_HIP_CHECK(hipStreamWaitEvent(hi, E(e_in_), 0));
    RMA_HIP_CHECK(hipEventRecord(E(e_hi_), hi));
    RMA_HIP_CHECK(hipEventRecord(E(e_lo_), lo));
    run_eager(steps);
    // join hi back
    RMA_HIP_CHECK(hipEventRecord(E(e_hi_), hi));
    RMA_HIP_CHECK(hipStreamWaitEvent(lo, E(e_hi_), 0));
  } catch (...) {
    // never leave a stream capturing: it would poison every later sync call
    hipGraph_t junk = nullptr;
    (void)hipStreamEndCapture(lo, &junk);
    if (junk) (void)hipGraphDestroy(junk);
    (void)hipGetLastError();
    parity_ = saved_parity;
    steps_ = saved_steps;
    throw;
  }
  RMA_HIP_CHECK(hipStreamEndCapture(lo, &g));
  hipGraphExec_t ge;
  RMA_HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  RMA_HIP_CHECK(hipGraphDestroy(g));
  graph_exec_ = ge;
  graph_len_ = steps;
  parity_ = saved_parity;  // capture enqueued nothing; restore bookkeeping
  steps_ = saved_steps;
}

void DiffusionExecutor::run(int64_t nsteps, stream_t caller_stream) {
  RMA_CHECK_ARG(nsteps >= 0, "nsteps=" << nsteps);
  if (nsteps == 0) return;
  hipStream_t caller = S(caller_stream);
  hipStream_t lo = S(s_lo_), hi = S(s_hi_);
  RMA_HIP_CHECK(hipEventRecord(E(e_in_), caller));
  RMA_HIP_CHECK(hipStreamWaitEvent(lo, E(e_in_), 0));
  RMA_HIP_CHECK(hipStreamWaitEvent(hi, E(e_in_), 0));
  // make the per-step cross-stream waits of kHide start from "caller done"
  RMA_HIP_CHECK(hipEventRecord(E(e_hi_), hi));
  RMA_HIP_CHECK(hipEventRecord(E(e_lo_), lo));
  int64_t left = nsteps;
  if (p_.use_graph) {
    int64_t gl = p_.graph_steps > 0 ? p_.graph_steps : 20;
    // keep the buffer parity of a replay neutral (K steps per swap)
    const int64_t q = 2 * p_.temporal;
    gl = (gl + q - 1) / q * q;
    if (left >= gl) {
      if (!graph_exec_ || graph_len_ != gl) build_graph(gl);
      while (left >= gl) {
        RMA_HIP_CHECK(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(graph_exec_), lo));
        steps_ += gl;
        left -= gl;
      }
      RMA_HIP_CHECK(hipEventRecord(E(e_lo_), lo));
      RMA_HIP_CHECK(hipStreamWaitEvent(hi, E(e_lo_), 0));
      RMA_HIP_CHECK(hipEventRecord(E(e_hi_), hi));
    }
  }
  run_eager(left);
  RMA_HIP_CHECK(hipEventRecord(E(e_hi_), hi));
  RMA_HIP_CHECK(hipEventRecord(E(e_lo_), lo));
  RMA_HIP_CHECK(hipStreamWaitEvent(caller, E(e_hi_), 0));
  RMA_HIP_CHECK(hipStreamWaitEvent(caller, E(e_lo_), 0));
}

}  // namespace rma
