#include "rma/executor.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <utility>

#include "rma/hip_check.h"
#include "rma/trace.h"

namespace rma {

namespace {
hipStream_t S(void* p) { return reinterpret_cast<hipStream_t>(p); }
hipEvent_t E(void* p) { return reinterpret_cast<hipEvent_t>(p); }
}  // namespace

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
  full_ = {1, nx - 1, 1, ny - 1};
  if (p.mode == Mode::kHide) {
    RMA_CHECK_ARG(p.bwx >= 1 && p.bwy >= 1,
                  "b_width must be >= 1 so the send planes belong to the boundary kernel");
    // Minimal frames: the send planes are x = 1, nx-2 and y = 1, ny-2, so a
    // frame of width 1 suffices; thin x-frames run in the kernel's column
    // mode and the interior keeps 98-99.99% of the cells (profiles/).
    const int64_t xi0 = 1 + p.bwx, xi1 = nx - 1 - p.bwx;
    const int64_t yi0 = 1 + p.bwy, yi1 = ny - 1 - p.bwy;
    if (xi0 >= xi1 || yi0 >= yi1) {
      interior_ = {0, 0, 0, 0};
      frame_ = {full_};
    } else {
      interior_ = {xi0, xi1, yi0, yi1};
      frame_ = {{1, nx - 1, 1, yi0},
                {1, nx - 1, yi1, ny - 1},
                {1, xi0, yi0, yi1},
                {xi1, nx - 1, yi0, yi1}};
    }
  } else {
    interior_ = full_;
  }
  int least = 0, greatest = 0;
  RMA_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t hi, lo;
  RMA_HIP_CHECK(hipStreamCreateWithPriority(&hi, hipStreamNonBlocking, greatest));
  RMA_HIP_CHECK(hipStreamCreateWithPriority(&lo, hipStreamNonBlocking, least));
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

void DiffusionExecutor::exchange(double* A, stream_t s) {
  if (!halo_) return;
  HaloField f;
  f.ptr = A;
  f.size = {nx_, ny_, 1};
  f.elem_bytes = 8;
  f.ol = {2, 2, 2};
  f.hw = {1, 1, 1};
  halo_->exchange({f}, s, 3);
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

void DiffusionExecutor::run_eager(int64_t nsteps) {
  for (int64_t i = 0; i < nsteps; ++i) {
    if (p_.mode == Mode::kKp) {
      enqueue_step(T_, nullptr);
    } else {
      double* Tin = parity_ ? T2_ : T_;
      double* Tout = parity_ ? T_ : T2_;
      enqueue_step(Tin, Tout);
      parity_ ^= 1;
    }
    ++steps_;
  }
}

void DiffusionExecutor::build_graph(int64_t steps) {
  if (graph_exec_) {
    (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(graph_exec_));
    graph_exec_ = nullptr;
  }
  if (halo_) {  // pack buffers must exist before capture (no hipMalloc inside)
    HaloField f;
    f.ptr = T_;
    f.size = {nx_, ny_, 1};
    halo_->prepare({f}, 3);
  }
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
    if (gl % 2) ++gl;  // keep the buffer parity of a replay neutral
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
