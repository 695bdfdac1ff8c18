// Native time-loop executor for the diffusion variants.
//
// The reference drives every step from the host with a blocking wait after
// each kernel (scripts/diffusion_2D_perf.jl:49, diffusion_2D_kp.jl:88-90) and
// never overlaps communication (perf_hide's overlap is commented "not ready
// yet", diffusion_2D_perf_hide.jl:94-101). Here the whole loop is enqueued
// from C++ with stream ordering only:
//
//   kPerf : [fused stencil] -> [halo(T2)] -> swap                    (1 stream)
//   kHide : hi-prio stream: [frame rects] -> [halo(T2): pack, RCCL, unpack]
//           lo-prio stream: [interior rect]            (concurrently)
//           join both, swap. This is the reference's intended variant (3)
//           with exact frame/interior grids.
//   kKp   : [flux] -> [residual] -> [update T in place] -> [halo(T)]
//   temporal=K>1 (kPerf/kHide): each pass advances K steps with the K-step
//           kernel (stencil_tb.hip for K=2, stencil_tbk.hip otherwise) on the
//           "owned" rect (the K cells next to a neighbour are left to the
//           width-K exchange), then one exchange of width K (overlap 2K).
//
// Python never waits inside the loop; run() returns as soon as n steps are
// enqueued, ordered after the caller's stream and before its next work.
#pragma once

#include <array>
#include <cstdint>
#include <memory>
#include <vector>

#include "rma/halo.h"
#include "rma/kernels.h"

namespace rma {

enum class Mode : int { kPerf = 0, kHide = 1, kKp = 2 };

struct ExecParams {
  Mode mode = Mode::kPerf;
  StencilCoef coef{};
  StencilTuning tune{};
  int64_t bwx = 1, bwy = 1;    // perf_hide frame widths (cells beyond the boundary)
  int use_graph = 0;           // capture steps into a hipGraph and replay
  int graph_steps = 0;         // steps per captured graph (even; 0 = auto)
  // Temporal blocking (kPerf/kHide): K = 2, 3, 4, 6, 8 (12, 16 with fast_math)
  // time steps per kernel pass and one halo exchange of width K per pass;
  // needs a grid overlap >= 2K in every dimension with a neighbour. 1 = one
  // step per pass.
  int temporal = 1;
  int64_t olx = 2, oly = 2;    // grid overlaps of the field (IGG overlaps)
  StencilTuning tune2{16, 3, 0, 2, 2, -1};  // K-step kernel tuning (K=2: 16-row chunks)
  // fast_math: K-step passes use the 5-point-sum arithmetic with one folded
  // per-cell factor (stencil_tbk.hip kernel 5; kernel 4 if lam == 0): same
  // scheme in fp64, not bitwise equal to the canonical expression (rounding
  // level, tests/test_temporal_gpu.py).
  int fast_math = 0;
};

// Measured defaults of the K-step kernels (profiles/SUMMARY_r1.md): K=2 uses
// the aligned two-step kernel with 16-row chunks; K>=3 the overlapped-strip
// kernel with the LDS 1/Cp ring, per-XCD task ranges and chunks growing with
// the tile height (they amortise the 2K-1 rows recomputed per chunk).
StencilTuning default_tune_k(int K, int64_t ny);
// The fast-math K-step passes (fast_math, stencil_tbk.hip kernels 5-7; needs
// fast5_ok): K=16 runs the 4-stage pipelined kernel with 4 cells per lane, K=12
// the 2-stage one with 4 cells per lane, K<=8 the single-wave kernel 5
// (measured, profiles/SUMMARY_r1.md). Kernel 4 when the coefficients cannot be
// folded (lam == 0; K <= 8 only).
StencilTuning fast_tune_k(int K, int64_t ny, const StencilCoef& c);

class DiffusionExecutor {
 public:
  // T, T2, iCp: (ny, nx) device fields; qx/qy/dTdt only for kKp.
  DiffusionExecutor(double* T, double* T2, const double* iCp, int64_t nx, int64_t ny,
                    const ExecParams& p, HaloExchanger* halo, double* qx = nullptr,
                    double* qy = nullptr, double* dTdt = nullptr);
  ~DiffusionExecutor();
  DiffusionExecutor(const DiffusionExecutor&) = delete;
  DiffusionExecutor& operator=(const DiffusionExecutor&) = delete;

  // Enqueue n steps after the work already on caller_stream; caller_stream is
  // made to wait for them. Asynchronous.
  void run(int64_t nsteps, stream_t caller_stream);
  // Number of completed buffer swaps mod 2: 0 -> current field is T, 1 -> T2.
  int parity() const { return parity_; }
  int64_t steps_done() const { return steps_; }
  std::vector<Rect> frame_rects() const { return frame_; }
  Rect interior_rect() const { return interior_; }
  Rect full_rect() const { return full_; }

 private:
  void enqueue_step(double* Tin, double* Tout);
  void enqueue_step2(double* Tin, double* Tout);  // temporal=K: one K-step pass
  void multi_step(double* Tin, double* Tout, const Rect* rects, int n, const StencilTuning& tn,
                  void* stream);
  void exchange(double* A, stream_t s);
  void split(const Rect& out, int64_t bwx, int64_t bwy, std::vector<Rect>& frame,
             Rect& interior) const;
  void build_graph(int64_t steps);
  void run_eager(int64_t nsteps);

  double* T_;
  double* T2_;
  const double* iCp_;
  int64_t nx_, ny_;
  ExecParams p_;
  HaloExchanger* halo_;
  double *qx_, *qy_, *dTdt_;
  Rect full_{}, interior_{};
  std::vector<Rect> frame_;
  Rect out2_{}, interior2_{};  // temporal=K: owned rect and its interior
  std::vector<Rect> frame2_;
  int64_t hwx_ = 1, hwy_ = 1;
  void* s_hi_ = nullptr;  // hipStream_t
  void* s_lo_ = nullptr;
  void* e_hi_ = nullptr;  // hipEvent_t
  void* e_lo_ = nullptr;
  void* e_in_ = nullptr;
  void* graph_exec_ = nullptr;  // hipGraphExec_t
  int64_t graph_len_ = 0;
  int parity_ = 0;
  int64_t steps_ = 0;
};

}  // namespace rma
