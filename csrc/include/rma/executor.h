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
//   temporal=K>1 (kPerf/kHide): run(n) plans passes of 1..K steps
//           (plan_passes: e.g. 20 steps = one 20-step pass, never 16 + 4);
//           a pass of k steps runs the k-step kernel (stencil_tb.hip k=2,
//           stencil_kstep.hip / stencil_pipe.h otherwise) on the "owned" rect
//           (the k cells next to a neighbour are left to the exchange), then
//           one exchange of width K (overlap 2K).
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
#include "rma/plan.h"

namespace rma {

enum class Mode : int { kPerf = 0, kHide = 1, kKp = 2 };

struct ExecParams {
  Mode mode = Mode::kPerf;
  StencilCoef coef{};
  StencilTuning tune{};
  int64_t bwx = 1, bwy = 1;    // perf_hide frame widths (cells beyond the boundary)
  int use_graph = 0;           // capture steps into a hipGraph and replay
  int graph_steps = 0;         // steps per captured graph (even; 0 = auto)
  // Temporal blocking (kPerf/kHide): at most K = temporal time steps per
  // kernel pass (1..kPipeMaxK) and one halo exchange of width K per pass;
  // needs a grid overlap >= 2K in every dimension with a neighbour. run(n)
  // splits n steps into passes of 1..K steps with plan_passes (rma/plan.h).
  int temporal = 1;
  int64_t olx = 2, oly = 2;    // grid overlaps of the field (IGG overlaps)
  StencilTuning tune2{16, 3, 0, 2, 2, -1};  // K-step kernel tuning (K=2: 16-row chunks)
  int chunk_rows2 = 0;         // K-step rows per task (0: default_tune_k per pass depth)
  // fast_math: every pass uses the fast5 arithmetic (5-point sum with one
  // folded per-cell factor, stencil_pipe.h), K = 1 included: same scheme in
  // fp64, not bitwise equal to the canonical expression (rounding level,
  // tests/test_pipe_gpu.py) but bitwise equal to its CPU twin.
  int fast_math = 0;
};

// Measured defaults of the K-step kernels (profiles/SUMMARY_r1.md): K=2 uses
// the aligned two-step kernel with 16-row chunks; K>=3 the overlapped-strip
// kernels with the LDS 1/Cp ring, per-XCD task ranges and chunks growing with
// the tile height (they amortise the 2K-1 rows recomputed per chunk).
StencilTuning default_tune_k(int K, int64_t ny);
// Kernel of a K-step pass: fast_math (and fast5_ok) -> the pipelined fast5
// kernel (9) with 4 cells per lane, at K >= 14 (K >= 10 from 65536 rows on) its
// register-factor variant (12, "piper"); canonical -> kernel 3 at K in
// {3,4,6,8}, the canonical pipelined kernel (10) at other K >= 3 (K = 1 and
// 2 have their own one- and two-step kernels).
StencilTuning fast_tune_k(int K, int64_t ny, const StencilCoef& c);
StencilTuning canonical_tune_k(int K, int64_t ny);

// Per-pass timing (set_timing): HIP events on the two streams, in ms from the
// pass start (after the cross-stream waits). frame: boundary-frame kernel
// (perf_hide with neighbours; 0 otherwise), halo: pack + RCCL group + unpack
// after it, interior: the interior launch(es). exposed_halo_ms: how long the
// exchange outlasted the interior (0 = fully hidden).
struct PassTiming {
  int K = 0;
  float frame_ms = 0, halo_ms = 0, interior_ms = 0, pass_ms = 0, exposed_halo_ms = 0;
};

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
  // Passes run(n) would launch (deepest first; K = 1 entries are one-step
  // updates).
  std::vector<int> plan(int64_t nsteps) const;
  const std::vector<double>& pass_costs() const { return cost_; }
  // Launch every kernel a run may use once on a tiny scratch field (first
  // launches stay out of timed regions); synchronous. Done by the constructor
  // unless RMA_DIAG=no_prime.
  void prime();
  // Record per-pass HIP events from now on (clears earlier records); read
  // them with timings() once the work is done (synchronises).
  void set_timing(bool on);
  std::vector<PassTiming> timings();
  // solo: run this tile as if it had no neighbour (no exchange, one launch per
  // pass over the whole interior) -- the same-run single-GPU reference of a
  // weak-scaling measurement (bench.py); the field is then NOT the
  // multi-rank solution. Off restores the real neighbours.
  void set_solo(bool on);
  bool solo() const { return solo_; }
  // Number of completed buffer swaps mod 2: 0 -> current field is T, 1 -> T2.
  int parity() const { return parity_; }
  int64_t steps_done() const { return steps_; }
  int64_t passes_done() const { return passes_; }
  // passes enqueued as frame-first fused launches (RMA_EXEC_FUSED)
  int64_t fused_passes() const { return fused_passes_; }
  // throws if a fused pass's bounded wait for its frame flag timed out (the
  // halos of that pass are wrong); also checked at every run() and timings()
  void check_error() const { check_fused_error(); }
  // Direct-store halos (kernels.h DirectStores), replacing the exchange: every
  // pass's pipelined kernel also stores the cells that are a neighbour's halo
  // straight into that neighbour's output field. peers[d] for the 8
  // directions d = (i, j) in kDirI / kDirJ order ((-1,-1), (0,-1), (1,-1),
  // (-1,0), (1,0), (-1,1), (0,1), (1,1); opposite(d) = 7 - d): the peer's
  // rank (-1: none, this rank: its own periodic images), its T / T2 (the same
  // roles as ours: every rank runs the same pass plan) and, for another rank,
  // the word of ITS in_flags that counts our passes. in_flags: this rank's 8
  // device words (zeroed, quiescent peers), in_flags[d] counted by the peer in
  // direction d. Pass n waits until every neighbour's count is >= n - 1 (its
  // frame of pass n - 1 is done: our halo of that pass is complete and it no
  // longer reads the field we are about to store into), then stores, and
  // raises its count to n at the neighbours once its frame tasks are done.
  // Needs fast-math K-step passes (pipelined kernels at every depth); no
  // hipGraph replay with another rank (the counts are pass numbers). An
  // all-(-1) peers array switches direct stores off (the halo exchange again).
  struct DirectPeer {
    int rank = -1;
    double* T = nullptr;
    double* T2 = nullptr;
    uint64_t* flag = nullptr;
  };
  static constexpr int kDirI[8] = {-1, 0, 1, -1, 1, -1, 0, 1};
  static constexpr int kDirJ[8] = {-1, -1, -1, 0, 0, 1, 1, 1};
  // host_wait: the ranks are threads of this process and in_flags / the
  // peers' words are pinned host memory; the host waits for the counts before
  // enqueueing a pass instead of a wait kernel on the stream (see direct_wait)
  void set_direct(const std::array<DirectPeer, 8>& peers, uint64_t* in_flags,
                  bool host_wait = false);
  bool direct() const { return direct_on_; }
  int64_t direct_passes() const { return direct_pass_; }
  std::vector<Rect> frame_rects() const { return frame_; }
  Rect interior_rect() const { return interior_; }
  Rect full_rect() const { return full_; }
  // Rects of a K-step pass with this rank's (or, solo, no) neighbours:
  // owned rect, frame (aligned: whole tasks of the interior's grid) and
  // interior (plan.h pass_geometry); cached per K.
  const PassGeom& geometry(int K);

 private:
  void enqueue_step(double* Tin, double* Tout);
  void enqueue_pass(int K, double* Tin, double* Tout);  // one K-step pass (K >= 2 or fast5)
  // kernel tuning of a K-step launch: part 0 = the interior / whole tile,
  // 1 = wide (y) frame strips, 2 = tall (x) frame strips
  StencilTuning pass_tuning(int K, int part = 0) const;
  // rows per task of the aligned frame launch (interior_rows: the interior's)
  int frame_chunk_rows(int K, int interior_rows) const;
  void multi_step(int K, double* Tin, double* Tout, const double* iCp, int64_t nx, int64_t ny,
                  const Rect* rects, int n, const StencilTuning& tn, void* stream) const;
  void exchange(double* A, stream_t s);
  bool cross_pass_ = false;  // this pass may use the one-group cross exchange (run_eager)
  void build_graph(int64_t steps, int reps);
  void run_eager(int64_t nsteps);
  bool fast5() const;

  double* T_;
  double* T2_;
  const double* iCp_;
  int64_t nx_, ny_;
  ExecParams p_;
  HaloExchanger* halo_;
  double *qx_, *qy_, *dTdt_;
  Neighbors nbr_{{{-1, -1}, {-1, -1}, {-1, -1}}};
  Rect full_{}, interior_{};
  std::vector<Rect> frame_;
  std::vector<PassGeom> geom_;   // index K (lazily filled)
  std::vector<char> geom_ok_;
  std::vector<double> cost_;     // index K: relative pass cost (plan_passes)
  std::vector<double> cost_base_;  // ...without the direct-store pricing (set_direct)
  int64_t hwx_ = 1, hwy_ = 1;
  void* s_hi_ = nullptr;  // hipStream_t
  void* s_lo_ = nullptr;
  void* e_hi_ = nullptr;  // hipEvent_t
  void* e_lo_ = nullptr;
  void* e_in_ = nullptr;
  // frame of the last overlapped pass done (s_hi, before its exchange): the
  // next pass's interior waits for this instead of the exchange (lag_)
  void* e_fr_ = nullptr;
  bool lag_ = true;
  // Frame-first fused passes (RMA_EXEC_FUSED): ONE pipelined launch per pass
  // with the frame rects' tasks dispatched first; they raise sig_[1] when all
  // are done and the exchange stream waits for that flag (flags.hip) instead
  // of a separate frame launch. sig_: 2 x u64 device words; ferr_*: mapped
  // host word the bounded flag wait reports a timeout into.
  int fused_ = 2;  // 0 off, 1 on, 2 auto (>= 2 waves of tasks)
  int cus_ = 256;  // compute units of the device
  int64_t fused_passes_ = 0;
  double fused_timeout_s_ = 60.0;
  uint64_t* sig_ = nullptr;
  uint32_t* ferr_host_ = nullptr;
  uint32_t* ferr_dev_ = nullptr;
  bool fused_pass_ok(const PassGeom& g, const StencilTuning& tn) const;
  // the frame-first fused pass around `launch(rects, n, tuning)`: one launch
  // of the frame rects + interior on the low stream, the frame-flag wait and
  // the exchange on the high one (tn gets the signal fields)
  template <typename Launch>
  void enqueue_fused(const std::vector<Rect>& frame, const Rect& interior, StencilTuning tn,
                     double* Tout, void* const* ev, Launch&& launch);
  void check_fused_error() const;
  // direct-store halos (set_direct)
  bool direct_on_ = false;
  std::array<DirectPeer, 8> dpeer_{};
  uint64_t* din_flags_ = nullptr;
  uint32_t din_mask_ = 0;      // directions with another rank (flags to wait on)
  FlagTargets dout_{};         // the neighbours' words counting our passes
  uint64_t direct_pass_ = 0;   // passes done in direct mode
  bool dhost_ = false;         // host waits for the counts (set_direct host_wait)
  void direct_wait(uint64_t want, void* stream);
  bool direct_active() const { return direct_on_ && !solo_; }
  bool direct_remote() const { return direct_active() && din_mask_ != 0; }
  DirectStores direct_stores(bool out_is_T2) const;
  bool images_in_frame(const PassGeom& g) const;
  DirectStores dstores_[2];  // [out is T2]
  void ensure_error_word();
  void* graph_exec_ = nullptr;  // hipGraphExec_t
  int64_t graph_len_ = 0;
  int parity_ = 0;
  int64_t steps_ = 0;
  int64_t passes_ = 0;
  bool solo_ = false;
  bool pooled_ = false;  // streams borrowed from the process-wide pool
  Neighbors real_nbr_{{{-1, -1}, {-1, -1}, {-1, -1}}};
  // timing: 5 events per pass (start, frame end, halo end on hi; interior
  // start, end on lo)
  bool timing_ = false;
  std::vector<void*> tev_;
  std::vector<int> tk_;
  std::vector<char> tseq_;  // 1: sequential pass (exchange after the kernel)
  size_t tused_ = 0;
  void* tevent();
  void release_timing();
  void release_resources();  // destructor and a throwing constructor
};

}  // namespace rma
