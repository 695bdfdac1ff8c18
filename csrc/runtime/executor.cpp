#include "rma/executor.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <mutex>
#include <string>
#include <thread>
#include <utility>

#include "rma/config.h"
#include "rma/hip_check.h"
#include "rma/trace.h"

namespace rma {

namespace {
hipStream_t S(void* p) { return reinterpret_cast<hipStream_t>(p); }
hipEvent_t E(void* p) { return reinterpret_cast<hipEvent_t>(p); }

// Process-wide pool of (low, high)-priority stream pairs: an executor takes a
// free pair (or creates one, low priority first) and returns it when it is
// destroyed, so rebuilding executors (set_temporal, loopback ranks, tests)
// reuses the same HIP streams instead of creating new ones
// (RMA_DIAG exec_streams=pool, the default; profiles/stream_order_r2.json).
std::mutex g_pool_mu;
std::vector<std::pair<hipStream_t, hipStream_t>> g_pool;
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
  else if (ny < 32768) t.chunk_rows = K <= 8 ? (K == 8 ? 128 : 256) : 256;  // K>=12: c256
  else if (K >= 20 && ny >= 98304) t.chunk_rows = 3072;  // K=20/24: 73.3/84.3 vs 73.8/84.8 ms (c1536)
  else if (K >= 12 && ny >= 98304) t.chunk_rows = 1536;  // 288 GB tile: 63.8 vs 64.5 ms (c1024)
  else t.chunk_rows = K >= 8 ? 1024 : 512;
  return t;
}

StencilTuning fast_tune_k(int K, int64_t ny, const StencilCoef& c) {
  StencilTuning t = default_tune_k(std::max(K, 3), ny);
  t.xcd_remap = 1;
  if (!fast5_ok(c)) return canonical_tune_k(K, ny);
  t.kernel = 9;  // stage-pipelined fast5, any K (stencil_pipe.h)
  t.vec = 4;
  if (const int ch = pipe_chunk_rows(K, ny, false)) t.chunk_rows = ch;
  // factor rows in registers instead of the LDS ring, stage-0 prefetch by
  // LDS-DMA ("piper"): per pass at 101120^2 K=10..24 -0.7..-7 % (K=20 -2.2 %,
  // K=24 -1.5 %); at 16384^2 K=14..20 -0.7..-8.5 % but K=10 / 12 +12 / +7 %
  // (profiles/SUMMARY_r3.md), so K = 10..13 only on the large tile classes
  if ((K >= 14 || (K >= 10 && ny >= 65536)) && pipe_has(K, pipe_default_stages(K), 3))
    t.kernel = 12;
  // K = 24: piper without the in-level sched_barriers under the iterative-ILP
  // scheduler (kernel 22, stencil_pipe_r24.hip): -1.3 % per pass at 101376^2
  if (K == 24 && t.kernel == 12) t.kernel = 22;  // 9 + kArFast5RegNoSB
  // RMA_DIAG pipe_fast=pipe | pipe5 forces the ring kernel at every depth (A/B
  // runs; pipe5 = 5 cells per lane, lab library, K = 16..20 and nx % 5 == 0)
  static const std::string force = diag_value("pipe_fast");
  RMA_CHECK_ARG(force.empty() || force == "pipe" || force == "pipe5",
                "RMA_DIAG pipe_fast=" << force << " (pipe | pipe5)");
  if (force == "pipe" || force == "pipe5") t.kernel = 9;
  if (force == "pipe5") t.vec = 5;
  return t;
}

StencilTuning canonical_tune_k(int K, int64_t ny) {
  StencilTuning t = default_tune_k(K, ny);
  // kernel 3 wins at K = 3, 4; the canonical pipelined kernel from K = 5 on
  // (K=6: 47.2 vs 48.9 ms, K=8: 55.9 vs 59.8 ms per pass at 101376^2,
  // profiles/pass_sweep_r2.json)
  if (K >= 5) {
    t.kernel = 10;
    t.vec = 4;
    if (const int ch = pipe_chunk_rows(K, ny, true)) t.chunk_rows = ch;
  }
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
  RMA_CHECK_ARG(p.temporal >= 1 && p.temporal <= kPipeMaxK,
                "temporal (max steps per pass) must be 1.." << kPipeMaxK << ", got " << p.temporal);
  RMA_CHECK_ARG(p.temporal == 1 || p.mode != Mode::kKp,
                "temporal blocking applies to perf / perf_hide, not kp");
  RMA_CHECK_ARG(p.olx >= 2 && p.oly >= 2, "overlaps must be >= 2");
  RMA_CHECK_ARG(p.temporal == 1 || ny < (int64_t(1) << 30),
                "K-step passes index rows in 32 bits, ny = " << ny);
  hwx_ = hwy_ = p.temporal;  // halo width = steps per exchange
  if (halo) nbr_ = halo->neighbors();
  real_nbr_ = nbr_;
  const int64_t ol[2] = {p.olx, p.oly};
  for (int d = 0; d < 2; ++d)
    RMA_CHECK_ARG((nbr_[d][0] < 0 && nbr_[d][1] < 0) || ol[d] >= 2 * p.temporal,
                  "temporal=" << p.temporal << " needs a grid overlap >= " << 2 * p.temporal
                              << " along dim " << d << " (init_global_grid overlaps=2K, "
                              << "halowidths=K), got " << ol[d]);
  full_ = {1, nx - 1, 1, ny - 1};
  // perf_hide one-step updates: the frame must contain the send planes
  // [ol-hw, ol) of every side with a neighbour, so it is at least ol-1 cells wide (the
  // reference's b_width >= overlap invariant); minimal frames
  // otherwise (width 1 for ol=2: thin x-frames run in the kernel's column mode)
  if (p.mode == Mode::kHide) {
    RMA_CHECK_ARG(p.bwx >= 1 && p.bwy >= 1,
                  "b_width must be >= 1 so the send planes belong to the boundary kernel");
    const int64_t fx = std::max(p.bwx, p.olx - 1), fy = std::max(p.bwy, p.oly - 1);
    const auto side = frame_sides(nbr_);
    split_rect_sides(full_, side[0][0] ? fx : 0, side[0][1] ? fx : 0, side[1][0] ? fy : 0,
                     side[1][1] ? fy : 0, frame_, interior_);
  } else {
    interior_ = full_;
  }
  if (p.temporal > 1 || fast5()) {
    cost_ = default_pass_costs(p.temporal, fast5(), (double)nx * (double)ny);
    {  // RMA_DIAG pass_costs=K:cost/K:cost/...
      std::string pc = diag_value("pass_costs");
      for (char& ch : pc)
        if (ch == '/') ch = ',';
      apply_cost_overrides(cost_, pc.empty() ? nullptr : pc.c_str());
    }
    geom_.resize(p.temporal + 1);
    geom_ok_.assign(p.temporal + 1, 0);
    (void)geometry(p.temporal);  // throws now if the tile is too small
  }
  // the destructor does not run for a constructor that throws: from here on
  // what was acquired (streams, events, signal words) is released before the
  // exception leaves
  try {
  int least = 0, greatest = 0;
  RMA_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t hi, lo;
  // Streams come from a process-wide pool, created low priority first.
  // Mechanism (bench/probe_stream_order.py, rocprofv3 kernel trace with queue
  // ids, profiles/stream_order_r2.md): every new HIP stream of a process is
  // bound to the next hardware queue, and on MI355X / ROCm 7 the one-step
  // kernel (many short workgroups, dispatch-rate sensitive) dispatched from
  // the process's 5th queue ran 28 % slower (1.32 vs 1.03 ms at 16384^2).
  // With two executors alive, creating high-priority streams first put the
  // SECOND executor's interior stream on that queue (r1's "every second
  // executor 25 % slower"); low-priority first puts only its tiny frame
  // kernels there. The pool additionally reuses the streams of destroyed
  // executors (rebuilds, set_temporal), so no new queues accumulate.
  // RMA_DIAG exec_streams=lofirst|hifirst|plain create per executor (diagnostics).
  const std::string mode = diag_value("exec_streams", "pool");
  RMA_CHECK_ARG(mode == "pool" || mode == "lofirst" || mode == "hifirst" || mode == "plain",
                "RMA_DIAG exec_streams=" << mode << " (pool | lofirst | hifirst | plain)");
  if (mode == "pool") {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (!g_pool.empty()) {
      lo = g_pool.back().first;
      hi = g_pool.back().second;
      g_pool.pop_back();
    } else {
      RMA_HIP_CHECK(hipStreamCreateWithPriority(&lo, hipStreamNonBlocking, least));
      RMA_HIP_CHECK(hipStreamCreateWithPriority(&hi, hipStreamNonBlocking, greatest));
    }
    pooled_ = true;
  } else if (mode == "plain") {
    RMA_HIP_CHECK(hipStreamCreateWithFlags(&lo, hipStreamNonBlocking));
    RMA_HIP_CHECK(hipStreamCreateWithFlags(&hi, hipStreamNonBlocking));
  } else if (mode == "hifirst") {
    RMA_HIP_CHECK(hipStreamCreateWithPriority(&hi, hipStreamNonBlocking, greatest));
    RMA_HIP_CHECK(hipStreamCreateWithPriority(&lo, hipStreamNonBlocking, least));
  } else {
    RMA_HIP_CHECK(hipStreamCreateWithPriority(&lo, hipStreamNonBlocking, least));
    RMA_HIP_CHECK(hipStreamCreateWithPriority(&hi, hipStreamNonBlocking, greatest));
  }
  if (diag_flag("exec_verbose"))
    fprintf(stderr, "[executor] priority range least=%d greatest=%d mode=%s hi=%p lo=%p\n", least,
            greatest, mode.c_str(), (void*)hi, (void*)lo);
  s_hi_ = hi;
  s_lo_ = lo;
  for (void** e : {&e_hi_, &e_lo_, &e_in_, &e_fr_})  // straight into the members (release)
    RMA_HIP_CHECK(hipEventCreateWithFlags(reinterpret_cast<hipEvent_t*>(e), hipEventDisableTiming));
  // The interior of pass n+1 reads cells >= K away from the halo (its rect is
  // inset by the frame, >= ol - K = K cells) and writes the other buffer, so
  // it depends on pass n's frame and interior, not on pass n's exchange: with
  // the lag the exchange of pass n overlaps the interior of pass n+1 and only
  // pass n+1's frame (same stream as the exchange) waits for it.
  // RMA_DIAG no_lag: every pass waits for the previous exchange.
  lag_ = !diag_flag("no_lag");
  // Frame-first fused passes (see enqueue_pass). RMA_EXEC_FUSED=1 always (where
  // the frame is aligned), 0 never, auto (default): by task waves (fused_pass_ok).
  const std::string fu = env_choice("RMA_EXEC_FUSED", "auto|0|1", "auto");
  fused_ = fu == "auto" ? 2 : fu == "1" ? 1 : 0;
  // bounded wait of the exchange stream for the frame tasks' flag (seconds)
  fused_timeout_s_ = env_double("RMA_EXEC_FUSED_TIMEOUT", 60.0, 1e-9, 1e6);
  {
    int dev = 0, cus = 0;
    RMA_HIP_CHECK(hipGetDevice(&dev));
    RMA_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    cus_ = cus > 0 ? cus : 256;
  }
    if (fused_ && p_.mode == Mode::kHide) {
      RMA_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&sig_), 2 * sizeof(uint64_t)));
      // zeroed ON the executor's stream and waited for: a null-stream hipMemset
      // is not ordered before work on these non-blocking streams, and a counter
      // zeroed after (or never before) the first signalling launch never reaches
      // its target, so the frame wait times out (seen with 4 processes sharing
      // a GPU: the bench's shared-GPU rehearsal, profiles/SUMMARY_r5.md §6)
      RMA_HIP_CHECK(hipMemsetAsync(sig_, 0, 2 * sizeof(uint64_t), S(s_lo_)));
      RMA_HIP_CHECK(hipStreamSynchronize(S(s_lo_)));
      RMA_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&ferr_host_), sizeof(uint32_t),
                                  hipHostMallocMapped));
      *ferr_host_ = 0;
      RMA_HIP_CHECK(
          hipHostGetDevicePointer(reinterpret_cast<void**>(&ferr_dev_), ferr_host_, 0));
    }
    if (!diag_flag("no_prime")) prime();
  } catch (...) {
    release_resources();
    throw;
  }
}

DiffusionExecutor::~DiffusionExecutor() { release_resources(); }

void DiffusionExecutor::release_resources() {
  release_timing();
  if (graph_exec_) (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(graph_exec_));
  graph_exec_ = nullptr;
  for (void** e : {&e_hi_, &e_lo_, &e_in_, &e_fr_}) {
    if (*e) (void)hipEventDestroy(E(*e));
    *e = nullptr;
  }
  if (sig_ || ferr_host_) {  // the streams' flag kernels may still use them
    if (s_hi_) (void)hipStreamSynchronize(S(s_hi_));
    if (s_lo_) (void)hipStreamSynchronize(S(s_lo_));
    if (sig_) (void)hipFree(sig_);
    if (ferr_host_) (void)hipHostFree(ferr_host_);
    sig_ = nullptr;
    ferr_host_ = nullptr;
    ferr_dev_ = nullptr;
  }
  if (!s_hi_ && !s_lo_) return;
  if (pooled_) {  // back to the pool, drained
    (void)hipStreamSynchronize(S(s_hi_));
    (void)hipStreamSynchronize(S(s_lo_));
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_pool.emplace_back(S(s_lo_), S(s_hi_));
  } else {
    if (s_hi_) (void)hipStreamDestroy(S(s_hi_));
    if (s_lo_) (void)hipStreamDestroy(S(s_lo_));
  }
  s_hi_ = s_lo_ = nullptr;
}

bool DiffusionExecutor::fast5() const {
  return p_.fast_math && p_.mode != Mode::kKp && fast5_ok(p_.coef);
}

const PassGeom& DiffusionExecutor::geometry(int K) {
  RMA_CHECK_ARG(K >= 1 && K < (int)geom_.size(), "pass depth " << K);
  if (!geom_ok_[K]) {
    // pipelined passes: the frame is whole tasks of the interior's grid
    const StencilTuning t = pass_tuning(K, 0);
    int64_t tw = 0, th = 0;
    int vec = t.vec;
    if (t.kernel >= 9) {
      // the cells per lane the kernel will run (its strip step), not the request
      vec = pipe_vec(K, t.stages, t.kernel - 9, nx_, t.vec, true);
      tw = (64 * vec - 2 * K) / vec * vec;
      th = t.chunk_rows;
    }
    // direct-store halos: every pass writes the owned rect of the full halo
    // width, never the halo planes its neighbours store into (a pass of depth
    // K < hw would otherwise also write [K, hw))
    geom_[K] = pass_geometry(nx_, ny_, K, nbr_, p_.mode == Mode::kHide, p_.bwx, p_.bwy, p_.olx,
                             p_.oly, tw, th, vec, frame_layout(ny_, nbr_).bands,
                             direct_active() ? (int)std::max(hwx_, hwy_) : 0);
    geom_[K].task_w = tw;
    geom_[K].task_h = th;
    geom_ok_[K] = 1;
  }
  return geom_[K];
}

std::vector<int> DiffusionExecutor::plan(int64_t nsteps) const {
  if (p_.mode == Mode::kKp || cost_.empty()) return std::vector<int>((size_t)nsteps, 1);
  return plan_passes(nsteps, cost_);
}

StencilTuning DiffusionExecutor::pass_tuning(int K, int part) const {
  StencilTuning t = fast5() ? fast_tune_k(K, ny_, p_.coef) : canonical_tune_k(K, ny_);
  t.nontemporal = p_.tune2.nontemporal;
  if (p_.chunk_rows2 > 0) t.chunk_rows = p_.chunk_rows2;
  if (K == 2 && !fast5()) t.unroll = p_.tune2.unroll;
  if (part == 0) return t;
  if (t.kernel >= 9 && part == 1) {
    // pipelined passes, wide y-frames (~2K rows, full width): the interior's
    // 4 cells per lane (1.23x column recompute instead of 1.6x at 2 cells).
    // RCCL-self halo overhead at 16384^2, K=24: 8.7 -> 6.6 % per step; the
    // tall x-frames keep 2 cells per lane and 64-row chunks (longer chunks:
    // no gain at 16384^2, +0.2-0.3 % at the 288 GB tile, where each long
    // frame block holds CU slots for the interior's whole block time;
    // profiles/frame_tuning_r2.json)
    return t;
  }
  // tall x-frames, and every frame of the fixed-depth kernels (K <= 4
  // canonical): the narrowest strip and short chunks
  t.chunk_rows = std::min(t.chunk_rows, 64);
  if (t.kernel >= 6) t.vec = std::min(t.vec, 2);
  return t;
}

int DiffusionExecutor::frame_chunk_rows(int K, int interior_rows) const {
  // the aligned frame's tasks: 1/chunk_div of the interior's rows (plan.cpp
  // frame_layout: per tile class and neighbour set, measured)
  (void)K;
  return std::max(1, interior_rows / frame_layout(ny_, nbr_).chunk_div);
}

void DiffusionExecutor::exchange(double* A, stream_t s) {
  if (!halo_ || solo_) return;
  // diagnosis only (profiles/SUMMARY_r2.md, x-neighbour pass cost): keep the
  // geometry of a rank with neighbours but skip its exchange (wrong results;
  // bench.py records it and refuses it with the halo check on)
  static const bool skip = [] {
    const bool on = diag_flag("skip_exchange");
    if (on)
      fprintf(stderr, "[rocm_mpi_amd] WARNING: RMA_DIAG skip_exchange: every halo exchange is "
                      "skipped, multi-rank results are WRONG (diagnosis only)\n");
    return on;
  }();
  if (skip) return;
  HaloField f;
  f.ptr = A;
  f.size = {nx_, ny_, 1};
  f.elem_bytes = 8;
  f.ol = {p_.olx, p_.oly, 2};
  f.hw = {hwx_, hwy_, 1};
  // one-step passes only (temporal = 1): the 5-point update never reads a
  // corner halo cell, so all dimensions go in ONE RCCL group (one enqueue and
  // one RCCL kernel per exchange instead of two; RMA_DIAG no_halo_cross: per dimension).
  // K-step passes read the corners (diagonal dependencies) and keep the
  // dimension-ordered exchange.
  static const bool cross_ok = !diag_flag("no_halo_cross");
  // The last pass of a run() exchanges with exact corners, so the arrays a
  // run leaves behind have consistent corner halos (IGG update_halo! semantics).
  // With x AND y neighbours the exact exchange is ONE group with the corner
  // blocks sent to the diagonal neighbours (halo_plan.h plan_exchange_merged)
  // instead of one group per dimension (RMA_DIAG no_halo_merged: per dimension).
  static const bool merged_ok = !diag_flag("no_halo_merged");
  const bool xy = (nbr_[0][0] >= 0 || nbr_[0][1] >= 0) && (nbr_[1][0] >= 0 || nbr_[1][1] >= 0);
  if (cross_ok && cross_pass_ && p_.temporal == 1 && p_.mode != Mode::kKp)
    halo_->exchange_cross({f}, s, 3);
  else if (merged_ok && xy && halo_->has_diagonals())
    halo_->exchange_merged({f}, s);
  else
    halo_->exchange({f}, s, 3);
}

void DiffusionExecutor::enqueue_step(double* Tin, double* Tout) {
  const StencilCoef& c = p_.coef;
  if (p_.mode == Mode::kKp) {
    TraceRange tr("rma.step.kp");
    flux_gpu(qx_, qy_, Tin, nx_, ny_, c.mlam, c.rdx, c.rdy, s_lo_);
    residual_gpu(dTdt_, qx_, qy_, iCp_, nx_, ny_, c.rdx, c.rdy, s_lo_);
    update_gpu(Tin, dTdt_, nx_, ny_, c.dt, s_lo_);
    exchange(Tin, s_lo_);
    return;
  }
  void* ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  if (timing_) {
    for (auto& e : ev) e = tevent();
    if (ev[4]) tk_.push_back(1);
  }
  auto rec = [&](int i, void* stream) {
    if (ev[4]) RMA_HIP_CHECK(hipEventRecord(E(ev[i]), S(stream)));
  };
  if (p_.mode == Mode::kPerf || solo_) {
    TraceRange tr("rma.step.perf");
    if (p_.mode == Mode::kHide) {  // solo perf_hide: one launch, streams joined
      RMA_HIP_CHECK(hipStreamWaitEvent(S(s_lo_), E(e_hi_), 0));
    }
    rec(0, s_lo_);
    rec(3, s_lo_);
    stencil_rects_gpu(Tout, Tin, iCp_, nx_, ny_, &full_, 1, c, p_.tune, s_lo_);
    rec(4, s_lo_);
    rec(1, s_lo_);
    exchange(Tout, s_lo_);
    rec(2, s_lo_);
    if (ev[4]) tseq_.push_back(1);
    // the high stream stays idle (no per-step round trip between the queues);
    // a later overlapped step makes it wait for e_lo first
    if (p_.mode == Mode::kHide) RMA_HIP_CHECK(hipEventRecord(E(e_lo_), S(s_lo_)));
    return;
  }
  TraceRange tr("rma.step.hide");
  // the frame waits for the previous step on both streams; the interior for
  // the previous frame and interior (lag_: not the previous exchange)
  RMA_HIP_CHECK(hipStreamWaitEvent(S(s_hi_), E(e_lo_), 0));
  RMA_HIP_CHECK(hipStreamWaitEvent(S(s_lo_), E(lag_ ? e_fr_ : e_hi_), 0));
  // a transport that synchronises on the host (loopback, IPC) blocks in
  // exchange() until the frame is done: enqueue the interior first, so it
  // overlaps the frame and the exchange all the same (its dependencies were set
  // just above; the order of the two streams' launches changes nothing else)
  const bool interior_first = halo_ && !halo_->capturable();
  auto interior = [&]() {
    rec(3, s_lo_);
    if (!interior_.empty()) {
      TraceRange ti("rma.interior");
      stencil_rects_gpu(Tout, Tin, iCp_, nx_, ny_, &interior_, 1, c, p_.tune, s_lo_);
    }
    rec(4, s_lo_);
    RMA_HIP_CHECK(hipEventRecord(E(e_lo_), S(s_lo_)));
  };
  if (interior_first) interior();
  rec(0, s_hi_);
  StencilTuning ft = p_.tune;
  ft.chunk_rows = std::min(ft.chunk_rows, 16);
  if (!frame_.empty()) {  // no frame without a neighbour: the interior is the whole tile
    TraceRange tb("rma.boundary");
    stencil_rects_gpu(Tout, Tin, iCp_, nx_, ny_, frame_.data(), (int)frame_.size(), c, ft, s_hi_);
  }
  RMA_HIP_CHECK(hipEventRecord(E(e_fr_), S(s_hi_)));
  rec(1, s_hi_);
  {
    TraceRange th("rma.halo");
    exchange(Tout, s_hi_);
  }
  rec(2, s_hi_);
  RMA_HIP_CHECK(hipEventRecord(E(e_hi_), S(s_hi_)));
  if (!interior_first) interior();
  if (ev[4]) tseq_.push_back(0);
}

void DiffusionExecutor::multi_step(int K, double* Tin, double* Tout, const double* iCp,
                                   int64_t nx, int64_t ny, const Rect* rects, int n,
                                   const StencilTuning& tn, void* stream) const {
  if (K == 2 && tn.kernel < 5)  // dedicated two-step kernel: faster at K=2
    stencil2_rects_gpu(Tout, Tin, iCp, nx, ny, rects, n, p_.coef, tn, stream);
  else
    stencilk_rects_gpu(K, Tout, Tin, iCp, nx, ny, rects, n, p_.coef, tn, stream);
}

bool DiffusionExecutor::fused_pass_ok(const PassGeom& g, const StencilTuning& tn) const {
  if (!sig_ || !g.aligned || tn.kernel < 9 || g.interior.empty()) return false;
  int nf = 0;
  for (const Rect& r : g.frame) nf += r.empty() ? 0 : 1;
  if (nf == 0 || (int)g.frame.size() + 1 > kMaxRects) return false;
  // auto: with more than one wave of tasks per pass (2 blocks of 4 waves per
  // CU at K = 10..24). Within one wave every task runs at once, the frame
  // tasks end with the whole launch and the exchange is exposed; the split
  // launches win there. RCCL-self x+y at K=24, equal coefficients
  // (profiles/r5/fused/): 2048^2 (~430 tasks) 44 % split vs 50 % fused, 4096^2
  // (440) 1.2 vs 8.7 %; 5120^2 (675) 12.2 vs 2.7 %, 6144^2 (720) 11.3 vs 2.0 %,
  // 7168^2 (980) 11.1 vs 0.4 %, 8192^2 5.6 vs 1.3 %
  return fused_ == 1 || g.tasks() > 2 * (int64_t)cus_;
}

template <typename Launch>
void DiffusionExecutor::enqueue_fused(const std::vector<Rect>& frame, const Rect& interior,
                                      StencilTuning tn, double* Tout, void* const* ev,
                                      Launch&& launch) {
  ++fused_passes_;
  auto rec = [&](int i, void* stream) {
    if (ev[4]) RMA_HIP_CHECK(hipEventRecord(E(ev[i]), S(stream)));
  };
  // the whole launch waits for the previous exchange (its frame tasks read the
  // halo) and, in stream order, for the previous launch
  RMA_HIP_CHECK(hipStreamWaitEvent(S(s_lo_), E(e_hi_), 0));
  // direct-store halos: every neighbour's frame of the previous pass is done
  // (our halo complete, its field free for our stores)
  const bool dr = direct_remote();
  if (dr) direct_wait(direct_pass_, s_lo_);
  Rect rs[kMaxRects];
  int n = 0;
  for (const Rect& r : frame) rs[n++] = r;
  tn.signal = sig_;
  tn.signal_rects = n;
  rs[n++] = interior;
  rec(0, s_hi_);
  rec(3, s_lo_);
  {
    TraceRange ti("rma.fused");
    launch(rs, n, tn);
  }
  rec(4, s_lo_);
  RMA_HIP_CHECK(hipEventRecord(E(e_lo_), S(s_lo_)));
  // exchange stream: the frame flag (bounded wait), lowered for the next pass
  flag_wait_gpu(sig_ + 1, 1, fused_timeout_s_, ferr_dev_, 1, s_hi_);
  flag_write_gpu(sig_ + 1, 0, s_hi_);
  RMA_HIP_CHECK(hipEventRecord(E(e_fr_), S(s_hi_)));
  rec(1, s_hi_);
  {
    TraceRange th("rma.halo");
    if (dr)  // the images are stored: raise our pass count at the neighbours
      flags_write_gpu(dout_, direct_pass_ + 1, s_hi_);
    else
      exchange(Tout, s_hi_);
  }
  rec(2, s_hi_);
  RMA_HIP_CHECK(hipEventRecord(E(e_hi_), S(s_hi_)));
  if (ev[4]) tseq_.push_back(0);
}

void DiffusionExecutor::check_fused_error() const {
  if (!ferr_host_) return;
  const uint32_t e = __atomic_load_n(ferr_host_, __ATOMIC_ACQUIRE);
  RMA_CHECK_ARG(e != 1, "frame-first fused pass: the exchange stream's wait for the frame tasks "
                        "timed out after "
                            << fused_timeout_s_
                            << " s (RMA_EXEC_FUSED_TIMEOUT); the halos of that pass are wrong");
  RMA_CHECK_ARG(e == 0, "direct-store halos: the wait for a neighbour's pass count timed out "
                        "after "
                            << fused_timeout_s_
                            << " s (RMA_EXEC_FUSED_TIMEOUT; a neighbour died or runs another "
                               "plan); the halos of that pass are wrong");
}

void DiffusionExecutor::ensure_error_word() {
  if (ferr_host_) return;
  RMA_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&ferr_host_), sizeof(uint32_t),
                              hipHostMallocMapped));
  *ferr_host_ = 0;
  RMA_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ferr_dev_), ferr_host_, 0));
}

void DiffusionExecutor::direct_wait(uint64_t want, void* stream) {
  if (!dhost_) {
    flags_wait_ge_gpu(din_flags_, din_mask_, want, fused_timeout_s_, ferr_dev_, 2, stream);
    return;
  }
  // ranks of one process (host_wait): the host waits before enqueueing. A
  // spinning wait kernel per rank would share the process's few hardware
  // queues with the neighbours' passes it waits for (8 rank streams over
  // GPU_MAX_HW_QUEUES = 4) and could block them behind itself.
  const auto t0 = std::chrono::steady_clock::now();
  for (int d = 0; d < 8; ++d) {
    if (!((din_mask_ >> d) & 1u)) continue;
    while (__atomic_load_n(din_flags_ + d, __ATOMIC_ACQUIRE) < want) {
      const double dt =
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      RMA_CHECK_ARG(dt < fused_timeout_s_,
                    "direct-store halos: the host wait for the pass count of direction "
                        << d << " timed out after " << fused_timeout_s_
                        << " s (RMA_EXEC_FUSED_TIMEOUT; a neighbour died or runs another plan)");
      std::this_thread::yield();
    }
  }
}

void DiffusionExecutor::set_direct(const std::array<DirectPeer, 8>& peers, uint64_t* in_flags,
                                   bool host_wait) {
  RMA_HIP_CHECK(hipStreamSynchronize(S(s_hi_)));
  RMA_HIP_CHECK(hipStreamSynchronize(S(s_lo_)));
  bool any = false;
  uint32_t mask = 0;
  FlagTargets out{};
  const auto& nb = real_nbr_;
  const bool diag = halo_ && halo_->has_diagonals();
  for (int d = 0; d < 8; ++d) {
    const int i = kDirI[d], j = kDirJ[d];
    int want = -1;
    if (j == 0)
      want = nb[0][i > 0];
    else if (i == 0)
      want = nb[1][j > 0];
    else if (nb[0][i > 0] >= 0 && nb[1][j > 0] >= 0) {
      RMA_CHECK_ARG(diag, "direct-store halos with x and y neighbours need the diagonal ranks");
      want = halo_->diagonals()[(j > 0) * 2 + (i > 0)];
    }
    const DirectPeer& p = peers[d];
    RMA_CHECK_ARG(p.rank == want, "direct-store peer of direction (" << i << "," << j << "): rank "
                                      << p.rank << ", the grid's neighbour is " << want);
    if (p.rank < 0) continue;
    any = true;
    RMA_CHECK_ARG(p.T && p.T2, "direct-store peer (" << i << "," << j << "): null fields");
    if (p.T == T_) {  // this rank: its own periodic images, ordered by the stream
      RMA_CHECK_ARG(p.T2 == T2_, "direct-store self peer with another T2");
      continue;
    }
    RMA_CHECK_ARG(p.flag, "direct-store peer (" << i << "," << j << "): null pass-count word");
    mask |= 1u << d;
    out.dst[d] = p.flag;
    if (host_wait)  // the peer's words are pinned host memory: their device address
      RMA_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&out.dst[d]), p.flag, 0));
  }
  if (any) {
    RMA_CHECK_ARG(nx_ < (int64_t(1) << 30) && ny_ < (int64_t(1) << 30),
                  "direct-store halos: 32-bit image ranges");
    RMA_CHECK_ARG(p_.mode != Mode::kKp && fast5(),
                  "direct-store halos need fast-math K-step passes (pipelined kernels at every "
                  "depth)");
    RMA_CHECK_ARG(mask == 0 || in_flags, "direct-store halos with another rank need in_flags");
    ensure_error_word();
  }
  dpeer_ = peers;
  // price the depths for the planner: a depth whose direct-store kernel holds
  // fewer blocks per CU than the plain one (the register cap, stencil_pipe.h
  // pipe_kernel_dir) costs that much more per pass
  if (cost_base_.empty()) cost_base_ = cost_;
  cost_ = cost_base_;
  if (any) {
    const bool al = ((reinterpret_cast<uintptr_t>(T_) | reinterpret_cast<uintptr_t>(T2_) |
                      reinterpret_cast<uintptr_t>(iCp_)) & 15) == 0;
    for (int K = 1; K < (int)cost_.size(); ++K) {
      if (!std::isfinite(cost_[K])) continue;
      const StencilTuning t = pass_tuning(K, 0);
      if (t.kernel < 9) {  // no pipelined kernel at this depth: no direct-store variant
        cost_[K] = std::numeric_limits<double>::infinity();
        continue;
      }
      const int arith = t.kernel - 9;
      const int S = t.stages > 0 ? t.stages : pipe_default_stages(K);
      int occ[2] = {0, 0};
      stencil_pipe_occupancy(K, S, arith, pipe_vec(K, S, arith, nx_, t.vec, al), occ);
      if (occ[1] <= 0)
        cost_[K] = std::numeric_limits<double>::infinity();
      else if (occ[1] < occ[0])
        cost_[K] *= (double)occ[0] / occ[1];
    }
  }
  if (any) {  // the descriptors of both buffer parities
    dstores_[0] = direct_stores(false);
    dstores_[1] = direct_stores(true);
  }
  din_flags_ = in_flags;
  dhost_ = host_wait;
  din_mask_ = any ? mask : 0;
  dout_ = any ? out : FlagTargets{};
  direct_on_ = any;
  direct_pass_ = 0;
  std::fill(geom_ok_.begin(), geom_ok_.end(), 0);  // pass rects follow direct_active()
  if (graph_exec_) {  // captured with the exchange
    (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(graph_exec_));
    graph_exec_ = nullptr;
  }
}

bool DiffusionExecutor::images_in_frame(const PassGeom& g) const {
  // the image strips (clamped to the pass's output) minus the frame rects
  // (disjoint) must be empty: compare areas
  const DirectStores& D = dstores_[0];
  const Rect& o = g.out;
  auto clip = [&](Rect r) {
    r.x0 = std::max(r.x0, o.x0), r.x1 = std::min(r.x1, o.x1);
    r.y0 = std::max(r.y0, o.y0), r.y1 = std::min(r.y1, o.y1);
    return r;
  };
  auto area = [](const Rect& r) { return r.empty() ? 0 : (r.x1 - r.x0) * (r.y1 - r.y0); };
  bool side[4] = {false, false, false, false};  // any peer at i = -1, +1, j = -1, +1
  for (int d = 0; d < 8; ++d) {
    if (!dstores_[0].dst[d]) continue;
    if (kDirI[d] < 0) side[0] = true;
    if (kDirI[d] > 0) side[1] = true;
    if (kDirJ[d] < 0) side[2] = true;
    if (kDirJ[d] > 0) side[3] = true;
  }
  const Rect strips[4] = {{D.xm0, D.xm1, o.y0, o.y1}, {D.xp0, D.xp1, o.y0, o.y1},
                          {o.x0, o.x1, D.ym0, D.ym1}, {o.x0, o.x1, D.yp0, D.yp1}};
  for (int k = 0; k < 4; ++k) {
    if (!side[k]) continue;
    const Rect st = clip(strips[k]);
    int64_t in = 0;
    for (const Rect& f : g.frame) {
      Rect c = st;
      c.x0 = std::max(c.x0, f.x0), c.x1 = std::min(c.x1, f.x1);
      c.y0 = std::max(c.y0, f.y0), c.y1 = std::min(c.y1, f.y1);
      in += area(c);
    }
    if (in != area(st)) return false;
  }
  return true;
}

DirectStores DiffusionExecutor::direct_stores(bool out_is_T2) const {
  DirectStores D;
  // my cells whose images are the neighbours' halos: x columns [ol-hw, ol)
  // (i = -1), [n-ol, n-ol+hw) (i = +1), any stored column (i = 0); same in y.
  // The neighbour at (i, j) starts (n - ol) cells further: my (x, y) is its
  // (x - i (nx - olx), y - j (ny - oly))
  D.xm0 = (int32_t)(p_.olx - hwx_);
  D.xm1 = (int32_t)p_.olx;
  D.xp0 = (int32_t)(nx_ - p_.olx);
  D.xp1 = (int32_t)(nx_ - p_.olx + hwx_);
  D.ym0 = (int32_t)(p_.oly - hwy_);
  D.ym1 = (int32_t)p_.oly;
  D.yp0 = (int32_t)(ny_ - p_.oly);
  D.yp1 = (int32_t)(ny_ - p_.oly + hwy_);
  D.sx = nx_ - p_.olx;
  D.syr = ny_ - p_.oly;
  for (int d = 0; d < 8; ++d) {
    const DirectPeer& p = dpeer_[d];
    if (p.rank < 0) continue;
    D.dst[d] = out_is_T2 ? p.T2 : p.T;
    D.on = 1;
  }
  return D;
}

void DiffusionExecutor::enqueue_pass(int K, double* Tin, double* Tout) {
  const PassGeom& g = geometry(K);
  // direct-store halos: the launches that hold image cells (the one launch of
  // perf and of a one-wave tile, the frame launches of a split pass) run the
  // kernels' direct-store variant instead of an exchange after the pass; a
  // split pass's interior launch stays the plain kernel
  // A rank whose only direct peer is itself, on a tile of several task waves,
  // keeps the exchange (local copies): there the direct-store variant's slower
  // row loop costs more than the exchange it saves (periodic x+y K=24 8192^2:
  // +9 % vs +0 %); the stores win where the exchange latency is the pass (one
  // wave of tasks: 2048^2 +4 % vs +53 %). Other ranks always store.
  const bool dr = direct_remote();
  const bool da = direct_active() && (dr || g.tasks() <= 2 * (int64_t)cus_);
  struct DirectCount {  // counted however the pass is enqueued
    uint64_t& n;
    bool on;
    ~DirectCount() {
      if (on) ++n;
    }
  } dcount{direct_pass_, da};
  StencilTuning tn = pass_tuning(K, 0);
  auto with_direct = [&](StencilTuning t) {
    if (da) t.direct = &dstores_[Tout == T2_ ? 1 : 0];
    return t;
  };
  // every image cell lies in the frame rects (else the interior carries the
  // stores as well: correct, slower)
  const StencilTuning tin = da && !images_in_frame(g) ? with_direct(tn) : tn;
  auto dwait = [&](void* stream) {
    if (dr) direct_wait(direct_pass_, stream);
  };
  auto dpost = [&](void* stream) {
    if (dr) flags_write_gpu(dout_, direct_pass_ + 1, stream);
  };
  // timing events of this pass (nullptr when off)
  void* ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  if (timing_) {
    for (auto& e : ev) e = tevent();
    if (ev[4]) tk_.push_back(K);
  }
  auto rec = [&](int i, void* stream) {
    if (ev[4]) RMA_HIP_CHECK(hipEventRecord(E(ev[i]), S(stream)));
  };
  if (p_.mode == Mode::kPerf) {  // no frame; the exchange follows the pass
    TraceRange tr("rma.pass.perf");
    rec(0, s_lo_);
    rec(3, s_lo_);
    dwait(s_lo_);
    multi_step(K, Tin, Tout, iCp_, nx_, ny_, &g.out, 1, with_direct(tn), s_lo_);
    rec(4, s_lo_);
    rec(1, s_lo_);
    if (da)
      dpost(s_lo_);
    else
      exchange(Tout, s_lo_);
    rec(2, s_lo_);
    if (ev[4]) tseq_.push_back(1);
    return;
  }
  if (da && (!dr || g.frame.empty() || g.tasks() <= 2 * (int64_t)cus_)) {
    // direct stores to this rank's own periodic images, or tiles of one wave
    // of tasks: ONE launch of the direct-store kernel over the owned rect
    // (one wave: every task starts at once, so a frame launch beside the
    // interior's would end with the pass anyway and only add its latency:
    // 2048^2 periodic x+y at K=24 +3-5 % vs +39-61 % split), after the
    // neighbours' counts of the previous pass, our count raised after it.
    // Several waves with other ranks: the fused pass below (counts raised
    // when the frame tasks are done)
    TraceRange tr("rma.pass.direct");
    RMA_HIP_CHECK(hipStreamWaitEvent(S(s_lo_), E(e_hi_), 0));
    rec(0, s_lo_);
    rec(3, s_lo_);
    dwait(s_lo_);
    if (g.aligned && !g.interior.empty() && g.frame.size() + 1 <= (size_t)kMaxRects) {
      // the aligned frame rects first with shorter tasks: the tasks that
      // store images are the launch's slowest, and in one wave of tasks the
      // slowest sets the pass (idle block slots take the extra tasks)
      Rect rs[kMaxRects];
      int n = 0;
      for (const Rect& r : g.frame) rs[n++] = r;
      rs[n++] = g.interior;
      StencilTuning t = with_direct(tn);
      t.signal_rects = n - 1;
      t.signal_chunk_rows = frame_chunk_rows(K, tn.chunk_rows);
      multi_step(K, Tin, Tout, iCp_, nx_, ny_, rs, n, t, s_lo_);
    } else {
      multi_step(K, Tin, Tout, iCp_, nx_, ny_, &g.out, 1, with_direct(tn), s_lo_);
    }
    rec(4, s_lo_);
    rec(1, s_lo_);
    dpost(s_lo_);
    rec(2, s_lo_);
    RMA_HIP_CHECK(hipEventRecord(E(e_lo_), S(s_lo_)));
    if (ev[4]) tseq_.push_back(1);
    return;
  }
  if (g.frame.empty()) {
    // no neighbour (or solo): nothing to overlap, one launch on the low
    // stream. The high stream is left alone, so the wait below is on an event
    // it completed long ago: no per-pass dependency round trip between the two
    // queues (measured neutral at 2048^2-16384^2: the per-pass cost there is
    // the host launch, which --graph removes)
    TraceRange tr("rma.pass.hide");
    RMA_HIP_CHECK(hipStreamWaitEvent(S(s_lo_), E(e_hi_), 0));
    rec(0, s_lo_);
    rec(3, s_lo_);
    multi_step(K, Tin, Tout, iCp_, nx_, ny_, &g.interior, 1, tn, s_lo_);
    rec(4, s_lo_);
    rec(1, s_lo_);
    exchange(Tout, s_lo_);  // no-op without neighbours
    rec(2, s_lo_);
    RMA_HIP_CHECK(hipEventRecord(E(e_lo_), S(s_lo_)));
    if (ev[4]) tseq_.push_back(1);
    return;
  }
  if (fused_pass_ok(g, tn)) {
    // Frame-first fused pass: ONE launch of the pass's task grid, the frame
    // rects (whole tasks of the same grid) first in dispatch order and never
    // XCD-remapped, so they finish in the launch's first task wave; their last
    // block raises sig_[1]. The exchange stream waits for that flag on the GPU
    // (bounded, flags.hip), lowers it and exchanges while the rest of the
    // launch runs. No frame launch beside the interior's, no frame-sized second
    // grid. The next pass waits for this exchange (its frame tasks read the
    // halo) and, in stream order, for this launch.
    TraceRange tr("rma.pass.fused");
    enqueue_fused(g.frame, g.interior, with_direct(tn), Tout, ev,
                  [&](const Rect* rs, int n, const StencilTuning& t) {
                    multi_step(K, Tin, Tout, iCp_, nx_, ny_, rs, n, t, s_lo_);
                  });
    return;
  }
  TraceRange tr("rma.pass.hide");
  RMA_HIP_CHECK(hipStreamWaitEvent(S(s_hi_), E(e_lo_), 0));
  RMA_HIP_CHECK(hipStreamWaitEvent(S(s_lo_), E(lag_ ? e_fr_ : e_hi_), 0));
  // host-synchronising transport (loopback, IPC): interior first, see enqueue_step
  // (direct stores never block the host)
  const bool interior_first = !da && halo_ && !halo_->capturable();
  auto interior = [&]() {
    rec(3, s_lo_);
    if (!g.interior.empty()) {
      TraceRange ti("rma.interior");
      multi_step(K, Tin, Tout, iCp_, nx_, ny_, &g.interior, 1, tin, s_lo_);
    }
    rec(4, s_lo_);
    RMA_HIP_CHECK(hipEventRecord(E(e_lo_), S(s_lo_)));
  };
  if (interior_first) interior();
  rec(0, s_hi_);
  dwait(s_hi_);
  if (!g.frame.empty()) {
    TraceRange tb("rma.boundary");
    if (g.aligned) {  // whole tasks of the interior grid: one launch, its tuning
      // ...but round-robin over the XCDs: with ol-K-row bands the launch
      // mixes ~1000 short band tasks with the tall frames' few dozen long
      // task-column tasks, and the interior's XCD-contiguous order would put
      // all long ones on the last XCD, which then finishes its share of the
      // interior one task-wave late (+3 ms per K=24 pass at the 288 GB tile
      // with x and y neighbours; profiles/SUMMARY_r3.md)
      StencilTuning ft = with_direct(tn);
      ft.xcd_remap = 0;
      ft.chunk_rows = frame_chunk_rows(K, tn.chunk_rows);
      multi_step(K, Tin, Tout, iCp_, nx_, ny_, g.frame.data(), (int)g.frame.size(), ft, s_hi_);
    } else {
      const StencilTuning tw = with_direct(pass_tuning(K, 1)), tt = with_direct(pass_tuning(K, 2));
      if (!g.frame_wide.empty())
        multi_step(K, Tin, Tout, iCp_, nx_, ny_, g.frame_wide.data(), (int)g.frame_wide.size(),
                   tw, s_hi_);
      if (!g.frame_tall.empty())
        multi_step(K, Tin, Tout, iCp_, nx_, ny_, g.frame_tall.data(), (int)g.frame_tall.size(),
                   tt, s_hi_);
    }
  }
  RMA_HIP_CHECK(hipEventRecord(E(e_fr_), S(s_hi_)));
  rec(1, s_hi_);
  {
    TraceRange th("rma.halo");
    if (da)
      dpost(s_hi_);
    else
      exchange(Tout, s_hi_);
  }
  rec(2, s_hi_);
  RMA_HIP_CHECK(hipEventRecord(E(e_hi_), S(s_hi_)));
  if (!interior_first) interior();
  if (ev[4]) tseq_.push_back(0);
}

void* DiffusionExecutor::tevent() {
  constexpr size_t kMaxEvents = 5 * 8192;
  if (tused_ >= kMaxEvents) return nullptr;
  if (tused_ == tev_.size()) {
    hipEvent_t e;
    RMA_HIP_CHECK(hipEventCreate(&e));
    tev_.push_back(e);
  }
  return tev_[tused_++];
}

void DiffusionExecutor::release_timing() {
  for (void* e : tev_) (void)hipEventDestroy(E(e));
  tev_.clear();
  tk_.clear();
  tseq_.clear();
  tused_ = 0;
}

void DiffusionExecutor::set_timing(bool on) {
  RMA_HIP_CHECK(hipStreamSynchronize(S(s_hi_)));
  RMA_HIP_CHECK(hipStreamSynchronize(S(s_lo_)));
  tused_ = 0;
  tk_.clear();
  tseq_.clear();
  timing_ = on;
}

std::vector<PassTiming> DiffusionExecutor::timings() {
  RMA_HIP_CHECK(hipStreamSynchronize(S(s_hi_)));
  RMA_HIP_CHECK(hipStreamSynchronize(S(s_lo_)));
  check_fused_error();
  std::vector<PassTiming> out;
  for (size_t i = 0; i < tk_.size(); ++i) {
    hipEvent_t* e = reinterpret_cast<hipEvent_t*>(&tev_[5 * i]);
    float t[5] = {0, 0, 0, 0, 0};
    for (int j = 1; j < 5; ++j) RMA_HIP_CHECK(hipEventElapsedTime(&t[j], e[0], e[j]));
    PassTiming pt;
    pt.K = tk_[i];
    // sequential passes (perf, solo): the exchange starts after the kernel
    pt.frame_ms = tseq_[i] ? 0.0f : t[1];
    pt.halo_ms = t[2] - t[1];
    pt.interior_ms = t[4] - t[3];
    pt.pass_ms = std::max(t[2], t[4]);
    pt.exposed_halo_ms = std::max(0.0f, t[2] - t[4]);
    out.push_back(pt);
  }
  return out;
}

void DiffusionExecutor::set_solo(bool on) {
  RMA_HIP_CHECK(hipStreamSynchronize(S(s_hi_)));
  RMA_HIP_CHECK(hipStreamSynchronize(S(s_lo_)));
  if (on == solo_) return;
  solo_ = on;
  nbr_ = on ? Neighbors{{{-1, -1}, {-1, -1}, {-1, -1}}} : real_nbr_;
  std::fill(geom_ok_.begin(), geom_ok_.end(), 0);  // pass rects follow the neighbours
  if (graph_exec_) {
    (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(graph_exec_));
    graph_exec_ = nullptr;
  }
}

void DiffusionExecutor::prime() {
  if (p_.mode == Mode::kKp || (p_.temporal == 1 && !fast5())) return;
  // drain both streams first: the priming signal below raises and lowers the
  // same flag words a fused pass's exchange stream may still be waiting on
  RMA_HIP_CHECK(hipStreamSynchronize(S(s_hi_)));
  RMA_HIP_CHECK(hipStreamSynchronize(S(s_lo_)));
  // a tiny field with the same cells-per-lane class as the real one (nx mod 4)
  const int64_t tnx = 256 + nx_ % 4, tny = 64;
  const size_t bytes = (size_t)(tnx * tny) * sizeof(double);
  double* buf = nullptr;
  RMA_HIP_CHECK(hipMalloc(&buf, 3 * bytes));
  double *a = buf, *b = buf + tnx * tny, *ic = buf + 2 * tnx * tny;
  RMA_HIP_CHECK(hipMemsetAsync(buf, 0, 3 * bytes, S(s_lo_)));
  const Rect r{1, tnx - 1, 1, tny - 1};
  try {
    for (int K = 1; K <= p_.temporal; ++K) {
      if (!std::isfinite(cost_[K])) continue;
      if (K == 1 && !fast5()) {
        stencil_rects_gpu(b, a, ic, tnx, tny, &r, 1, p_.coef, p_.tune, s_lo_);
        continue;
      }
      multi_step(K, a, b, ic, tnx, tny, &r, 1, pass_tuning(K, 0), s_lo_);
      if (sig_ && K == p_.temporal) {  // the flag kernels' first launches, and a signal
        const Rect rr[2] = {Rect{1, tnx - 1, 1, 9}, Rect{1, tnx - 1, 9, tny - 1}};
        StencilTuning st = pass_tuning(K, 0);
        if (st.kernel >= 9) {
          st.signal = sig_;
          st.signal_rects = 1;
          multi_step(K, a, b, ic, tnx, tny, rr, 2, st, s_lo_);
          flag_wait_gpu(sig_ + 1, 1, fused_timeout_s_, ferr_dev_, 1, s_lo_);
          flag_write_gpu(sig_ + 1, 0, s_lo_);
        }
      }
      if (p_.mode == Mode::kHide)
        for (int part = 1; part <= 2; ++part)
          multi_step(K, a, b, ic, tnx, tny, &r, 1, pass_tuning(K, part), s_lo_);
    }
    RMA_HIP_CHECK(hipStreamSynchronize(S(s_lo_)));
  } catch (...) {
    (void)hipStreamSynchronize(S(s_lo_));
    (void)hipFree(buf);
    throw;
  }
  RMA_HIP_CHECK(hipFree(buf));
}

void DiffusionExecutor::run_eager(int64_t nsteps) {
  if (p_.mode == Mode::kKp) {
    for (int64_t i = 0; i < nsteps; ++i) {
      enqueue_step(T_, nullptr);
      ++steps_;
      ++passes_;
    }
    return;
  }
  const std::vector<int> passes =
      cost_.empty() ? std::vector<int>((size_t)nsteps, 1) : plan_passes(nsteps, cost_);
  // cross_pass_ is set per pass below; reset it however this loop ends (a
  // pass that throws must not leave later exchanges -- graph capture, the
  // next run -- on the one-group cross exchange with stale corners)
  struct ResetCross {
    bool& f;
    ~ResetCross() { f = false; }
  } reset_cross{cross_pass_};
  for (size_t pi = 0; pi < passes.size(); ++pi) {
    const int K = passes[pi];
    cross_pass_ = pi + 1 < passes.size();  // corners exact after the last pass
    double* Tin = parity_ ? T2_ : T_;
    double* Tout = parity_ ? T_ : T2_;
    if (K == 1 && !fast5()) {
      // one canonical step (with overlap 2K and halo width K the one-step
      // update + exchange stays consistent)
      enqueue_step(Tin, Tout);
    } else {
      enqueue_pass(K, Tin, Tout);
    }
    steps_ += K;
    ++passes_;
    parity_ ^= 1;
  }
}

void DiffusionExecutor::build_graph(int64_t steps, int reps) {
  if (graph_exec_) {
    (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(graph_exec_));
    graph_exec_ = nullptr;
  }
  if (halo_) {  // pack buffers must exist before capture (no hipMalloc inside)
    HaloField f;
    f.ptr = T_;
    f.size = {nx_, ny_, 1};
    f.elem_bytes = 8;
    f.ol = {p_.olx, p_.oly, 2};
    f.hw = {hwx_, hwy_, 1};
    halo_->prepare({f}, 3);
    if (halo_->has_diagonals()) halo_->prepare({f}, HaloExchanger::kMerged | 3);
    halo_->prepare({f}, 3);  // (a larger merged slot may have reallocated: re-plan)
  }
  hipStream_t lo = S(s_lo_), hi = S(s_hi_);
  const int saved_parity = parity_;
  const int64_t saved_steps = steps_, saved_passes = passes_;
  RMA_HIP_CHECK(hipStreamBeginCapture(lo, hipStreamCaptureModeThreadLocal));
  hipGraph_t g = nullptr;
  try {
    // fork hi into the capture
    RMA_HIP_CHECK(hipEventRecord(E(e_in_), lo));
    RMA_HIP_CHECK(hipStreamWaitEvent(hi, E(e_in_), 0));
    RMA_HIP_CHECK(hipEventRecord(E(e_hi_), hi));
    RMA_HIP_CHECK(hipEventRecord(E(e_fr_), hi));
    RMA_HIP_CHECK(hipEventRecord(E(e_lo_), lo));
    for (int r = 0; r < reps; ++r) run_eager(steps);
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
    passes_ = saved_passes;
    throw;
  }
  RMA_HIP_CHECK(hipStreamEndCapture(lo, &g));
  hipGraphExec_t ge;
  RMA_HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  RMA_HIP_CHECK(hipGraphDestroy(g));
  graph_exec_ = ge;
  graph_len_ = steps * reps;
  parity_ = saved_parity;  // capture enqueued nothing; restore bookkeeping
  steps_ = saved_steps;
  passes_ = saved_passes;
}

void DiffusionExecutor::run(int64_t nsteps, stream_t caller_stream) {
  RMA_CHECK_ARG(nsteps >= 0, "nsteps=" << nsteps);
  check_fused_error();
  if (nsteps == 0) return;
  hipStream_t caller = S(caller_stream);
  hipStream_t lo = S(s_lo_), hi = S(s_hi_);
  RMA_HIP_CHECK(hipEventRecord(E(e_in_), caller));
  RMA_HIP_CHECK(hipStreamWaitEvent(lo, E(e_in_), 0));
  RMA_HIP_CHECK(hipStreamWaitEvent(hi, E(e_in_), 0));
  // make the per-step cross-stream waits of kHide start from "caller done"
  RMA_HIP_CHECK(hipEventRecord(E(e_hi_), hi));
  RMA_HIP_CHECK(hipEventRecord(E(e_fr_), hi));
  RMA_HIP_CHECK(hipEventRecord(E(e_lo_), lo));
  int64_t left = nsteps;
  if (p_.use_graph && !direct_remote()) {
    // a replay must leave the buffer parity unchanged: capture the plan of gl
    // steps twice when it has an odd number of passes
    const int64_t gl = p_.graph_steps > 0 ? p_.graph_steps : 20;
    const int64_t np = (int64_t)plan(gl).size();
    const int reps = np % 2 ? 2 : 1;
    const int64_t glen = gl * reps;
    if (left >= glen) {
      if (!graph_exec_ || graph_len_ != glen) build_graph(gl, reps);
      while (left >= glen) {
        RMA_HIP_CHECK(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(graph_exec_), lo));
        steps_ += glen;
        passes_ += np * reps;
        left -= glen;
      }
      RMA_HIP_CHECK(hipEventRecord(E(e_lo_), lo));
      RMA_HIP_CHECK(hipStreamWaitEvent(hi, E(e_lo_), 0));
      RMA_HIP_CHECK(hipEventRecord(E(e_hi_), hi));
      RMA_HIP_CHECK(hipEventRecord(E(e_fr_), hi));
    }
  }
  run_eager(left);
  // direct-store halos: the field this run leaves is complete only once every
  // neighbour's frame of the last pass has stored into our halo (the caller
  // reads it: gather, checks, the next update_halo_; and a neighbour must not
  // store into a field its owner already released)
  if (direct_remote()) direct_wait(direct_pass_, hi);
  RMA_HIP_CHECK(hipEventRecord(E(e_hi_), hi));
  RMA_HIP_CHECK(hipEventRecord(E(e_lo_), lo));
  RMA_HIP_CHECK(hipStreamWaitEvent(caller, E(e_hi_), 0));
  RMA_HIP_CHECK(hipStreamWaitEvent(caller, E(e_lo_), 0));
}

}  // namespace rma
