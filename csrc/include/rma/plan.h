// Host-only planning of the executor's kernel passes (no HIP): the rects a
// pass of K steps updates, the boundary-frame / interior split of perf_hide
// and the pass planner that decomposes n time steps into passes. Kept in a
// HIP-free translation unit so the sanitizer build (tests/native/
// host_selftest.cpp) runs it under ASan/UBSan.
#pragma once

#include <array>
#include <cstdint>
#include <vector>

#include "rma/common.h"

namespace rma {

using Neighbors = std::array<std::array<int, 2>, 3>;  // (dim, side) -> rank, -1 = none

// out minus a frame of widths (bwx, bwy): the 4 frame rects (lo-y, hi-y, lo-x,
// hi-x strips) and the interior. If the frame swallows the rect, frame = {out}
// and interior is empty.
void split_rect(const Rect& out, int64_t bwx, int64_t bwy, std::vector<Rect>& frame,
                Rect& interior);
// The same with one width per side (0: no frame rect on that side).
void split_rect_sides(const Rect& out, int64_t xlo, int64_t xhi, int64_t ylo, int64_t yhi,
                      std::vector<Rect>& frame, Rect& interior);

// Cells a K-step pass owns: next to a neighbour the K cells [0,K) are halo
// (level j of the pass is valid from column j on, so the pass outputs from
// column K; the width-hw exchange refreshes [0,hw) afterwards), elsewhere the
// fixed boundary cell 0 stays.
Rect owned_rect(int64_t nx, int64_t ny, int K, const Neighbors& nbr);

// Sides [dim][lo/hi] whose cells perf_hide computes ahead of the exchange:
// those with a neighbour (their send planes), all four under
// RMA_DIAG frame_sides=all (the r1-r2 layout, for A/B runs).
std::array<std::array<bool, 2>, 2> frame_sides(const Neighbors& nbr);

struct PassGeom {
  Rect out{};                // cells the pass writes
  std::vector<Rect> frame;   // perf_hide: computed first (high-priority stream)
  Rect interior{};           // perf_hide: the rest (low-priority stream)
  // the frame split by shape: wide (y-frames: full width, ~ol rows) and tall
  // (x-frames: ~ol columns, full height) strips run with different tunings
  std::vector<Rect> frame_wide, frame_tall;
  // aligned: the tall frames are whole strip columns of the interior's own
  // task grid (task_w given) and the bands whole task rows (task_h <= 1024)
  // or the ol-K rows the exchange needs (taller tasks), so frame + interior do
  // the work of ONE launch; frame launches then use the interior tuning
  bool aligned = false;
  // task grid of the pass's pipelined launch over `out` (0: not pipelined):
  // strip tasks of task_w output columns and task_h rows
  int64_t task_w = 0, task_h = 0;
  int64_t tasks() const {
    if (task_w <= 0 || task_h <= 0 || out.empty()) return 0;
    return ((out.x1 - out.x0 + task_w - 1) / task_w) * ((out.y1 - out.y0 + task_h - 1) / task_h);
  }
};

// Geometry of one pass. hide: split into frame + interior so that the frame
// holds the send planes [ol-hw, ol) of every side with a neighbour (width >= ol - out.x0, the
// reference's b_width >= overlap invariant); without any
// neighbour there is nothing to overlap and the owned rect is one launch.
// task_w / task_h > 0 (pipelined passes): output columns per strip and rows
// per chunk of the interior launch (strips start at x0 - K rounded down to
// `vec` cells, stencil_device.h plan_strip_tasks); the frame is then its
// first / last strip column and chunk row (a few % of the tile) instead of
// ol-wide strips, which a trapezoid kernel computes at several times the
// interior's cost per cell.
// bands: height of the aligned y-bands, -1 = the default / RMA_DIAG frame_bands,
// 0 = the ol-K rows the exchange needs, 1 = whole task rows.
// out_k > 0: the output rect is owned_rect(out_k) whatever K (direct-store
// halos: a pass never writes the halo planes [K, hw) its neighbours store).
PassGeom pass_geometry(int64_t nx, int64_t ny, int K, const Neighbors& nbr, bool hide,
                       int64_t bwx, int64_t bwy, int64_t olx, int64_t oly, int64_t task_w = 0,
                       int64_t task_h = 0, int vec = 1, int bands = -1, int out_k = 0);

// Aligned frame layout per tile class and neighbour set (perf_hide K-step
// passes, measured: RCCL-self overhead at K = 24, equal coefficients,
// profiles/SUMMARY_r4.md section 3): the frame launch's rows per task as a
// divisor of the interior's (chunk_div) and the y-band height (bands, as
// above). Below ~1 wave of tasks per pass every task runs concurrently, so a
// frame of whole interior tasks finishes with the interior and the exchange
// is exposed; half-height frame tasks finish at ~60 % of the pass (4096^2:
// x 10.5 -> 1.1 %, y 7.6 -> 3.1 %, x+y 17.6 -> 2.2 % with ol-K bands; 8192^2
// y 8.2 -> 3.1 % with ol-K bands).
// RMA_DIAG frame_chunk_div / frame_bands override.
struct FrameLayout {
  int chunk_div = 1;
  int bands = -1;
};
FrameLayout frame_layout(int64_t ny, const Neighbors& nbr);

// Relative cost of one pass of K steps (index K = 1..Kmax; index 0 unused;
// +inf = no kernel), in units of one HBM sweep of the 3 arrays. Measured on
// MI355X (profiles/pass_sweep*_r2.json); fast5 = the
// fast-math arithmetic (every K on the pipelined kernel), otherwise the
// canonical kernels (K = 1 one-step march, 2 two-step, 3/4 kernel 3,
// the rest the canonical pipelined kernel).
// cells = nx*ny of the tile (0: the 288 GB tile): the nearest measured tile
// class (4096^2, 8192^2, 16384^2, 101376^2) in log scale.
std::vector<double> default_pass_costs(int kmax, bool fast5, double cells = 0);
// RMA_DIAG pass_costs=K:cost/K:cost/... overrides entries (sweeps, tests;
// this function takes the entries comma-separated).
void apply_cost_overrides(std::vector<double>& cost, const char* spec);

// Rows per (strip, chunk) task of the pipelined K-step kernels (stencil_pipe.h)
// on a tile of ny rows, fast5 or canonical arithmetic: a chunk recomputes
// ~2K+S rows of overlap, so short chunks waste work on the deep passes while
// long ones leave small tiles with too few blocks. Measured best per tile
// class and depth (profiles/chunk_sweep_r2.json, bench/pass_sweep.py
// --chunks): 4096^2 K=24 192 rows (-38 % vs r1's 32), 8192^2 256 (-23 %),
// 16384^2 512 (-7 %); 0 = no table entry (the one-step kernels' rule).
int pipe_chunk_rows(int K, int64_t ny, bool canonical);

// Decompose n steps into passes of 1..Kmax steps minimising the summed cost
// (dynamic programme; ties -> fewer passes). Returned deepest first. E.g. the
// driver's 20 timed steps: one 20-step pass (~73 ms at the 288 GB tile)
// instead of 16 + 4 (~56 + 43 ms).
std::vector<int> plan_passes(int64_t n, const std::vector<double>& cost);

}  // namespace rma
