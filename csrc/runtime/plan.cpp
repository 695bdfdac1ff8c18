#include "rma/config.h"
#include "rma/plan.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <limits>
#include <string>

namespace rma {

void split_rect_sides(const Rect& out, int64_t xlo, int64_t xhi, int64_t ylo, int64_t yhi,
                      std::vector<Rect>& frame, Rect& interior) {
  RMA_CHECK_ARG(xlo >= 0 && xhi >= 0 && ylo >= 0 && yhi >= 0,
                "frame widths " << xlo << "," << xhi << "," << ylo << "," << yhi);
  frame.clear();
  const int64_t xi0 = out.x0 + xlo, xi1 = out.x1 - xhi;
  const int64_t yi0 = out.y0 + ylo, yi1 = out.y1 - yhi;
  if (xi0 >= xi1 || yi0 >= yi1) {
    interior = {0, 0, 0, 0};
    if (!out.empty()) frame.push_back(out);
    return;
  }
  interior = {xi0, xi1, yi0, yi1};
  if (ylo > 0) frame.push_back({out.x0, out.x1, out.y0, yi0});
  if (yhi > 0) frame.push_back({out.x0, out.x1, yi1, out.y1});
  if (xlo > 0) frame.push_back({out.x0, xi0, yi0, yi1});
  if (xhi > 0) frame.push_back({xi1, out.x1, yi0, yi1});
}

void split_rect(const Rect& out, int64_t bwx, int64_t bwy, std::vector<Rect>& frame,
                Rect& interior) {
  RMA_CHECK_ARG(bwx >= 0 && bwy >= 0, "frame widths " << bwx << "," << bwy);
  split_rect_sides(out, bwx, bwx, bwy, bwy, frame, interior);
}

std::array<std::array<bool, 2>, 2> frame_sides(const Neighbors& nbr) {
  // Only a side that sends needs its cells before the exchange: a side
  // without a neighbour (open boundary) is computed by the interior launch.
  // RMA_DIAG frame_sides=all: every side once any neighbour exists (the r1-r2
  // layout, kept for A/B runs).
  static const bool fs_all = diag_value("frame_sides") == "all";
  const bool any = nbr[0][0] >= 0 || nbr[0][1] >= 0 || nbr[1][0] >= 0 || nbr[1][1] >= 0;
  const bool all = any && fs_all;
  std::array<std::array<bool, 2>, 2> on{};
  for (int d = 0; d < 2; ++d)
    for (int s = 0; s < 2; ++s) on[d][s] = all || nbr[d][s] >= 0;
  return on;
}

Rect owned_rect(int64_t nx, int64_t ny, int K, const Neighbors& nbr) {
  RMA_CHECK_ARG(K >= 1, "K=" << K);
  const Rect r{nbr[0][0] >= 0 ? K : 1, nx - (nbr[0][1] >= 0 ? K : 1), nbr[1][0] >= 0 ? K : 1,
               ny - (nbr[1][1] >= 0 ? K : 1)};
  RMA_CHECK_ARG(!r.empty(), "tile " << nx << "x" << ny << " too small for " << K
                                    << "-step passes");
  return r;
}

FrameLayout frame_layout(int64_t ny, const Neighbors& nbr) {
  const bool x = nbr[0][0] >= 0 || nbr[0][1] >= 0, y = nbr[1][0] >= 0 || nbr[1][1] >= 0;
  FrameLayout f;
  // 4096^2 class (one wave of tasks per K=24 pass): half-height frame tasks,
  // and with x AND y neighbours ol-K bands (whole-task-row bands at half
  // height overflow the wave: x+y 29.6 %). 8192^2 class (~2.5 waves): y only:
  // ol-K bands (8.2 -> 3.1 %); x and y: half-height frame tasks (8.2 -> 5.7-
  // 6.1 %, ol bands 6.1 %); x only: whole tasks (half height: 0.8 -> 6.2 %).
  // 2048^2 (47 -> 58 %) and >= 16384^2 (x+y 0.7 -> 5.8 %): whole tasks.
  if (ny >= 3072 && ny < 6144) {
    f.chunk_div = 2;
    if (x && y) f.bands = 0;
  } else if (ny >= 6144 && ny < 12288 && y) {
    if (x)
      f.chunk_div = 2;
    else
      f.bands = 0;
  }
  static const std::string cd = diag_value("frame_chunk_div");  // RMA_DIAG frame_chunk_div=N
  if (!cd.empty()) f.chunk_div = std::max(1, std::atoi(cd.c_str()));
  return f;
}

PassGeom pass_geometry(int64_t nx, int64_t ny, int K, const Neighbors& nbr, bool hide,
                       int64_t bwx, int64_t bwy, int64_t olx, int64_t oly, int64_t task_w,
                       int64_t task_h, int vec, int bands, int out_k) {
  PassGeom g;
  g.out = out_k > 0 ? owned_rect(nx, ny, out_k, nbr)
          : K == 1  ? Rect{1, nx - 1, 1, ny - 1}
                    : owned_rect(nx, ny, K, nbr);
  const bool any_nbr = nbr[0][0] >= 0 || nbr[0][1] >= 0 || nbr[1][0] >= 0 || nbr[1][1] >= 0;
  const Rect& o = g.out;
  const int64_t need_x = std::max(bwx, olx - o.x0), need_y = std::max(bwy, oly - o.y0);
  // Frame layout (perf_hide with a neighbour). Tall x-frames are whole strip
  // columns of the interior launch's task grid ("aligned": every frame cell
  // is computed once, with the interior's tuning and recompute). The y-bands
  // are whole task rows when tasks are short (<= 1024 rows) and only the ol-K
  // rows the exchange needs otherwise: a 3072-row task row would put 6 % of
  // the pass ahead of the exchange on the high-priority stream, and capping
  // the tasks at 1536 rows costs a rank ~1 % on its own. Measured RCCL-self
  // overhead at K=24 and EQUAL coefficients (dx = dy; the coefficients alone
  // move the power-capped pass by ~2 %, profiles/SUMMARY_r3.md), 288 GB tile:
  // x-periodic 0.35 % (tall task columns, 3072-row tasks) vs 1.3 % (1536-row
  // tasks) vs 1.7 % (128-column strips); y 0.4-0.7 % (ol-wide bands) vs
  // 1.6 % (task-row bands); smaller tiles (profiles/frame_aligned_r2.json):
  // 16384^2 5.7 -> 0.1 %, 32768^2 2.3-3.1 -> ~0 %, 65536^2 1.9-2.2 -> 0.1-0.4 %.
  // RMA_DIAG frame_aligned=0 / 1 forces the layout (0: ol-wide strips
  // everywhere); frame_bands=task / ol forces the band height.
  static const std::string fa = diag_value("frame_aligned");
  static const std::string fb = diag_value("frame_bands");
  const bool want = fa.empty() ? true : fa[0] != '0';
  const bool task_bands = !fb.empty() ? fb[0] == 't' : bands >= 0 ? bands == 1 : task_h <= 1024;
  const int64_t band = task_bands ? task_h : need_y;  // y-band height
  if (want && hide && any_nbr && task_w >= need_x && task_h >= 1 && band >= need_y &&
      o.x1 - o.x0 >= 3 * task_w && o.y1 - o.y0 >= (task_bands ? 3 * task_h : 2 * band + 1)) {
    // frame = the interior launch's first / last strip column (tall strips)
    // and its first / last task row, or the ol-K rows the exchange needs
    // (bands): every frame cell is computed once
    g.aligned = true;
    const auto side = frame_sides(nbr);
    const int64_t V = std::max(1, vec);
    auto floor_v = [&](int64_t a) { return a - (((a % V) + V) % V); };
    // left strip: exactly the first strip of the owned rect's grid
    const int64_t xl = side[0][0] ? floor_v(o.x0 - K) + K + task_w : o.x0;
    // right strip: starts where a strip's origin (start - K) is V-aligned and
    // its output still reaches x1
    int64_t xr = o.x1;
    if (side[0][1]) {
      xr = o.x1 - task_w;
      xr += ((V - ((xr - K) % V + V) % V) % V);
    }
    const int64_t yb = side[1][0] ? o.y0 + band : o.y0;
    const int64_t yt = side[1][1] ? o.y1 - band : o.y1;
    if (side[1][0]) g.frame_wide.push_back({o.x0, o.x1, o.y0, yb});
    if (side[1][1]) g.frame_wide.push_back({o.x0, o.x1, yt, o.y1});
    if (side[0][0]) g.frame_tall.push_back({o.x0, xl, yb, yt});
    if (side[0][1]) g.frame_tall.push_back({xr, o.x1, yb, yt});
    g.frame = g.frame_wide;
    g.frame.insert(g.frame.end(), g.frame_tall.begin(), g.frame_tall.end());
    g.interior = {xl, xr, yb, yt};
    return g;
  }
  if (hide && any_nbr) {
    int64_t fx = std::max(bwx, olx - g.out.x0);
    // the tall x-frames of a pipelined pass (K >= 5) run in 128-column strips
    // (2 cells per lane) that output 128 - 2K columns whatever the frame
    // width: widen the frame to that capacity, so those columns leave the
    // interior instead of being computed twice (RMA_DIAG no_frame_fill: off)
    static const bool fill = !diag_flag("no_frame_fill");
    if (K >= 5 && fill)
      fx = std::max<int64_t>(fx, std::min<int64_t>(128 - 2 * K, (g.out.x1 - g.out.x0) / 4));
    const int64_t fy = std::max(bwy, oly - g.out.y0);
    const auto side = frame_sides(nbr);
    split_rect_sides(g.out, side[0][0] ? fx : 0, side[0][1] ? fx : 0, side[1][0] ? fy : 0,
                     side[1][1] ? fy : 0, g.frame, g.interior);
    for (const Rect& r : g.frame)
      (r.x1 - r.x0 >= r.y1 - r.y0 ? g.frame_wide : g.frame_tall).push_back(r);
  } else {
    g.interior = g.out;
  }
  return g;
}

namespace {
constexpr double kInf = std::numeric_limits<double>::infinity();

// Pass time per depth K = 1..24 relative to the one-step march kernel on the
// same tile (one HBM sweep of the three arrays), measured on MI355X with the
// kernel the executor runs at each depth (bench/pass_sweep.py; emitted by
// scripts/fit_pass_costs.py from profiles/pass_sweep_{101376,16384,8192,4096}_r2_final.json;
// canonical depths that were not swept are interpolated). fast5: the
// pipelined fast-math kernel at every K; canonical: K=1 one-step march, 2
// two-step kernel, 3/4 kernel 3, K >= 5 the canonical pipelined kernel.
// On the 288 GB tile a pass costs at least the sweep plus the strip-overlap
// reads up to K~12 and the fp64 arithmetic beyond; on smaller tiles the
// deeper passes fill the chip worse. With the per-tile chunk table
// (pipe_chunk_rows) K=24 has the lowest time per step at every class
// (0.084-0.109 one-step units); the 288 GB row's K = 10..24 entries are scaled
// by the measured piper / pipe pass ratios (the executor's kernel there since
// round 3, profiles/r3/pass_sweep_piper_{lowK_101120,glds_boxE}.json; K = 11,
// 13, 15, 19 interpolated; scripts/fit_pass_costs.py apply_ratios); round 4: K = 17..20 of
// every class scaled by the measured unroll-by-6 / unroll-by-3 piper ratios (same box,
// profiles/r4/u6_{ab_all_stages,16384,8192,4096}.json); canonical: K=12 (K=20 at 101376^2), and
// K >= 21 canonical passes drop to one wave per SIMD (188 ms at 101376^2). Round 6: the
// fast5 K = 20 entry of the 288 GB row and the K = 24 entries of the 8192^2 / 16384^2 /
// 288 GB rows scaled by the measured scheduler / no-sched-barrier ratios
// (profiles/r6/sched_strategy_ab.md; scripts/fit_pass_costs.py r6_ratios: K = 20 x0.9886;
// K = 24 x0.9320 / x0.9975 / x0.9893).
constexpr int kTables = 4;
constexpr double kTileCells[kTables] = {4096.0 * 4096, 8192.0 * 8192, 16384.0 * 16384,
                                        101376.0 * 101376};
constexpr double kFast5[kTables][25] = {
    {0, 1.087, 1.056, 1.102, 1.123, 1.173, 1.169, 1.207, 1.228, 1.579, 1.404, 1.355, 1.379,
     1.598, 1.638, 1.745, 1.811, 2.056, 2.170, 2.198, 2.211, 2.553, 2.575, 2.617, 2.607},
    {0, 1.530, 1.519, 1.452, 1.377, 1.487, 1.432, 1.473, 1.334, 1.823, 1.414, 1.422, 1.391,
     1.488, 1.529, 1.745, 1.782, 2.259, 2.214, 2.176, 2.182, 2.390, 2.419, 2.434, 2.283},
    {0, 1.373, 1.375, 1.412, 1.298, 1.282, 1.275, 1.273, 1.217, 1.414, 1.326, 1.328, 1.294,
     1.410, 1.440, 1.605, 1.575, 1.896, 1.922, 1.885, 1.943, 2.101, 2.119, 2.168, 2.197},
    {0, 1.235, 1.230, 1.215, 1.163, 1.232, 1.210, 1.199, 1.126, 1.149, 1.138, 1.144, 1.119,
     1.244, 1.306, 1.371, 1.399, 1.595, 1.640, 1.676, 1.658, 1.886, 1.903, 1.971, 1.962}
};
constexpr double kCanon[kTables][25] = {
    {0, 1.000, 1.058, 1.095, 1.246, 1.335, 1.326, 1.757, 1.897, 2.226, 2.214, 2.295, 2.384,
     3.189, 3.233, 3.308, 3.355, 4.007, 4.073, 4.101, 4.158, 6.194, 6.136, 6.273, 6.421},
    {0, 1.000, 1.107, 1.406, 1.375, 1.462, 1.476, 1.646, 1.596, 1.830, 1.959, 2.005, 2.095,
     2.944, 3.023, 3.038, 3.010, 3.566, 3.589, 3.593, 3.659, 5.558, 5.537, 5.664, 5.745},
    {0, 1.000, 1.124, 1.382, 1.302, 1.444, 1.436, 1.451, 1.455, 1.733, 1.867, 1.889, 1.970,
     2.784, 2.772, 2.798, 2.857, 3.333, 3.319, 3.364, 3.467, 5.660, 5.443, 5.489, 5.591},
    {0, 1.000, 1.079, 1.146, 1.067, 1.212, 1.178, 1.362, 1.398, 1.597, 1.755, 1.833, 1.885,
     2.306, 2.383, 2.491, 2.533, 2.863, 2.947, 3.079, 3.131, 4.643, 4.586, 4.713, 4.770}};
}  // namespace

int pipe_chunk_rows(int K, int64_t ny, bool canonical) {
  if (ny < 1024) return 0;
  if (ny < 3072) {  // 2048^2 class: K=24 c48 0.083 vs 0.140 ms (the one-step rule's c16)
    if (canonical) return K <= 6 ? 16 : K <= 8 ? 32 : 48;
    return K <= 8 ? 16 : K <= 14 ? 32 : 48;
  }
  if (ny < 6144) {  // 4096^2 class
    if (canonical) return K <= 12 ? 64 : 192;
    return K <= 4 ? 32 : K <= 9 ? 64 : K <= 16 ? 128 : 192;
  }
  if (ny < 12288) {  // 8192^2
    if (canonical) return K <= 12 ? 128 : 256;
    return K <= 9 ? 256 : K <= 16 ? 128 : 256;
  }
  if (ny < 24576) {  // 16384^2 (12288^2: K=24 c512 within 2 % of the best)
    if (canonical) return K <= 9 ? 256 : K <= 12 ? 512 : 384;
    return K <= 4 ? 768 : K <= 9 ? 1536 : 512;
  }
  if (ny < 32768) {  // 24576^2: K=24 c768 5.07 vs 5.47 ms (the old c256)
    if (K <= 9) return 0;
    return canonical ? 512 : 768;
  }
  return 0;  // 32768^2 .. 101376^2: the r1 table is within 1-2 % of the best
}

std::vector<double> default_pass_costs(int kmax, bool fast5, double cells) {
  RMA_CHECK_ARG(kmax >= 1 && kmax <= 24, "kmax=" << kmax << " (tables cover 1..24)");
  // the measured tile class nearest in log(cells); 0 = the 288 GB tile
  int t = kTables - 1;
  if (cells > 0) {
    double best = 1e300;
    for (int i = 0; i < kTables; ++i) {
      const double d = std::fabs(std::log(cells / kTileCells[i]));
      if (d < best) {
        best = d;
        t = i;
      }
    }
  }
  std::vector<double> c(kmax + 1, kInf);
  for (int K = 1; K <= kmax; ++K) c[K] = fast5 ? kFast5[t][K] : kCanon[t][K];
  return c;
}

void apply_cost_overrides(std::vector<double>& cost, const char* spec) {
  if (!spec || !*spec) return;
  std::string s(spec);
  size_t pos = 0;
  while (pos < s.size()) {
    size_t end = s.find(',', pos);
    if (end == std::string::npos) end = s.size();
    const std::string item = s.substr(pos, end - pos);
    const size_t colon = item.find(':');
    RMA_CHECK_ARG(colon != std::string::npos, "pass_costs item '" << item << "' is not K:cost");
    const int K = std::atoi(item.substr(0, colon).c_str());
    const double v = std::atof(item.substr(colon + 1).c_str());
    RMA_CHECK_ARG(K >= 1 && K < (int)cost.size(), "pass_costs: K=" << K << " out of range");
    RMA_CHECK_ARG(v > 0, "pass_costs: cost must be > 0 (inf disables), got " << v);
    cost[K] = v;
    pos = end + 1;
  }
}

std::vector<int> plan_passes(int64_t n, const std::vector<double>& cost) {
  RMA_CHECK_ARG(n >= 0, "n=" << n);
  const int kmax = (int)cost.size() - 1;
  RMA_CHECK_ARG(kmax >= 1, "empty cost table");
  std::vector<int> out;
  if (n == 0) return out;
  // long runs: whole passes of the best steady-state depth first, the DP on
  // the last <= 4096 steps (the DP is O(n * Kmax))
  int kbest = 0;
  for (int K = 1; K <= kmax; ++K)
    if (std::isfinite(cost[K]) && (kbest == 0 || cost[K] / K < cost[kbest] / kbest)) kbest = K;
  RMA_CHECK_ARG(kbest > 0, "no pass depth available");
  int64_t rest = n;
  if (rest > 4096) {
    const int64_t q = (rest - 4096) / kbest;
    out.assign((size_t)q, kbest);
    rest -= q * kbest;
  }
  const int m = (int)rest;
  std::vector<double> best(m + 1, kInf);
  std::vector<int> pick(m + 1, 0), npass(m + 1, 0);
  best[0] = 0;
  for (int s = 1; s <= m; ++s) {
    for (int K = std::min(kmax, s); K >= 1; --K) {
      if (!std::isfinite(cost[K]) || !std::isfinite(best[s - K])) continue;
      const double v = best[s - K] + cost[K];
      const int np = npass[s - K] + 1;
      // strictly cheaper (beyond rounding noise), or as cheap with fewer passes
      if (v < best[s] - 1e-9 || (v <= best[s] + 1e-9 && np < npass[s])) {
        best[s] = v;
        pick[s] = K;
        npass[s] = np;
      }
    }
    RMA_CHECK_ARG(pick[s] > 0, "no pass sequence covers " << s << " steps");
  }
  for (int s = m; s > 0; s -= pick[s]) out.push_back(pick[s]);
  std::sort(out.begin(), out.end(), [](int a, int b) { return a > b; });
  return out;
}

}  // namespace rma
