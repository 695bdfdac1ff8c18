#include "rma/plan.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <limits>
#include <string>

namespace rma {

void split_rect(const Rect& out, int64_t bwx, int64_t bwy, std::vector<Rect>& frame,
                Rect& interior) {
  RMA_CHECK_ARG(bwx >= 0 && bwy >= 0, "frame widths " << bwx << "," << bwy);
  frame.clear();
  const int64_t xi0 = out.x0 + bwx, xi1 = out.x1 - bwx;
  const int64_t yi0 = out.y0 + bwy, yi1 = out.y1 - bwy;
  if (xi0 >= xi1 || yi0 >= yi1) {
    interior = {0, 0, 0, 0};
    if (!out.empty()) frame.push_back(out);
    return;
  }
  interior = {xi0, xi1, yi0, yi1};
  frame = {{out.x0, out.x1, out.y0, yi0},
           {out.x0, out.x1, yi1, out.y1},
           {out.x0, xi0, yi0, yi1},
           {xi1, out.x1, yi0, yi1}};
}

Rect owned_rect(int64_t nx, int64_t ny, int K, const Neighbors& nbr) {
  RMA_CHECK_ARG(K >= 1, "K=" << K);
  const Rect r{nbr[0][0] >= 0 ? K : 1, nx - (nbr[0][1] >= 0 ? K : 1), nbr[1][0] >= 0 ? K : 1,
               ny - (nbr[1][1] >= 0 ? K : 1)};
  RMA_CHECK_ARG(!r.empty(), "tile " << nx << "x" << ny << " too small for " << K
                                    << "-step passes");
  return r;
}

PassGeom pass_geometry(int64_t nx, int64_t ny, int K, const Neighbors& nbr, bool hide,
                       int64_t bwx, int64_t bwy, int64_t olx, int64_t oly) {
  PassGeom g;
  g.out = K == 1 ? Rect{1, nx - 1, 1, ny - 1} : owned_rect(nx, ny, K, nbr);
  const bool any_nbr = nbr[0][0] >= 0 || nbr[0][1] >= 0 || nbr[1][0] >= 0 || nbr[1][1] >= 0;
  if (hide && any_nbr) {
    split_rect(g.out, std::max(bwx, olx - g.out.x0), std::max(bwy, oly - g.out.y0), g.frame,
               g.interior);
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
// scripts/fit_pass_costs.py from profiles/pass_sweep{,_16384,_8192,_4096}_r2.json;
// canonical depths that were not swept are interpolated). fast5: the
// pipelined fast-math kernel at every K; canonical: K=1 one-step march, 2
// two-step kernel, 3/4 kernel 3, K >= 5 the canonical pipelined kernel.
// On the 288 GB tile a pass costs at least the sweep plus the strip-overlap
// reads up to K~12 and the fp64 arithmetic beyond; on smaller tiles the
// deeper passes fill the chip worse (4096^2: the best depth per step is 12,
// 16384^2: 16, 101376^2: 24).
constexpr int kTables = 4;
constexpr double kTileCells[kTables] = {4096.0 * 4096, 8192.0 * 8192, 16384.0 * 16384,
                                        101376.0 * 101376};
constexpr double kFast5[kTables][25] = {
    {0, 1.054, 1.111, 1.119, 1.128, 1.232, 1.223, 1.318, 1.366, 1.550, 1.512, 1.581, 1.645,
     1.898, 1.991, 2.264, 2.369, 3.249, 3.353, 3.464, 3.608, 4.101, 4.214, 4.338, 4.462},
    {0, 1.343, 1.406, 1.460, 1.365, 1.398, 1.337, 1.342, 1.274, 1.302, 1.347, 1.402, 1.423,
     1.586, 1.652, 1.796, 1.885, 2.696, 2.697, 2.680, 2.731, 3.221, 3.254, 3.312, 3.341},
    {0, 1.422, 1.503, 1.468, 1.361, 1.417, 1.377, 1.376, 1.268, 1.329, 1.273, 1.298, 1.284,
     1.408, 1.440, 1.499, 1.535, 2.014, 1.957, 1.964, 1.989, 2.225, 2.215, 2.279, 2.337},
    {0, 1.230, 1.225, 1.209, 1.158, 1.242, 1.205, 1.192, 1.122, 1.140, 1.187, 1.222, 1.222,
     1.319, 1.357, 1.400, 1.424, 1.730, 1.762, 1.836, 1.853, 2.023, 2.055, 2.124, 2.133}};
constexpr double kCanon[kTables][25] = {
    {0, 1.000, 1.071, 1.093, 1.188, 1.371, 1.421, 1.732, 1.884, 2.270, 2.514, 2.600, 2.758,
     3.244, 3.731, 4.217, 4.704, 5.102, 5.500, 5.899, 6.297, 6.695, 7.094, 7.492, 7.890},
    {0, 1.000, 1.070, 1.278, 1.261, 1.317, 1.332, 1.416, 1.588, 1.908, 2.195, 2.322, 2.395,
     2.754, 3.114, 3.473, 3.833, 4.111, 4.390, 4.669, 4.947, 5.226, 5.504, 5.783, 6.061},
    {0, 1.000, 1.088, 1.325, 1.248, 1.394, 1.380, 1.392, 1.425, 1.758, 1.862, 1.862, 1.951,
     2.200, 2.449, 2.697, 2.946, 3.105, 3.264, 3.423, 3.582, 3.740, 3.899, 4.058, 4.217},
    {0, 1.000, 1.074, 1.141, 1.065, 1.208, 1.193, 1.374, 1.413, 1.637, 1.793, 1.872, 1.927,
     2.096, 2.264, 2.433, 2.601, 2.758, 2.915, 3.073, 3.230, 3.640, 4.051, 4.461, 4.872}};
}  // namespace

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
    RMA_CHECK_ARG(colon != std::string::npos, "RMA_PASS_COSTS item '" << item << "' is not K:cost");
    const int K = std::atoi(item.substr(0, colon).c_str());
    const double v = std::atof(item.substr(colon + 1).c_str());
    RMA_CHECK_ARG(K >= 1 && K < (int)cost.size(), "RMA_PASS_COSTS: K=" << K << " out of range");
    RMA_CHECK_ARG(v > 0, "RMA_PASS_COSTS: cost must be > 0 (inf disables), got " << v);
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
