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
// scripts/fit_pass_costs.py from profiles/pass_sweep_{101376,16384,8192,4096}_r2_final.json;
// canonical depths that were not swept are interpolated). fast5: the
// pipelined fast-math kernel at every K; canonical: K=1 one-step march, 2
// two-step kernel, 3/4 kernel 3, K >= 5 the canonical pipelined kernel.
// On the 288 GB tile a pass costs at least the sweep plus the strip-overlap
// reads up to K~12 and the fp64 arithmetic beyond; on smaller tiles the
// deeper passes fill the chip worse (best depth per step: 4096^2 and 8192^2
// 12, 16384^2 24 (16 within 2 %), 101376^2 24).
constexpr int kTables = 4;
constexpr double kTileCells[kTables] = {4096.0 * 4096, 8192.0 * 8192, 16384.0 * 16384,
                                        101376.0 * 101376};
constexpr double kFast5[kTables][25] = {
    {0, 1.104, 1.089, 1.099, 1.143, 1.174, 1.185, 1.272, 1.311, 1.502, 1.551, 1.625, 1.684,
     1.949, 2.042, 2.405, 2.529, 3.357, 3.447, 3.593, 3.591, 4.124, 4.266, 4.393, 4.477},
    {0, 1.462, 1.551, 1.591, 1.497, 1.493, 1.499, 1.494, 1.383, 1.443, 1.480, 1.540, 1.507,
     1.654, 1.760, 1.900, 2.036, 2.769, 2.823, 2.793, 2.746, 3.115, 3.161, 3.235, 3.281},
    {0, 1.379, 1.440, 1.417, 1.310, 1.356, 1.341, 1.336, 1.223, 1.282, 1.237, 1.254, 1.272,
     1.418, 1.406, 1.502, 1.522, 1.974, 1.877, 1.897, 1.923, 2.230, 2.221, 2.283, 2.236},
    {0, 1.234, 1.230, 1.214, 1.161, 1.232, 1.210, 1.198, 1.126, 1.152, 1.200, 1.227, 1.239,
     1.335, 1.367, 1.445, 1.473, 1.753, 1.764, 1.827, 1.824, 1.989, 2.028, 2.085, 2.099}};
constexpr double kCanon[kTables][25] = {
    {0, 1.000, 1.060, 1.090, 1.258, 1.359, 1.402, 1.841, 1.946, 2.296, 2.582, 2.696, 2.837,
     3.355, 3.873, 4.391, 4.909, 5.344, 5.779, 6.213, 6.648, 7.083, 7.518, 7.952, 8.387},
    {0, 1.000, 1.105, 1.412, 1.374, 1.464, 1.480, 1.552, 1.663, 1.958, 2.287, 2.362, 2.462,
     2.827, 3.192, 3.557, 3.922, 4.201, 4.480, 4.759, 5.038, 5.317, 5.596, 5.875, 6.154},
    {0, 1.000, 1.080, 1.284, 1.218, 1.338, 1.337, 1.361, 1.477, 1.753, 1.874, 1.885, 2.016,
     2.230, 2.444, 2.658, 2.872, 3.011, 3.150, 3.289, 3.428, 3.566, 3.705, 3.844, 3.983},
    {0, 1.000, 1.080, 1.143, 1.068, 1.208, 1.200, 1.401, 1.431, 1.650, 1.808, 1.882, 1.927,
     2.110, 2.293, 2.476, 2.659, 2.820, 2.981, 3.142, 3.303, 3.465, 3.626, 3.787, 3.948}};
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
