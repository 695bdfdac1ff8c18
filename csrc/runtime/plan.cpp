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

// Pass time relative to one HBM sweep (the one-step march kernel: 39.5 ms at
// 101376^2), measured on MI355X: profiles/pass_sweep_r2.json (bench/pass_sweep.py,
// median of 3 interleaved rounds, the executor's kernel and chunk rows per
// depth). A pass costs at least the sweep plus the strip-overlap reads
// (~1.12-1.24 up to K=12); from K~13 the fp64 VALU work dominates, and
// K=17..24 run 5-6 levels per wave at 2 waves per SIMD.
constexpr double kFast5[] = {0,     1.230, 1.225, 1.209, 1.158, 1.242, 1.205, 1.192, 1.122,
                             1.140, 1.187, 1.222, 1.222, 1.319, 1.357, 1.400, 1.424, 1.730,
                             1.762, 1.836, 1.853, 2.023, 2.055, 2.124, 2.133};
// canonical: K=1 one-step march, 2 two-step kernel, 3/4 kernel 3 (lds_dpp),
// the rest the canonical pipelined kernel (K=13-15, 17-19, 21-23 interpolated;
// K=24 at 1 wave per SIMD)
constexpr double kCanon[] = {0,     1.000, 1.074, 1.141, 1.065, 1.208, 1.193, 1.374, 1.413,
                             1.637, 1.793, 1.872, 1.927, 2.096, 2.264, 2.433, 2.601, 2.758,
                             2.916, 3.073, 3.230, 3.641, 4.051, 4.462, 4.872};
}  // namespace

std::vector<double> default_pass_costs(int kmax, bool fast5) {
  RMA_CHECK_ARG(kmax >= 1, "kmax=" << kmax);
  std::vector<double> c(kmax + 1, kInf);
  const int nf = sizeof(kFast5) / sizeof(double) - 1, nc = sizeof(kCanon) / sizeof(double) - 1;
  for (int K = 1; K <= kmax; ++K) {
    if (fast5) {
      c[K] = K <= nf ? kFast5[K] : kFast5[nf] * (K * (256.0 / (256 - 2 * K))) /
                                       (nf * (256.0 / (256 - 2 * nf)));
    } else {
      c[K] = K <= nc ? kCanon[K] : kCanon[nc] * K / nc;  // (nc == kPipeMaxK today)
    }
  }
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
