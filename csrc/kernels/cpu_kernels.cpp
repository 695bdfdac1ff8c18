// Host (CPU) twins of the GPU kernels. Same expressions, same operation order,
// compiled with -ffp-contract=off, so CPU and GPU results agree bitwise (the
// exp() of init_gaussian excepted: libm vs OCML may differ by one ulp).
// These serve the CPU array path (BASELINE.json configs[0]: "ap 256x256 fp64
// single-rank CPU array path") and multi-rank CPU runs over gloo.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

#include <vector>

#include "rma/kernels.h"
#include "rma/parallel_for.h"

namespace rma {

namespace {
inline double cell(double xl, double c, double xr, double up, double dn, double ic,
                   const StencilCoef& k) {
  const double qxR = (k.mlam * (xr - c)) * k.rdx;
  const double qxL = (k.mlam * (c - xl)) * k.rdx;
  const double qyU = (k.mlam * (dn - c)) * k.rdy;
  const double qyD = (k.mlam * (c - up)) * k.rdy;
  return c + k.dt * (ic * ((-(qxR - qxL)) * k.rdx - (qyU - qyD) * k.rdy));
}
}  // namespace

void stencil_rects_cpu(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                       const Rect* rects, int nrects, const StencilCoef& c) {
  RMA_CHECK_ARG(nrects >= 0 && nrects <= kMaxRects, "nrects=" << nrects);
  for (int i = 0; i < nrects; ++i) {
    const Rect r = rects[i];
    if (r.empty()) continue;
    RMA_CHECK_ARG(r.x0 >= 1 && r.x1 <= nx - 1 && r.y0 >= 1 && r.y1 <= ny - 1,
                  "rect outside interior");
    parallel_for(r.y0, r.y1, 64, [&](int64_t y) {
      const double* up = T + (y - 1) * nx;
      const double* cu = T + y * nx;
      const double* dn = T + (y + 1) * nx;
      const double* ic = iCp + y * nx;
      double* out = T2 + y * nx;
      for (int64_t x = r.x0; x < r.x1; ++x)
        out[x] = cell(cu[x - 1], cu[x], cu[x + 1], up[x], dn[x], ic[x], c);
    });
  }
}

void stencil2_rects_cpu(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                        const Rect* rects, int nrects, const StencilCoef& c) {
  RMA_CHECK_ARG(T2 != T, "two-step update cannot run in place");
  std::vector<double> S1(T, T + nx * ny);  // step 1 on the interior, T elsewhere
  const Rect interior{1, nx - 1, 1, ny - 1};
  stencil_rects_cpu(S1.data(), T, iCp, nx, ny, &interior, 1, c);
  stencil_rects_cpu(T2, S1.data(), iCp, nx, ny, rects, nrects, c);
}

void stencilk_rects_cpu(int K, double* T2, const double* T, const double* iCp, int64_t nx,
                        int64_t ny, const Rect* rects, int nrects, const StencilCoef& c) {
  RMA_CHECK_ARG(K >= 1, "K=" << K);
  RMA_CHECK_ARG(T2 != T, "multi-step update cannot run in place");
  std::vector<double> a(T, T + nx * ny), b(a);
  const Rect interior{1, nx - 1, 1, ny - 1};
  for (int j = 1; j < K; ++j) {  // levels 1..K-1 on the interior, T elsewhere
    stencil_rects_cpu(b.data(), a.data(), iCp, nx, ny, &interior, 1, c);
    a.swap(b);
  }
  stencil_rects_cpu(T2, a.data(), iCp, nx, ny, rects, nrects, c);
}

bool fast5_ok(const StencilCoef& c) {
  const double ax = (-c.mlam) * c.rdx * c.rdx, ay = (-c.mlam) * c.rdy * c.rdy;
  return ax != 0.0 && std::isfinite(ax) && std::isfinite(ay) && std::isfinite(ay / ax) &&
         std::isfinite(c.dt * ax);
}

// fast5 arithmetic (csrc/lab/stencil_kstep_lab.hip kernel 5, stencil_pipe.h): the 5-point sum
// with the constants folded into one per-cell factor g = dt*lam/dx^2 * 1/Cp,
//   T2 = fma(g, fma(r, U+D, fma(-2(1+r), c, R+L)), c),  r = (lam/dy^2)/(lam/dx^2).
// std::fma rounds once like v_fma_f64, so this twin is bitwise equal to the
// GPU kernels (tests/test_fast5_cpu.py, tests/test_pipe_gpu.py).
void stencil5_rects_cpu(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                        const Rect* rects, int nrects, const StencilCoef& c) {
  RMA_CHECK_ARG(nrects >= 0 && nrects <= kMaxRects, "nrects=" << nrects);
  RMA_CHECK_ARG(fast5_ok(c), "fast5 needs lam != 0 and finite coefficients");
  const double ax = (-c.mlam) * c.rdx * c.rdx;
  const double ay = (-c.mlam) * c.rdy * c.rdy;
  const double ry = ay / ax;
  const double mkc = -2.0 * (1.0 + ry);
  const double gs = c.dt * ax;
  for (int i = 0; i < nrects; ++i) {
    const Rect r = rects[i];
    if (r.empty()) continue;
    RMA_CHECK_ARG(r.x0 >= 1 && r.x1 <= nx - 1 && r.y0 >= 1 && r.y1 <= ny - 1,
                  "rect outside interior");
    parallel_for(r.y0, r.y1, 64, [&](int64_t y) {
      const double* up = T + (y - 1) * nx;
      const double* cu = T + y * nx;
      const double* dn = T + (y + 1) * nx;
      const double* ic = iCp + y * nx;
      double* out = T2 + y * nx;
      for (int64_t x = r.x0; x < r.x1; ++x) {
        const double g = gs * ic[x];
        const double sx = cu[x + 1] + cu[x - 1];
        const double sy = up[x] + dn[x];
        double t = std::fma(mkc, cu[x], sx);
        t = std::fma(ry, sy, t);
        out[x] = std::fma(g, t, cu[x]);
      }
    });
  }
}

void stencilk5_rects_cpu(int K, double* T2, const double* T, const double* iCp, int64_t nx,
                         int64_t ny, const Rect* rects, int nrects, const StencilCoef& c) {
  RMA_CHECK_ARG(K >= 1, "K=" << K);
  RMA_CHECK_ARG(T2 != T, "multi-step update cannot run in place");
  std::vector<double> a(T, T + nx * ny), b(a);
  const Rect interior{1, nx - 1, 1, ny - 1};
  for (int j = 1; j < K; ++j) {
    stencil5_rects_cpu(b.data(), a.data(), iCp, nx, ny, &interior, 1, c);
    a.swap(b);
  }
  stencil5_rects_cpu(T2, a.data(), iCp, nx, ny, rects, nrects, c);
}

// The split fast-math form (kernels 14 / 15, stencil_pipe.h kArFast6Reg /
// kArFast7Reg): T2 = fma(g, fma(ry, fma(-2, c, U+D), fma(-2, c, L+R)), c).
void stencil6_rects_cpu(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                        const Rect* rects, int nrects, const StencilCoef& c) {
  RMA_CHECK_ARG(nrects >= 0 && nrects <= kMaxRects, "nrects=" << nrects);
  RMA_CHECK_ARG(fast5_ok(c), "fast-math needs lam != 0 and finite coefficients");
  const double ax = (-c.mlam) * c.rdx * c.rdx;
  const double ay = (-c.mlam) * c.rdy * c.rdy;
  const double ry = ay / ax;
  const double gs = c.dt * ax;
  for (int i = 0; i < nrects; ++i) {
    const Rect r = rects[i];
    if (r.empty()) continue;
    RMA_CHECK_ARG(r.x0 >= 1 && r.x1 <= nx - 1 && r.y0 >= 1 && r.y1 <= ny - 1,
                  "rect outside interior");
    parallel_for(r.y0, r.y1, 64, [&](int64_t y) {
      const double* up = T + (y - 1) * nx;
      const double* cu = T + y * nx;
      const double* dn = T + (y + 1) * nx;
      const double* ic = iCp + y * nx;
      double* out = T2 + y * nx;
      for (int64_t x = r.x0; x < r.x1; ++x) {
        const double g = gs * ic[x];
        const double sx = cu[x + 1] + cu[x - 1];
        const double sy = up[x] + dn[x];
        const double t = std::fma(ry, std::fma(-2.0, cu[x], sy), std::fma(-2.0, cu[x], sx));
        out[x] = std::fma(g, t, cu[x]);
      }
    });
  }
}

void stencilk6_rects_cpu(int K, double* T2, const double* T, const double* iCp, int64_t nx,
                         int64_t ny, const Rect* rects, int nrects, const StencilCoef& c) {
  RMA_CHECK_ARG(K >= 1, "K=" << K);
  RMA_CHECK_ARG(T2 != T, "multi-step update cannot run in place");
  std::vector<double> a(T, T + nx * ny), b(a);
  const Rect interior{1, nx - 1, 1, ny - 1};
  for (int j = 1; j < K; ++j) {
    stencil6_rects_cpu(b.data(), a.data(), iCp, nx, ny, &interior, 1, c);
    a.swap(b);
  }
  stencil6_rects_cpu(T2, a.data(), iCp, nx, ny, rects, nrects, c);
}

void flux_cpu(double* QX, double* QY, const double* T, int64_t nx, int64_t ny, double mlam,
              double rdx, double rdy) {
  parallel_for(0, ny - 1, 64, [&](int64_t y) {
    const double* r0 = T + y * nx;
    const double* r1 = r0 + nx;
    for (int64_t x = 1; x < nx - 1; ++x) QY[y * nx + x] = (mlam * (r1[x] - r0[x])) * rdy;
    if (y >= 1)
      for (int64_t x = 0; x < nx - 1; ++x) QX[y * nx + x] = (mlam * (r0[x + 1] - r0[x])) * rdx;
  });
}

void residual_cpu(double* D, const double* QX, const double* QY, const double* iCp, int64_t nx,
                  int64_t ny, double rdx, double rdy) {
  parallel_for(1, ny - 1, 64, [&](int64_t y) {
    for (int64_t x = 1; x < nx - 1; ++x) {
      const int64_t o = y * nx + x;
      const double ddx = (QX[o] - QX[o - 1]) * rdx;
      const double ddy = (QY[o] - QY[o - nx]) * rdy;
      D[o] = iCp[o] * (-(ddx + ddy));
    }
  });
}

void update_cpu(double* T, const double* D, int64_t nx, int64_t ny, double dt) {
  parallel_for(1, ny - 1, 64, [&](int64_t y) {
    for (int64_t x = 1; x < nx - 1; ++x) {
      double* p = T + y * nx + x;
      *p = *p + dt * D[y * nx + x];
    }
  });
}

void copy2d_cpu(void* dst, int64_t dst_ld, const void* src, int64_t src_ld, int64_t n_o,
                int64_t n_k, int elem_bytes) {
  RMA_CHECK_ARG(elem_bytes == 2 || elem_bytes == 4 || elem_bytes == 8 || elem_bytes == 16,
                "unsupported element size " << elem_bytes);
  char* d = static_cast<char*>(dst);
  const char* s = static_cast<const char*>(src);
  for (int64_t o = 0; o < n_o; ++o)
    std::memcpy(d + o * dst_ld * elem_bytes, s + o * src_ld * elem_bytes, n_k * elem_bytes);
}

void copy2d_batch_cpu(const Copy2d* copies, int n, int elem_bytes) {
  RMA_CHECK_ARG(n >= 0 && n <= kCopy2dBatch, "copy2d batch of " << n);
  for (int i = 0; i < n; ++i) {
    const Copy2d& c = copies[i];
    if (c.n_o <= 0 || c.n_k <= 0) continue;
    RMA_CHECK_ARG(c.dst_ld >= c.n_k && c.src_ld >= c.n_k, "leading dims smaller than row length");
    copy2d_cpu(c.dst, c.dst_ld, c.src, c.src_ld, c.n_o, c.n_k, elem_bytes);
  }
}

double reduce_cpu(const double* A, int64_t n, int op) {
  double v = (op == kMax) ? -std::numeric_limits<double>::infinity()
                          : (op == kMin ? std::numeric_limits<double>::infinity() : 0.0);
  for (int64_t i = 0; i < n; ++i) {
    const double a = A[i];
    switch (op) {
      case kSum: v += a; break;
      case kMax: v = std::fmax(v, a); break;
      case kMin: v = std::fmin(v, a); break;
      case kMaxAbs: v = std::fmax(v, std::fabs(a)); break;
      case kNonFinite: v += std::isfinite(a) ? 0.0 : 1.0; break;
      default: RMA_CHECK_ARG(false, "bad reduce op " << op);
    }
  }
  return v;
}

// CPU twin of field_stats_gpu (misc.hip)
void field_stats_cpu(const double* A, int64_t n, double* out3) {
  double bad = 0.0, lo = INFINITY, hi = -INFINITY;
  for (int64_t i = 0; i < n; ++i) {
    const double v = A[i];
    if (!std::isfinite(v)) {
      bad += 1.0;
      continue;
    }
    lo = std::fmin(lo, v);
    hi = std::fmax(hi, v);
  }
  out3[0] = bad;
  out3[1] = lo;
  out3[2] = hi;
}

}  // namespace rma
