// Overlapped-strip K-step kernels (K = 2, 3, 4, 6, 8): the device templates
// shared by the core's bitwise default (kernel 3, stencil_kstep.hip) and the
// experimental / oracle variants in csrc/lab (kernels 0-2, 4). Scheme notes:
// K explicit-Euler steps per pass (K = 2, 3, 4, 6, 8; 12, 16 fast-math):
// deep temporal blocking in registers, overlapped strips.
//
// Kernels (StencilTuning::kernel):
//   0-3  canonical arithmetic, face-flux reuse, bitwise equal to K one-step
//        launches (1/Cp window in registers or an LDS ring; lane moves by
//        ds_bpermute or DPP). 3 is the bitwise default.
//   4    "fast": reassociated fluxes, 7 fp64 ops per cell update.
//   5    "fast5": 5-point sum with one folded per-cell factor, 5 fp64 ops.
//   6/7  "fast5p2"/"fast5p4": kernel 5's arithmetic with the K levels of one
//        strip pipelined over 2 / 4 waves of a block; 4 cells per lane fit,
//        halving the strip overlap. fast_tune_k picks 7 at K=16, 6 at K=12.
// The notes below describe the common scheme (written for kernels 0-3).
//
// The one-step kernel moves the minimum 24 B/cell of a step at the HBM
// roofline; the only way to go faster per step is to touch HBM once per K
// steps. A wave marching down its strip keeps, for every time level
// j = 0..K-1, two rows in registers and computes level j+1 of row i-j one row
// behind level j (a skewed wavefront in y). HBM sees 24 B/cell per K steps,
// so from K ~ 3 on the kernel is VALU-bound and the instruction count is what
// matters (measured: profiles/SUMMARY_r1.md):
//   * overlapped strips: a wave loads 64V columns and every lane updates its
//     V cells at every level; level j is valid on strip positions [j, 64V-j)
//     (strip-edge garbage moves in one column per level), so a strip outputs
//     its inner columns and consecutive strips overlap by ~2K columns. (A
//     variant with dedicated edge lanes computing the outside columns cost
//     one extra evaluation per lane and level: 15.5 vs 19.5 TB/s at K=4.)
//   * face fluxes are computed once and shared by the two cells of a face —
//     x-faces with the left lane (one shuffle of the flux instead of the
//     value), y-faces with the next row (the lower face flux of row r is the
//     upper one of row r-1, kept in a register). Same expressions, same
//     rounding as rma/common.h, so the result is bitwise equal to K one-step
//     launches: 14 fp64 ops per cell update instead of 21.
//   * no per-level selects: 1/Cp is kept in a K-row register window, zeroed
//     outside the interior, so boundary/halo cells compute c + dt*(0*...) == c.
//   * two-row windows alternate slots with the iteration parity (loop
//     unrolled by two): no copies; the T and 1/Cp rows are prefetched two
//     iterations ahead (one ahead made every iteration wait for the previous
//     iteration's store as well: its vmcnt count is path-dependent).
// Step-j values outside the interior [1,nx-1)x[1,ny-1) stay T (fixed
// boundary / halo cells). Multi-rank use: halo width K, overlap 2K.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>

#include "rma/hip_check.h"
#include "rma/kernels.h"
#include "stencil_device.h"

namespace rma {
namespace kstep {
using namespace march;

// Cross-lane moves by one lane. kDpp: DPP wave shifts (VALU, a few cycles of
// latency); otherwise ds_bpermute (LDS pipe, ~100+ cycles round trip). The
// lane that has no source (63 for next, 0 for prev) gets garbage: those strip
// positions are invalid at every level anyway.
template <bool kDpp>
__device__ __forceinline__ double from_next_lane(double v) {
  if constexpr (kDpp) {
    // bound_ctrl: lanes without a source read 0 (no `old` register to set up)
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x130, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);  // wave_shl:1 -> lane i gets lane i+1
  } else {
    return __shfl_down(v, 1);
  }
}
template <bool kDpp>
__device__ __forceinline__ double from_prev_lane(double v) {
  if constexpr (kDpp) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x138, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);  // wave_shr:1 -> lane i gets lane i-1
  } else {
    return __shfl_up(v, 1);
  }
}

__device__ __forceinline__ double face(double lv, double rv, double mlam, double rd) {
  return (mlam * (rv - lv)) * rd;  // flux lv -> rv: qxR of the left cell == qxL of the right one
}


// kLds: keep the masked 1/Cp window in an LDS ring (per wave, slot = row mod
// K) instead of K*V registers, for occupancy (kernel=1 of StencilTuning).
// kFast: the same scheme with reassociated arithmetic (NOT bitwise equal to
// the canonical expression): differences instead of fluxes, the constants
// folded (ax = lam/dx^2, ay = lam/dy^2, g = dt/Cp) and FMAs:
//   T2 = fma(g, fma(ay, dU - dD, ax * (dR - dL)), c)   — 7 fp64 ops per cell.
template <int K, int V, bool NT, bool kLds, bool kDpp, bool kFast = false>
__device__ __forceinline__ void stencilk_body(
    double* __restrict__ T2, const double* __restrict__ T, const double* __restrict__ iCp,
    int64_t nx, int64_t ny, const RectList& L, const StencilCoef& k, int chunk_rows, int remap) {
  constexpr int W = kWave * V;
  constexpr int kStep = (W - 2 * K) / V * V;  // output columns per strip (plan_rects)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = remap ? xcd_remap(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  int ri = 0;
  while (ri < L.n - 1 && b >= L.block_end[ri]) ++ri;
  int64_t strip, chunk;
  if (!locate_task(L, ri, b, wave, strip, chunk)) return;  // whole wave exits
  const Rect r = L.r[ri];
  const int64_t xs = L.xa[ri] + strip * kStep;  // first loaded column
  const int64_t ya = r.y0 + chunk * chunk_rows;
  const int64_t yb = min(r.y1, ya + (int64_t)chunk_rows);

  const int64_t x = xs + (int64_t)lane * V;
  bool m[V], cin[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int p = lane * V + v;
    m[v] = p >= K && p < K + kStep && x + v >= r.x0 && x + v < r.x1;
    cin[v] = (x + v >= 1) && (x + v <= nx - 2);
  }
  const int64_t xl = min(max(x, (int64_t)0), nx - V);

  // w[j][s]: level j rows (slot parity alternates per iteration: new row ->
  // slot P, previous -> 1-P); fy[j]: upper face flux of the previous
  // level-(j+1) row (== lower face flux of the current one); gic[j]: 1/Cp of
  // the row level j+1 updates, ZEROED outside the interior (boundary rows and
  // columns): the canonical update then returns c + dt*(0*(...)) == c for
  // them, bitwise, without a select per level (all values are finite).
  double w[K][2][V], fy[K][V], gic[K][V], pT[V], pC[V], qT[V], qC[V];  // q: 2 rows ahead
#pragma unroll
  for (int j = 0; j < K; ++j) {
#pragma unroll
    for (int v = 0; v < V; ++v) w[j][0][v] = w[j][1][v] = fy[j][v] = gic[j][v] = 0.0;
  }
  int64_t i = ya - K;
  const int64_t iend = yb + K - 2;
  auto rowc = [&](int64_t y) { return min(max(y, (int64_t)0), ny - 1); };
  load_row<V>(w[0][1], T + rowc(i) * nx + xl);
  load_row<V>(pT, T + rowc(i + 1) * nx + xl);
  load_row<V>(pC, iCp + rowc(i) * nx + xl);
  load_row<V>(qT, T + rowc(i + 2) * nx + xl);
  load_row<V>(qC, iCp + rowc(i + 1) * nx + xl);

  const double ax = (-k.mlam) * k.rdx * k.rdx;  // kFast only
  const double ay = (-k.mlam) * k.rdy * k.rdy;
  // LDS ring of masked 1/Cp rows: [wave][slot][lane*V + v] (16-B per lane)
  __shared__ double ring[kLds ? kWavesPerBlock * K * W : 1];
  double* myring = ring + (kLds ? wave * K * W + lane * V : 0);
  int slot = 0;  // ring slot of the current level-1 row (iteration count mod K)
  if constexpr (kLds) {  // slots read before their first write feed only discarded rows
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
      for (int v = 0; v < V; ++v) myring[j * W + v] = 0.0;
  }

  auto iter = [&](auto Pc) {
    constexpr int P = decltype(Pc)::value;
    // level 0 <- prefetched T row i+1; 1/Cp window <- prefetched row i (masked)
    const bool rin1 = i >= 1 && i <= ny - 2;  // row of level 1 (wave-uniform)
#pragma unroll
    for (int v = 0; v < V; ++v) w[0][P][v] = pT[v];
    if constexpr (kLds) {
      double g[V];
#pragma unroll
      for (int v = 0; v < V; ++v) g[v] = (rin1 && cin[v]) ? (kFast ? k.dt * pC[v] : pC[v]) : 0.0;
      double* dst = myring + slot * W;
      if constexpr (V == 1) {
        dst[0] = g[0];
      } else {
#pragma unroll
        for (int h = 0; h < V / 2; ++h) {
          dbl2 t2;
          t2.x = g[2 * h];
          t2.y = g[2 * h + 1];
          reinterpret_cast<dbl2*>(dst)[h] = t2;
        }
      }

    } else {
#pragma unroll
      for (int j = K - 1; j > 0; --j) {
#pragma unroll
        for (int v = 0; v < V; ++v) gic[j][v] = gic[j - 1][v];
      }
#pragma unroll
      for (int v = 0; v < V; ++v)
        gic[0][v] = (rin1 && cin[v]) ? (kFast ? k.dt * pC[v] : pC[v]) : 0.0;
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {  // see stencilk5_body: two rows of prefetch
      pT[v] = qT[v];
      pC[v] = qC[v];
    }
    load_row<V>(qT, T + rowc(i + 3) * nx + xl);
    load_row<V>(qC, iCp + rowc(i + 2) * nx + xl);
#pragma unroll
    for (int j = 1; j <= K; ++j) {
      const int64_t row = i - (j - 1);
      double icl[V];  // masked 1/Cp of `row` (written j-1 iterations ago)
      if constexpr (kLds) {
        const int sl = slot - (j - 1) < 0 ? slot - (j - 1) + K : slot - (j - 1);
        const double* src = myring + sl * W;
        if constexpr (V == 1) {
          icl[0] = src[0];
        } else {
#pragma unroll
          for (int h = 0; h < V / 2; ++h) {
            const dbl2 t2 = reinterpret_cast<const dbl2*>(src)[h];
            icl[2 * h] = t2.x;
            icl[2 * h + 1] = t2.y;
          }
        }
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) icl[v] = gic[j - 1][v];
      }
      const double(&c)[V] = w[j - 1][1 - P];
      const double(&dn)[V] = w[j - 1][P];
      const double rn = from_next_lane<kDpp>(c[0]);  // lane 63: garbage (invalid column)
      double qr[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const double rv = v + 1 < V ? c[v + 1] : rn;
        qr[v] = kFast ? rv - c[v] : face(c[v], rv, k.mlam, k.rdx);
      }
      const double ql0 = from_prev_lane<kDpp>(qr[V - 1]);  // lane 0: garbage
      double res[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const double qU = kFast ? dn[v] - c[v] : face(c[v], dn[v], k.mlam, k.rdy);
        const double qD = fy[j - 1][v];
        fy[j - 1][v] = qU;
        const double qL = v == 0 ? ql0 : qr[v - 1];
        if constexpr (kFast)
          res[v] = __builtin_fma(icl[v], __builtin_fma(ay, qU - qD, ax * (qr[v] - qL)), c[v]);
        else
          res[v] = c[v] + k.dt * (icl[v] * ((-(qr[v] - qL)) * k.rdx - (qU - qD) * k.rdy));
      }
      if (j < K) {
        const int jj = j < K ? j : K - 1;
#pragma unroll
        for (int v = 0; v < V; ++v) w[jj][P][v] = res[v];
      } else if (row >= ya && row < yb) {
        store_row<V, NT>(T2 + row * nx + x, res, m);
      }
    }
    if constexpr (kLds) slot = slot + 1 == K ? 0 : slot + 1;
  };
  for (;;) {
    iter(std::integral_constant<int, 0>{});
    if (++i > iend) break;
    iter(std::integral_constant<int, 1>{});
    if (++i > iend) break;
  }
}

template <int K, int V, bool NT, bool kLds, bool kDpp, bool kFast = false>
__global__ __launch_bounds__(kBlock) void stencilk_ovl_kernel(
    double* __restrict__ T2, const double* __restrict__ T, const double* __restrict__ iCp,
    int64_t nx, int64_t ny, RectList L, StencilCoef k, int chunk_rows, int remap) {
  stencilk_body<K, V, NT, kLds, kDpp, kFast>(T2, T, iCp, nx, ny, L, k, chunk_rows, remap);
}


// Host-side argument checks of the overlapped-strip K-step launchers (core
// and lab): cells per lane V and the task order.
struct KstepLaunch {
  int V, remap;
};
inline KstepLaunch check_launch(int K, const double* T2, const double* T, const double* iCp,
                                int64_t nx, int64_t ny, const Rect* rects, int nrects,
                                const StencilCoef& c, const StencilTuning& tune) {
  RMA_CHECK_ARG(K == 2 || K == 3 || K == 4 || K == 6 || K == 8 || K == 12 || K == 16,
                "steps per pass must be 2, 3, 4, 6, 8, 12 or 16 (any K: kernels 9/10), got " << K);
  RMA_CHECK_ARG(K <= 8 || tune.kernel >= 5,
                "12 or 16 steps per pass need a fast5 kernel (kernel 5, 6, 7 or 8), got kernel "
                    << tune.kernel);
  RMA_CHECK_ARG(nrects >= 0 && nrects <= kMaxRects, "nrects=" << nrects);
  RMA_CHECK_ARG(nx >= 3 && ny >= 3, "grid too small: nx=" << nx << " ny=" << ny);
  RMA_CHECK_ARG(T2 != T, "multi-step kernel cannot run in place");
  for (int i = 0; i < nrects; ++i) {
    const Rect& r = rects[i];
    if (r.empty()) continue;
    RMA_CHECK_ARG(r.x0 >= 1 && r.x1 <= nx - 1 && r.y0 >= 1 && r.y1 <= ny - 1,
                  "rect " << i << " outside the interior of " << nx << "x" << ny);
  }
  RMA_CHECK_ARG(tune.chunk_rows >= 1, "chunk_rows=" << tune.chunk_rows);
  RMA_CHECK_ARG(tune.kernel < 5 || fast5_ok(c),
                "kernel 5 folds dy^-2/dx^-2 into one factor: needs lam != 0 and finite "
                "coefficients");
  const bool aligned = ((reinterpret_cast<uintptr_t>(T) & 15) == 0) &&
                       ((reinterpret_cast<uintptr_t>(T2) & 15) == 0) &&
                       ((reinterpret_cast<uintptr_t>(iCp) & 15) == 0);
  int V = 1;
  if (aligned && nx % 2 == 0)
    V = (tune.vec == 4 && nx % 4 == 0 && (K <= 8 || tune.kernel >= 6)) ? 4 : 2;
  return {V, tune.xcd_remap >= 0 ? tune.xcd_remap : (nx > 65536 ? 1 : 0)};
}

}  // namespace kstep
}  // namespace rma
