// Two explicit-Euler steps per pass: temporal blocking in registers.
//
// The one-step kernel (stencil.hip) already moves exactly the minimum bytes
// of a step (read T, read 1/Cp, write T2: 24 B/cell) at the HBM roofline, so
// the only way to go faster per time step is to touch HBM less often. Here a
// wave marching down its 64*V-cell strip computes step t+1 for row i (from T
// rows i-1..i+1 in registers) and immediately step t+2 for row i-1 (from the
// step-(t+1) rows i-2..i, also in registers): 24 B/cell per TWO steps.
//
// The arithmetic is the canonical cell update of rma/common.h applied twice
// in the same order, so the result is bitwise identical to two one-step
// launches (tests/test_temporal_gpu.py). Step-1 values outside the interior
// [1,nx-1)x[1,ny-1) are T itself (fixed boundary / halo cells).
//
// Strip edges: step 2 at the first/last cell of a strip needs the step-1
// value one column outside the strip, so each wave also evaluates step 1 at
// its two edge columns: lanes 0-31 compute column xs-1 and lanes 32-63 column
// xs+64V in one extra wave instruction per row (redundant with the
// neighbouring strip, ~25% extra VALU work that the HBM-bound kernel hides).
//
// Rows: output rows [ya,yb) need step-1 rows ya-1..yb and T rows ya-2..yb+1,
// i.e. chunk_rows+4 T rows per chunk; the re-read rows of adjacent chunks hit
// L2 with the same XCD-aware block order as the one-step kernel.
//
// Multi-rank use (executor, temporal=2): halo width 2 / overlap 4, one
// exchange per two steps; cells adjacent to a neighbour's halo are not output.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rma/hip_check.h"
#include "rma/kernels.h"
#include "stencil_device.h"

namespace rma {
namespace {
using namespace march;

template <int V, bool NT, bool NTL, int U>
__global__ __launch_bounds__(kBlock) void stencil2_march_kernel(
    double* __restrict__ T2, const double* __restrict__ T, const double* __restrict__ iCp,
    int64_t nx, int64_t ny, RectList L, StencilCoef k, int chunk_rows, int remap) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = remap ? xcd_remap(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  int ri = 0;
  while (ri < L.n - 1 && b >= L.block_end[ri]) ++ri;
  int64_t strip, chunk;
  if (!locate_task(L, ri, b, wave, strip, chunk)) return;  // whole wave exits
  const Rect r = L.r[ri];
  const int64_t xs = L.xa[ri] + strip * (kWave * V);
  const int64_t ya = r.y0 + chunk * chunk_rows;
  const int64_t yb = min(r.y1, ya + (int64_t)chunk_rows);

  const int64_t x = xs + (int64_t)lane * V;
  bool m[V];
  bool cin[V];  // own cell inside the step-1 domain (columns)
#pragma unroll
  for (int v = 0; v < V; ++v) {
    m[v] = (x + v >= r.x0) && (x + v < r.x1);
    cin[v] = (x + v >= 1) && (x + v <= nx - 2);
  }
  const int64_t xl = min(x, nx - V);  // clamped load column
  const bool left = lane < 32;
  const int64_t ce = left ? xs - 1 : xs + kWave * V;  // step-1 edge column of this lane
  const int64_t cf = left ? xs - 2 : xs + kWave * V + 1;
  const bool ce_in = ce >= 1 && ce <= nx - 2;
  const int64_t eidx = min(max(ce, (int64_t)0), nx - 1);
  const int64_t fidx = min(max(cf, (int64_t)0), nx - 1);
  const int src = left ? 0 : kWave - 1;

  // windows (k = slot): t[k], te[k]: T row i-1+k; s[k], se[k]: step-1 row i-2+k;
  // ic[k]: 1/Cp row i-1+k
  double t[U + 2][V], te[U + 2];
  double s[U + 2][V], se[U + 2];
  double ic[U + 1][V];
  int64_t i = ya - 1;
  {
    const int64_t y0 = max(i - 1, (int64_t)0), y1 = i;  // i >= 0 since ya >= 1
    load_row<V>(t[0], T + y0 * nx + xl);
    load_row<V>(t[1], T + y1 * nx + xl);
    te[0] = T[y0 * nx + eidx];
    te[1] = T[y1 * nx + eidx];
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {  // feed only step-2 rows < ya (never stored)
    ic[0][v] = 0.0;
    s[0][v] = 0.0;
    s[1][v] = 0.0;
  }
  se[0] = se[1] = 0.0;

  for (; i - 1 < yb; i += U) {  // step-1 rows i..i+U-1, step-2 rows i-1..i+U-2
    double tf[U], ice[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t yn = min(i + u + 1, ny - 1);
      const int64_t yc = min(i + u, ny - 1);
      load_row<V>(t[u + 2], T + yn * nx + xl);
      te[u + 2] = T[yn * nx + eidx];
      load_row<V, NTL>(ic[u + 1], iCp + yc * nx + xl);
      tf[u] = T[yc * nx + fidx];
      ice[u] = iCp[yc * nx + eidx];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t y1 = i + u;
      const bool rin = y1 >= 1 && y1 <= ny - 2;  // wave-uniform
      double res[V];
      row_update<V>(res, t[u], t[u + 1], t[u + 2], ic[u + 1], te[u + 1], lane, k);
#pragma unroll
      for (int v = 0; v < V; ++v) s[u + 2][v] = (rin && cin[v]) ? res[v] : t[u + 1][v];
      // step 1 at this lane's edge column
      const double nb = __shfl(left ? t[u + 1][0] : t[u + 1][V - 1], src);
      const double ev = cell(left ? tf[u] : nb, te[u + 1], left ? nb : tf[u], te[u], te[u + 2],
                             ice[u], k);
      se[u + 2] = (rin && ce_in) ? ev : te[u + 1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t y2 = i - 1 + u;
      if (y2 >= ya && y2 < yb) {  // wave-uniform
        double res[V];
        row_update<V>(res, s[u], s[u + 1], s[u + 2], ic[u], se[u + 1], lane, k);
        store_row<V, NT>(T2 + y2 * nx + x, res, m);
      }
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
      t[0][v] = t[U][v];
      t[1][v] = t[U + 1][v];
      s[0][v] = s[U][v];
      s[1][v] = s[U + 1][v];
      ic[0][v] = ic[U][v];
    }
    te[0] = te[U];
    te[1] = te[U + 1];
    se[1] = se[U + 1];
  }
}

}  // namespace

void stencil2_rects_gpu(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                        const Rect* rects, int nrects, const StencilCoef& c,
                        const StencilTuning& tune, stream_t stream) {
  RMA_CHECK_ARG(nrects >= 0 && nrects <= kMaxRects, "nrects=" << nrects);
  RMA_CHECK_ARG(nx >= 3 && ny >= 3, "grid too small: nx=" << nx << " ny=" << ny);
  RMA_CHECK_ARG(T2 != T, "two-step kernel cannot run in place");
  for (int i = 0; i < nrects; ++i) {
    const Rect& r = rects[i];
    if (r.empty()) continue;
    RMA_CHECK_ARG(r.x0 >= 1 && r.x1 <= nx - 1 && r.y0 >= 1 && r.y1 <= ny - 1,
                  "rect " << i << " outside the interior of " << nx << "x" << ny);
  }
  RMA_CHECK_ARG(tune.chunk_rows >= 1, "chunk_rows=" << tune.chunk_rows);
  const bool aligned = ((reinterpret_cast<uintptr_t>(T) & 15) == 0) &&
                       ((reinterpret_cast<uintptr_t>(T2) & 15) == 0) &&
                       ((reinterpret_cast<uintptr_t>(iCp) & 15) == 0);
  const int V = (aligned && nx % 2 == 0) ? 2 : 1;
  const int remap = tune.xcd_remap >= 0 ? tune.xcd_remap : (nx > 65536 ? 1 : 0);
  RectList L;
  const int64_t total = plan_rects(L, rects, nrects, V, tune.chunk_rows, remap, false);
  if (L.n == 0) return;
  RMA_CHECK_ARG(total < (int64_t(1) << 31), "grid too large: " << total << " blocks");
  const dim3 grid((unsigned)total), block(kBlock);
  hipStream_t s = as_stream(stream);
  const bool nts = tune.nontemporal & 1, ntl = (tune.nontemporal >> 1) & 1;
  const int u = tune.unroll;
  RMA_CHECK_ARG(u == 2 || u == 4, "two-step kernel: unroll must be 2 or 4");
#define RMA_TB(VV, NTS, NTL, UU)                                                         \
  stencil2_march_kernel<VV, NTS, NTL, UU><<<grid, block, 0, s>>>(T2, T, iCp, nx, ny, L, c, \
                                                                  tune.chunk_rows, remap)
#define RMA_TB_U(VV, NTS, NTL) \
  if (u == 4) RMA_TB(VV, NTS, NTL, 4); else RMA_TB(VV, NTS, NTL, 2);
  if (V == 2) {
    if (nts && ntl) { RMA_TB_U(2, true, true) }
    else if (nts) { RMA_TB_U(2, true, false) }
    else if (ntl) { RMA_TB_U(2, false, true) }
    else { RMA_TB_U(2, false, false) }
  } else {
    if (nts) { RMA_TB_U(1, true, false) }
    else { RMA_TB_U(1, false, false) }
  }
#undef RMA_TB_U
#undef RMA_TB
  RMA_HIP_LAUNCH_CHECK();
}

}  // namespace rma
