// librma_lab.so, one-step unit: the LDS-tiled one-step kernel (kernel 1), the
// measured alternative to the core's register march (csrc/kernels/stencil.hip):
// 16384^2 one-step 3.90 vs 6.20 TB/s (profiles/SUMMARY_r1.md). Kept as a test
// oracle and for sweeps (bench/stencil_sweep.py); the core dispatches
// tune.kernel == 1 here through lab_hooks().onestep (lab_hooks.h).
//
#include <hip/hip_runtime.h>

#include "../kernels/lab_hooks.h"
#include "../kernels/stencil_device.h"
#include "rma/hip_check.h"

namespace rma {
namespace {
using namespace march;

// LDS-tiled variant (kernel=1), kept as the measured alternative to the march:
// a 256-thread block stages a (TY+2) x (TX+2) tile of T in LDS (one row per
// wave-instruction, 16-B loads), then every thread updates TY/4 cells of its
// column from LDS. T is re-read (TY+2)/TY times through L2/MALL instead of
// once; see profiles/ for the A/B against the march.
// ---------------------------------------------------------------------------
constexpr int kTileX = 256;  // cells per tile row (one double per thread)
constexpr int kTileY = 16;

template <bool NT>
__global__ __launch_bounds__(kBlock) void stencil_lds_kernel(double* __restrict__ T2,
                                                             const double* __restrict__ T,
                                                             const double* __restrict__ iCp,
                                                             int64_t nx, RectList L,
                                                             StencilCoef k) {
  __shared__ double tile[kTileY + 2][kTileX + 2];
  const int64_t b = xcd_remap(blockIdx.x, gridDim.x);
  int ri = 0;
  while (ri < L.n - 1 && b >= L.block_end[ri]) ++ri;
  const int64_t bstart = ri ? L.block_end[ri - 1] : 0;
  const int64_t ntx = L.strips[ri];
  const int64_t t = b - bstart;
  const Rect r = L.r[ri];
  const int64_t tx = t % ntx, ty = t / ntx;
  const int64_t x0 = r.x0 + tx * kTileX;
  const int64_t y0 = r.y0 + ty * kTileY;
  const int tid = threadIdx.x;
  // Stage rows y0-1 .. y0+TY (clamped to the rect's +-1 neighbourhood).
  for (int j = tid >> 6; j < kTileY + 2; j += kWavesPerBlock) {
    const int64_t gy = min(y0 - 1 + j, r.y1);
    const double* src = T + gy * nx;
    for (int i = tid & 63; i < kTileX + 2; i += kWave) {
      const int64_t gx = min(x0 - 1 + i, r.x1);
      tile[j][i] = src[gx];
    }
  }
  __syncthreads();
  const int64_t gx = x0 + tid;
  if (gx >= r.x1) return;
  for (int j = 1; j <= kTileY; ++j) {
    const int64_t gy = y0 - 1 + j;
    if (gy >= r.y1) break;
    const double c = tile[j][tid + 1];
    const double v = cell(tile[j][tid], c, tile[j][tid + 2], tile[j - 1][tid + 1],
                          tile[j + 1][tid + 1], iCp[gy * nx + gx], k);
    if constexpr (NT) {
      __builtin_nontemporal_store(v, T2 + gy * nx + gx);
    } else {
      T2[gy * nx + gx] = v;
    }
  }
}

}  // namespace

namespace lab {
bool onestep(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
             const Rect* rects, int nrects, const StencilCoef& c, const StencilTuning& tune,
             stream_t stream) {
  (void)ny;  // rects were validated by the core launcher
  if (tune.kernel != 1) return false;
  RectList L{};
  int64_t total = 0;
  for (int i = 0; i < nrects; ++i) {
    const Rect& r = rects[i];
    if (r.empty()) continue;
    const int n = L.n++;
    L.r[n] = r;
    L.xa[n] = r.x0;
    L.strips[n] = (r.x1 - r.x0 + kTileX - 1) / kTileX;
    L.chunks[n] = (r.y1 - r.y0 + kTileY - 1) / kTileY;
    total += L.strips[n] * L.chunks[n];
    L.block_end[n] = total;
  }
  if (L.n == 0) return true;
  RMA_CHECK_ARG(total < (int64_t(1) << 31), "grid too large: " << total << " blocks");
  const dim3 grid((unsigned)total), block(kBlock);
  hipStream_t s = as_stream(stream);
  if (tune.nontemporal)
    stencil_lds_kernel<true><<<grid, block, 0, s>>>(T2, T, iCp, nx, L, c);
  else
    stencil_lds_kernel<false><<<grid, block, 0, s>>>(T2, T, iCp, nx, L, c);
  RMA_HIP_LAUNCH_CHECK();
  return true;
}
}  // namespace lab
}  // namespace rma
