// Fused 5-point diffusion stencil for CDNA4 (gfx950).
//
// Reference behaviour: scripts/diffusion_2D_perf.jl:3-13 (fused update, one
// work-item per cell, (32,8) groups) and scripts/diffusion_2D_perf_hide.jl:15-29
// (boundary/interior split with masks). Here both are one kernel that updates
// an explicit list of rectangles, so the split variant has exact frame and
// interior grids (no masked-off work-items, and no coverage holes — the
// reference's active perf_hide launch leaves ~10% of cells un-updated,
// SURVEY.md §2.3).
//
// Design ("register march", MI355X-first):
//   * The problem is HBM-bound: 24 B/cell (read T, read 1/Cp, write T2) vs
//     ~15 fp64 flops. Every byte of T must be read from HBM exactly once.
//   * One 64-lane wave owns an x-strip of 64*V cells (V=2: one 16-byte
//     dwordx4 load per lane per row, 1 KiB per wave-instruction) and marches
//     down `chunk_rows` rows, keeping rows y-1, y, y+1 in registers. Each T row
//     is therefore loaded once per strip; the y±1 neighbours never re-touch
//     memory.
//   * x±1 neighbours come from the adjacent lane via a cross-lane shuffle
//     (ds_bpermute); only the two strip-edge cells need a load, issued as ONE
//     wave instruction (lanes 0-31 fetch the left edge, 32-63 the right).
//   * U rows are unrolled and their loads issued before any arithmetic, so a
//     wave keeps ~U*40 B/lane in flight; with <=64 VGPRs 8 waves/SIMD fit, i.e.
//     hundreds of KB in flight per CU — enough to cover HBM latency.
//   * A block is 4 waves = 4 adjacent strips of the same row chunk (they share
//     the edge cache lines through L1); narrow rects (perf_hide x-frames) give
//     the 4 waves 4 consecutive row chunks instead, so no wave idles.
//   * 64-bit row offsets: tiles beyond 2^31 cells (288 GB HBM).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rma/hip_check.h"
#include "rma/kernels.h"
#include "lab_hooks.h"
#include "stencil_device.h"

namespace rma {
namespace {
using namespace march;

template <int V, bool NT, int kUnroll, bool NTL, bool NTT>
__device__ __forceinline__ void march_body(double* __restrict__ T2, const double* __restrict__ T,
                                           const double* __restrict__ iCp, int64_t nx,
                                           const RectList& L, const StencilCoef& k,
                                           int chunk_rows, int64_t b) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int lane = threadIdx.x & (kWave - 1);
  int ri = 0;
  while (ri < L.n - 1 && b >= L.block_end[ri]) ++ri;  // wave-uniform, <= 8 steps
  const int64_t bstart = ri ? L.block_end[ri - 1] : 0;
  if (L.gpad[ri] < 0) {
    // column mode for thin rects (perf_hide x-frames, a few cells wide): one
    // thread per row, scalar loads; a 128-cell wave strip would load 64x the
    // bytes it updates. The whole block takes this branch (uniform).
    const Rect r = L.r[ri];
    const int64_t y = r.y0 + (b - bstart) * kBlock + threadIdx.x;
    if (y >= r.y1) return;
    const double* up = T + (y - 1) * nx;
    const double* cu = T + y * nx;
    const double* dn = T + (y + 1) * nx;
    for (int64_t xx = r.x0; xx < r.x1; ++xx) {
      const double v = cell(cu[xx - 1], cu[xx], cu[xx + 1], up[xx], dn[xx], iCp[y * nx + xx], k);
      if constexpr (NT) {
        __builtin_nontemporal_store(v, T2 + y * nx + xx);
      } else {
        T2[y * nx + xx] = v;
      }
    }
    return;
  }
  int64_t strip, chunk;
  if (!locate_task(L, ri, b, wave, strip, chunk)) return;  // padding: whole wave exits
  const Rect r = L.r[ri];
  const int64_t xs = L.xa[ri] + strip * (kWave * V);
  const int64_t ya = r.y0 + chunk * chunk_rows;
  const int64_t yb = min(r.y1, ya + (int64_t)chunk_rows);

  const int64_t x = xs + (int64_t)lane * V;
  bool m[V];
#pragma unroll
  for (int v = 0; v < V; ++v) m[v] = (x + v >= r.x0) && (x + v < r.x1);
  const int64_t xl = min(x, nx - V);  // clamped load column (lanes past the array edge)
  const int64_t eidx = (lane < 32) ? max(xs - 1, (int64_t)0) : min(xs + kWave * V, nx - 1);

  double rows[kUnroll + 2][V];
  load_row<V>(rows[0], T + (ya - 1) * nx + xl);
  load_row<V>(rows[1], T + ya * nx + xl);

  int64_t y = ya;
  for (; y + kUnroll <= yb; y += kUnroll) {
    double ic[kUnroll][V];
    double ed[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      load_row<V, NTT>(rows[u + 2], T + (y + u + 1) * nx + xl);
      load_row<V, NTL>(ic[u], iCp + (y + u) * nx + xl);
      ed[u] = T[(y + u) * nx + eidx];
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      double res[V];
      row_update<V>(res, rows[u], rows[u + 1], rows[u + 2], ic[u], ed[u], lane, k);
      store_row<V, NT>(T2 + (y + u) * nx + x, res, m);
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
      rows[0][v] = rows[kUnroll][v];
      rows[1][v] = rows[kUnroll + 1][v];
    }
  }
  for (; y < yb; ++y) {
    double ic[V];
    load_row<V>(rows[2], T + (y + 1) * nx + xl);
    load_row<V, NTL>(ic, iCp + y * nx + xl);
    const double ed = T[y * nx + eidx];
    double res[V];
    row_update<V>(res, rows[0], rows[1], rows[2], ic, ed, lane, k);
    store_row<V, NT>(T2 + y * nx + x, res, m);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      rows[0][v] = rows[1][v];
      rows[1][v] = rows[2][v];
    }
  }
}

template <int V, bool NT, int kUnroll, bool NTL, bool NTT = false>
__global__ __launch_bounds__(kBlock) void stencil_march_kernel(double* __restrict__ T2,
                                                               const double* __restrict__ T,
                                                               const double* __restrict__ iCp,
                                                               int64_t nx, RectList L,
                                                               StencilCoef k, int chunk_rows,
                                                               int remap) {
  const int64_t b = remap ? xcd_remap(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  march_body<V, NT, kUnroll, NTL, NTT>(T2, T, iCp, nx, L, k, chunk_rows, b);
}

void validate_rects(int64_t nx, int64_t ny, const Rect* rects, int nrects) {
  RMA_CHECK_ARG(nrects >= 0 && nrects <= kMaxRects, "nrects=" << nrects);
  RMA_CHECK_ARG(nx >= 3 && ny >= 3, "grid too small: nx=" << nx << " ny=" << ny);
  for (int i = 0; i < nrects; ++i) {
    const Rect& r = rects[i];
    if (r.empty()) continue;
    RMA_CHECK_ARG(r.x0 >= 1 && r.x1 <= nx - 1 && r.y0 >= 1 && r.y1 <= ny - 1,
                  "rect " << i << " [" << r.x0 << "," << r.x1 << ")x[" << r.y0 << "," << r.y1
                          << ") outside the interior of " << nx << "x" << ny);
  }
}

}  // namespace

// stencil_vec, stencil_strip_cells: kernel_select.cpp

void stencil_rects_gpu(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                       const Rect* rects, int nrects, const StencilCoef& c,
                       const StencilTuning& tune, stream_t stream) {
  validate_rects(nx, ny, rects, nrects);
  RMA_CHECK_ARG(tune.chunk_rows >= 1, "chunk_rows=" << tune.chunk_rows);
  const bool aligned = ((reinterpret_cast<uintptr_t>(T) & 15) == 0) &&
                       ((reinterpret_cast<uintptr_t>(T2) & 15) == 0) &&
                       ((reinterpret_cast<uintptr_t>(iCp) & 15) == 0);
  const int V = aligned ? stencil_vec(nx, tune) : 1;
  // Block order (measured, profiles/SUMMARY_r1.md): chip-wide row bands with
  // 8-padded block rows win up to 64K-wide tiles (16384^2: 6.44 vs 6.26 TB/s);
  // per-XCD contiguous ranges win on the 288 GB tiles (101376^2: 6.25 vs 5.93).
  const int remap = tune.xcd_remap >= 0 ? tune.xcd_remap : (nx > 65536 ? 1 : 0);
  // the LDS-tiled one-step kernel (kernel 1, the measured loser against the
  // march, 3.90 vs 6.20 TB/s at 16384^2: profiles/SUMMARY_r1.md) lives in the lab library
  if (tune.kernel == 1) {
    if (!lab_hooks().onestep) lab_missing("the LDS-tiled one-step kernel (kernel 1)");
    RMA_CHECK_ARG(lab_hooks().onestep(T2, T, iCp, nx, ny, rects, nrects, c, tune, stream),
                  "one-step kernel " << tune.kernel);
    return;
  }
  RMA_CHECK_ARG(!tune.signal, "a signalling launch needs a pipelined K-step kernel");
  RMA_CHECK_ARG(!tune.direct || !tune.direct->on,
                "direct-store halos need a pipelined K-step kernel");
  RectList L{};
  const int64_t total = plan_rects(L, rects, nrects, V, tune.chunk_rows, remap, true);
  if (L.n == 0) return;
  RMA_CHECK_ARG(total < (int64_t(1) << 31), "grid too large: " << total << " blocks");
  const dim3 grid((unsigned)total), block(kBlock);
  hipStream_t s = as_stream(stream);
  {
    const int u = tune.unroll;
    RMA_CHECK_ARG(u == 2 || u == 4 || u == 8, "unroll must be 2, 4 or 8");
    const bool nts = tune.nontemporal & 1, ntl = (tune.nontemporal >> 1) & 1;
    const bool ntt = (tune.nontemporal >> 2) & 1;  // bit 2: also T loads (implies 1|2)
#define RMA_MARCH(VV, UU, NTS, NTL)                                                  \
  stencil_march_kernel<VV, NTS, UU, NTL><<<grid, block, 0, s>>>(T2, T, iCp, nx, L, c, \
                                                                 tune.chunk_rows, remap)
#define RMA_MARCH_NT(VV, UU)                                                            \
  if (ntt) {                                                                            \
    stencil_march_kernel<VV, true, UU, true, true><<<grid, block, 0, s>>>(                \
        T2, T, iCp, nx, L, c, tune.chunk_rows, remap);                           \
  } else if (nts) {                                                                     \
    if (ntl) RMA_MARCH(VV, UU, true, true);                                              \
    else RMA_MARCH(VV, UU, true, false);                                                 \
  } else {                                                                              \
    if (ntl) RMA_MARCH(VV, UU, false, true);                                             \
    else RMA_MARCH(VV, UU, false, false);                                                \
  }
#define RMA_MARCH_U(VV)                     \
  switch (u) {                              \
    case 2: RMA_MARCH_NT(VV, 2) break;      \
    case 8: RMA_MARCH_NT(VV, 8) break;      \
    default: RMA_MARCH_NT(VV, 4) break;     \
  }
    if (V == 4) {
      RMA_MARCH_U(4)
    } else if (V == 2) {
      RMA_MARCH_U(2)
    } else {
      if (nts) RMA_MARCH(1, 4, true, false);
      else RMA_MARCH(1, 4, false, false);
    }
#undef RMA_MARCH_U
#undef RMA_MARCH_NT
#undef RMA_MARCH
  }
  RMA_HIP_LAUNCH_CHECK();
}

}  // namespace rma
