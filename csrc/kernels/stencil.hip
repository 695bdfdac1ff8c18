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

namespace rma {
namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int64_t kColMaxWidth = 8;  // rects at most this wide run in column mode
typedef double dbl2 __attribute__((ext_vector_type(2)));  // native 16-byte vector

struct RectList {
  Rect r[kMaxRects];
  int64_t xa[kMaxRects];         // strip origin (aligned down to V)
  int64_t strips[kMaxRects];
  int64_t chunks[kMaxRects];
  int64_t block_end[kMaxRects];  // inclusive prefix sum of blocks per rect
  int64_t gpad[kMaxRects];       // >0: row-aligned mapping with gpad blocks per chunk row,
                                 // 0: linear task mapping, -1: column mode (thin rects)
  int n;
};

template <int V, bool NTL = false>
__device__ __forceinline__ void load_row(double (&out)[V], const double* __restrict__ p) {
  if constexpr (V == 1) {
    out[0] = NTL ? __builtin_nontemporal_load(p) : *p;
  } else {
#pragma unroll
    for (int h = 0; h < V / 2; ++h) {
      const dbl2* q = reinterpret_cast<const dbl2*>(p) + h;
      const dbl2 t = NTL ? __builtin_nontemporal_load(q) : *q;
      out[2 * h] = t.x;
      out[2 * h + 1] = t.y;
    }
  }
}

template <int V, bool NT>
__device__ __forceinline__ void store_row(double* __restrict__ p, const double (&v)[V],
                                          const bool (&m)[V]) {
  if constexpr (V >= 2) {
    bool all = true;
#pragma unroll
    for (int i = 0; i < V; ++i) all = all && m[i];
    if (all) {
#pragma unroll
      for (int h = 0; h < V / 2; ++h) {
        dbl2 t;
        t.x = v[2 * h];
        t.y = v[2 * h + 1];
        dbl2* q = reinterpret_cast<dbl2*>(p) + h;
        if constexpr (NT) {
          __builtin_nontemporal_store(t, q);
        } else {
          *q = t;
        }
      }
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) {
    if (m[i]) {
      if constexpr (NT) {
        __builtin_nontemporal_store(v[i], p + i);
      } else {
        p[i] = v[i];
      }
    }
  }
}

// XCD-aware block order. Workgroups are dealt round-robin over the 8 XCDs
// (block b runs on XCD b % 8; MI355X_MICROARCH.md §Workgroup dispatch). The
// march tasks are numbered row-chunk-major, strip-group fastest, so
// vertically adjacent chunks share a halo row and horizontally adjacent ones
// share edge cache lines. Giving each XCD a CONTIGUOUS 1/8 of the task range
// keeps both neighbours on the same XCD (same L2) whatever the strip count.
// Bijective for any grid size (cdna_hip_programming.md "XCD swizzle must be
// bijective"). Speed only: any mapping computes the same cells.
__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nwg) {
  constexpr int64_t kXcd = 8;
  if (nwg < kXcd) return b;
  const int64_t q = nwg / kXcd, r = nwg % kXcd;
  const int64_t xcd = b % kXcd, slot = b / kXcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

// The canonical cell update (see rma/common.h StencilCoef). Compiled with
// -ffp-contract=off: every operation rounds exactly as written, in this order.
__device__ __forceinline__ double cell(double xl, double c, double xr, double up, double dn,
                                       double ic, const StencilCoef& k) {
  const double qxR = (k.mlam * (xr - c)) * k.rdx;
  const double qxL = (k.mlam * (c - xl)) * k.rdx;
  const double qyU = (k.mlam * (dn - c)) * k.rdy;
  const double qyD = (k.mlam * (c - up)) * k.rdy;
  return c + k.dt * (ic * ((-(qxR - qxL)) * k.rdx - (qyU - qyD) * k.rdy));
}

template <int V>
__device__ __forceinline__ void row_update(double (&res)[V], const double (&up)[V],
                                           const double (&cu)[V], const double (&dn)[V],
                                           const double (&ic)[V], double edge, int lane,
                                           const StencilCoef& k) {
  // x-neighbours across lanes: lane-1's last cell, lane+1's first cell.
  double left = __shfl_up(cu[V - 1], 1);
  double right = __shfl_down(cu[0], 1);
  if (lane == 0) left = edge;
  if (lane == kWave - 1) right = edge;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const double xl = (v == 0) ? left : cu[v - 1];
    const double xr = (v == V - 1) ? right : cu[v + 1];
    res[v] = cell(xl, cu[v], xr, up[v], dn[v], ic[v], k);
  }
}

template <int V, bool NT, int kUnroll, bool NTL, bool NTT = false>
__global__ __launch_bounds__(kBlock) void stencil_march_kernel(double* __restrict__ T2,
                                                               const double* __restrict__ T,
                                                               const double* __restrict__ iCp,
                                                               int64_t nx, RectList L,
                                                               StencilCoef k, int chunk_rows,
                                                               int remap) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = remap ? xcd_remap(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
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
  const int64_t nstrips = L.strips[ri];
  int64_t strip, chunk;
  if (L.gpad[ri] > 0) {
    // wide rect: one block row per chunk row, padded to a multiple of 8 blocks so
    // the chunk below runs on the same XCD (shares its halo row through L2)
    // while the whole chip still streams one compact band of rows
    const int64_t lb = b - bstart;
    chunk = lb / L.gpad[ri];
    strip = (lb % L.gpad[ri]) * kWavesPerBlock + wave;
    if (strip >= nstrips) return;  // padding / last partial group
  } else {
    // narrow rect (< 4 strips, e.g. perf_hide x-frames): the block's waves take
    // consecutive chunks so none idles
    const int64_t task = (b - bstart) * kWavesPerBlock + wave;
    if (task >= nstrips * L.chunks[ri]) return;  // whole wave exits together
    strip = task % nstrips;
    chunk = task / nstrips;
  }
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

// ---------------------------------------------------------------------------
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

int stencil_vec(int64_t nx, const StencilTuning& tune) {
  // cells per lane: 16-byte rows need an even nx; V=4 also needs nx % 4 == 0
  // (a clamped lane past the row end must still load its own cells)
  if (nx % 2) return 1;
  if (tune.vec == 4 && nx % 4 == 0) return 4;
  return 2;
}

int stencil_strip_cells(int64_t nx, const StencilTuning& tune) {
  return kWave * stencil_vec(nx, tune);
}

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
  const bool lds = tune.kernel == 1;
  RectList L{};
  int64_t total = 0;
  for (int i = 0; i < nrects; ++i) {
    const Rect& r = rects[i];
    if (r.empty()) continue;
    const int n = L.n++;
    L.r[n] = r;
    int64_t blocks;
    if (lds) {
      L.xa[n] = r.x0;
      L.strips[n] = (r.x1 - r.x0 + kTileX - 1) / kTileX;
      L.chunks[n] = (r.y1 - r.y0 + kTileY - 1) / kTileY;
      blocks = L.strips[n] * L.chunks[n];
    } else {
      const int64_t sw = (int64_t)kWave * V;
      // strips start on multiples of the strip width (1 KiB of a row for V=2),
      // whatever the rect's x0: a rect starting at x=2 would otherwise make
      // every wave access straddle one extra 128-B line (measured -9%, r1)
      L.xa[n] = r.x0 - (r.x0 % sw);
      L.strips[n] = (r.x1 - L.xa[n] + sw - 1) / sw;
      L.chunks[n] = (r.y1 - r.y0 + tune.chunk_rows - 1) / tune.chunk_rows;
      if (r.x1 - r.x0 <= kColMaxWidth && r.y1 - r.y0 > r.x1 - r.x0) {
        L.gpad[n] = -1;  // thin column: one thread per row
        blocks = (r.y1 - r.y0 + kBlock - 1) / kBlock;
      } else if (L.strips[n] >= kWavesPerBlock && !remap) {
        const int64_t groups = (L.strips[n] + kWavesPerBlock - 1) / kWavesPerBlock;
        L.gpad[n] = (groups + 7) / 8 * 8;
        blocks = L.gpad[n] * L.chunks[n];
      } else {
        L.gpad[n] = 0;
        blocks = (L.strips[n] * L.chunks[n] + kWavesPerBlock - 1) / kWavesPerBlock;
      }
    }
    total += blocks;
    L.block_end[n] = total;
  }
  if (L.n == 0) return;
  RMA_CHECK_ARG(total < (int64_t(1) << 31), "grid too large: " << total << " blocks");
  const dim3 grid((unsigned)total), block(kBlock);
  hipStream_t s = as_stream(stream);
  if (lds) {
    if (tune.nontemporal)
      stencil_lds_kernel<true><<<grid, block, 0, s>>>(T2, T, iCp, nx, L, c);
    else
      stencil_lds_kernel<false><<<grid, block, 0, s>>>(T2, T, iCp, nx, L, c);
  } else {
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
