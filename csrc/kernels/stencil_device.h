// Device helpers shared by the one-step (stencil.hip) and two-step
// (stencil_tb.hip) register-march kernels, plus the host-side planner that
// maps a rect list onto wave tasks. Included by .hip sources only.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "rma/kernels.h"

namespace rma {
namespace march {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int64_t kColMaxWidth = 8;  // rects at most this wide run in column mode
typedef double dbl2 __attribute__((ext_vector_type(2)));  // native 16-byte vector
// 16-byte vector at 8-byte alignment: 5 cells per lane put every other lane's
// pairs on an odd cell (global_load/store_dwordx4 take dword alignment)
typedef double dbl2u __attribute__((ext_vector_type(2), aligned(8)));

// the 16-byte vector type of a V-cell row access (odd V: 8-byte aligned)
template <int V>
using dbl2v = typename std::conditional<V % 2 == 0, dbl2, dbl2u>::type;

struct RectList {
  Rect r[kMaxRects];
  int64_t xa[kMaxRects];         // strip origin (aligned down to V)
  int64_t strips[kMaxRects];
  int64_t chunks[kMaxRects];
  int64_t block_end[kMaxRects];  // inclusive prefix sum of blocks per rect
  int64_t gpad[kMaxRects];       // >0: row-aligned mapping with gpad blocks per chunk row,
                                 // 0: linear task mapping, -1: column mode (thin rects)
  int64_t crows[kMaxRects];      // pipelined kernels: rows per task of each rect
  int n;
  // frame-first fused pass (pipelined kernels; executor RMA_EXEC_FUSED): the
  // first sig_blocks blocks (the frame rects' tasks, dispatched first, never
  // XCD-remapped) count their completion in sig[0]; the last one re-arms the
  // counter and raises sig[1], which the exchange stream waits on.
  uint64_t* sig;
  int64_t sig_blocks;
};

template <int V, bool NTL = false>
__device__ __forceinline__ void load_row(double (&out)[V], const double* __restrict__ p) {
  if constexpr (V == 1) {
    out[0] = NTL ? __builtin_nontemporal_load(p) : *p;
  } else {
#pragma unroll
    for (int h = 0; h < V / 2; ++h) {
      const dbl2v<V>* q = reinterpret_cast<const dbl2v<V>*>(p + 2 * h);
      const dbl2v<V> t = NTL ? __builtin_nontemporal_load(q) : *q;
      out[2 * h] = t.x;
      out[2 * h + 1] = t.y;
    }
    if constexpr (V % 2 == 1) out[V - 1] = NTL ? __builtin_nontemporal_load(p + V - 1) : p[V - 1];
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
        dbl2v<V> t;
        t.x = v[2 * h];
        t.y = v[2 * h + 1];
        dbl2v<V>* q = reinterpret_cast<dbl2v<V>*>(p + 2 * h);
        if constexpr (NT) {
          __builtin_nontemporal_store(t, q);
        } else {
          *q = t;
        }
      }
      if constexpr (V % 2 == 1) {
        if constexpr (NT) {
          __builtin_nontemporal_store(v[V - 1], p + V - 1);
        } else {
          p[V - 1] = v[V - 1];
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

// Block b of a launch whose first `first` blocks keep dispatch order (the
// frame tasks of a fused pass) and whose rest is XCD-remapped among itself.
__device__ __forceinline__ int64_t xcd_remap_after(int64_t b, int64_t nwg, int64_t first) {
  return b < first ? b : first + xcd_remap(b - first, nwg - first);
}

// End of a signalling block (RectList::sig): every wave's stores are complete
// at workgroup scope after the barrier; thread 0's acquire-release increment
// chains them (and, through the counter, every earlier frame block's) to the
// last block's system-scope release of the flag. The last block re-arms the
// counter before raising the flag; the exchange stream lowers the flag after
// its wait (flags.hip), before the next pass can start.
__device__ __forceinline__ void signal_block_done(uint64_t* sig, int64_t nblocks) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t old =
        __hip_atomic_fetch_add(sig, (uint64_t)1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if ((int64_t)old + 1 == nblocks) {
      __hip_atomic_store(sig, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sig + 1, (uint64_t)1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Per-wave variant for kernels whose waves leave independently (the one-step
// march: column-mode threads, padding waves): lane 0 of every wave of the
// signalling blocks counts, after the wave's own stores (the release fence
// waits for all of the wave's memory operations, whatever the EXEC mask).
__device__ __forceinline__ void signal_wave_done(uint64_t* sig, int64_t nwaves) {
  if ((threadIdx.x & 63) == 0) {
    const uint64_t old =
        __hip_atomic_fetch_add(sig, (uint64_t)1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if ((int64_t)old + 1 == nwaves) {
      __hip_atomic_store(sig, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sig + 1, (uint64_t)1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
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


// Host planner: strips/chunks/blocks per rect (see stencil.hip for the block
// orders). `column_mode` enables the thin-rect column path (one-step only).
// halo > 0 (overlapped strips of the multi-step kernel): a strip loads 64V
// columns starting at a multiple of V and outputs `step` = (64V - 2*halo)
// rounded down to a multiple of V columns from position halo on;
// consecutive strips advance by step.
inline int64_t plan_rects(RectList& L, const Rect* rects, int nrects, int V, int chunk_rows,
                          int remap, bool column_mode, int halo = 0) {
  L = RectList{};
  int64_t total = 0;
  for (int i = 0; i < nrects; ++i) {
    const Rect& r = rects[i];
    if (r.empty()) continue;
    const int n = L.n++;
    L.r[n] = r;
    const int64_t sw = (int64_t)kWave * V;
    // strips start on multiples of the strip width (1 KiB of a row for V=2),
    // whatever the rect's x0: a rect starting at x=2 would otherwise make
    // every wave access straddle one extra 128-B line (measured -9%, r1)
    if (halo > 0) {
      // strip origins on multiples of V: a lane's V cells never straddle the
      // array edge (clamped loads) and 16-B accesses stay aligned
      const int64_t step = (sw - 2 * halo) / V * V;
      const int64_t x0 = r.x0 - halo;
      L.xa[n] = x0 - (((x0 % V) + V) % V);
      L.strips[n] = (r.x1 - (L.xa[n] + halo) + step - 1) / step;
    } else {
      L.xa[n] = r.x0 - (r.x0 % sw);
      L.strips[n] = (r.x1 - L.xa[n] + sw - 1) / sw;
    }
    L.chunks[n] = (r.y1 - r.y0 + chunk_rows - 1) / chunk_rows;
    int64_t blocks;
    if (column_mode && r.x1 - r.x0 <= kColMaxWidth && r.y1 - r.y0 > r.x1 - r.x0) {
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
    total += blocks;
    L.block_end[n] = total;
  }
  return total;
}

// Planner of the stage-pipelined K-step kernels (lab kernels 6-8,
// stencil_pipe.h kernels 9/10):
// one block per (strip, chunk) task, strips as in plan_rects with halo > 0;
// block b of a rect is (chunk = lb / strips, strip = lb % strips).
// sw_block: input columns of one strip task (0: one wave window, 64 V).
// rect_rows (optional): rows per task of each rect instead of chunk_rows
// (a fused pass's frame rects, RectList::sig).
inline int64_t plan_strip_tasks(RectList& L, const Rect* rects, int nrects, int V,
                                int chunk_rows, int halo, int64_t sw_block = 0,
                                const int* rect_rows = nullptr) {
  L = RectList{};
  int64_t total = 0;
  const int64_t sw = sw_block > 0 ? sw_block : (int64_t)kWave * V;
  const int64_t step = (sw - 2 * halo) / V * V;
  for (int i = 0; i < nrects; ++i) {
    const Rect& r = rects[i];
    if (r.empty()) continue;
    const int n = L.n++;
    L.r[n] = r;
    const int64_t x0 = r.x0 - halo;
    L.xa[n] = x0 - (((x0 % V) + V) % V);
    L.strips[n] = (r.x1 - (L.xa[n] + halo) + step - 1) / step;
    const int64_t cr = rect_rows && rect_rows[i] > 0 ? rect_rows[i] : chunk_rows;
    L.crows[n] = cr;
    L.chunks[n] = (r.y1 - r.y0 + cr - 1) / cr;
    L.gpad[n] = 0;
    total += L.strips[n] * L.chunks[n];
    L.block_end[n] = total;
  }
  return total;
}

// Wave task of block b (wide rects: one block row per chunk row, padded to a
// multiple of 8 blocks; narrow rects: consecutive chunks per wave). Returns
// false for padding / idle waves (the whole wave exits together).
__device__ __forceinline__ bool locate_task(const RectList& L, int ri, int64_t b, int wave,
                                            int64_t& strip, int64_t& chunk) {
  const int64_t bstart = ri ? L.block_end[ri - 1] : 0;
  const int64_t nstrips = L.strips[ri];
  if (L.gpad[ri] > 0) {
    const int64_t lb = b - bstart;
    chunk = lb / L.gpad[ri];
    strip = (lb % L.gpad[ri]) * kWavesPerBlock + wave;
    return strip < nstrips;
  }
  const int64_t task = (b - bstart) * kWavesPerBlock + wave;
  if (task >= nstrips * L.chunks[ri]) return false;
  strip = task % nstrips;
  chunk = task / nstrips;
  return true;
}

}  // namespace march
}  // namespace rma
