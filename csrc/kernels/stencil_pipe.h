// Stage-pipelined K-step kernel for ANY K (1..kPipeMaxK), fast5 or canonical
// arithmetic. Included by the stencil_pipe_*.hip translation units only.
//
// One block = one (strip, row-chunk) task; its S waves split the K time levels
// of the strip: stage s < S-1 owns H = ceil(K/S) levels, the last stage the
// remaining HL = K - (S-1)H (1 <= HL <= H). Stage 0 streams T and 1/Cp from
// HBM, writes the per-strip factor ring (R = K+S-1 rows, plus H-1 mirrored
// rows where they cost no occupancy) in LDS and runs its levels; stage s
// reads its input level from an LDS hand-off row that stage s-1 wrote one
// row-iteration earlier and runs s(H+1) rows behind stage 0; the last stage
// stores. One barrier per row iteration. Measured: profiles/SUMMARY_r2.md,
// profiles/pmc_pipe_r2.md (what was tried and not kept is listed there).
//
// Generalises kernels 6-8 of csrc/lab/stencil_kstep_lab.hip (fixed K in {8,12,16}, H = K/S)
// so that the executor's pass planner (executor.cpp plan_passes) can run a
// pass of any depth: e.g. the 20 timed steps of the driver's bench command as
// ONE 20-step pass (~70 ms) instead of 16 + 4 (each pass costs at least one
// HBM sweep of the 3 arrays, ~40 ms at the 288 GB tile).
//
// Arithmetic (template Ar: kArFast5 = 0, kArCanon = 1; kArFast5Perm = 2 is
// fast5 with the lane moves done by ds_bpermute on the LDS pipe instead of
// DPP on the VALU, an energy / issue experiment, profiles/SUMMARY_r2.md):
//   false  fast5: T2 = fma(g, fma(r, U+D, fma(-2(1+r), c, L+R)), c), g = dt*lam/dx^2/Cp
//          (LDS ring holds g, zero outside the interior). Bitwise equal to
//          kernel 5 (csrc/lab) and to the CPU twin stencilk5_rects_cpu.
//   true   the canonical flux form of rma/common.h (scripts/diffusion_2D_perf.jl:8-10
//          with 1/Cp): x face flux shared with the left lane, y face flux
//          carried from the previous row; bitwise equal to K one-step launches.
//          The ring holds 1/Cp (zero outside the interior: c + dt*(0*...) == c).
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "pipe_arith.h"
#include "rma/common.h"
#include "rma/hip_check.h"
#include "rma/kernels.h"
#include "stencil_device.h"

namespace rma {
namespace pipe {
using namespace march;

template <int K, int S>
struct Plan {
  static constexpr int H = (K + S - 1) / S;       // levels of stages 0..S-2
  static constexpr int HL = K - (S - 1) * H;      // levels of the last stage
  static constexpr int R = K + S - 1;             // factor ring rows
  static_assert(S >= 1 && HL >= 1 && HL <= H, "bad stage split");
};

// Five cells per lane (fast5, one column wave): 320-column windows recompute
// 2K of 320 columns instead of 2K of 256 (K=24: 1.185x vs 1.231x, K=20:
// 1.143x vs 1.185x fp64 work) and move 4 lane values per 5 cells instead of
// per 4. Two blocks per CU need <= 80 KiB of LDS per block, so at V = 5:
//  * LDS rows are v-major (cell v of lane l at v*64 + l): every access is a
//    contiguous 512-B ds_*_b64 per v (no bank conflicts at 40-B lane pitch),
//    and rows sit on 512-B multiples, so one base VGPR with immediate
//    offsets (ds_read2st64_b64) reaches every row of the ring;
//  * stage 0 writes its factor row one iteration late (row i-1 at iteration
//    i, levels 1/2 use the factors of rows i/i-1 from registers), which saves
//    one ring row: R = K + S - 2 (K=20: 22 + 4 mirrors + 6 hand-off rows =
//    exactly 80 KiB; without mirrors the level loop takes one immediate-
//    offset path whenever the stage's rows do not wrap).
// Registers bound the depth: K <= 20 (236 VGPRs at K = 20; the 6-level
// stages of K >= 21 spill). An experiment in the lab library
// (csrc/lab/stencil_pipe5_lab.hip): 0.8-1.6 % per K=20 pass.
template <int V>
constexpr bool kDelayedRing = V == 5;
template <int K, int S, int V>
constexpr int ring_rows() {
  return Plan<K, S>::R - (kDelayedRing<V> ? 1 : 0);
}

// Block geometry with C column waves per stage (C = 1: one 64V-column window
// per strip). With C > 1 the C waves of a stage sit D = 64V - 2*Hp columns
// apart (Hp = H rounded up to even) and all exchange through the block-wide
// LDS rows once per row iteration, so a stage boundary inside the block
// recomputes only ~2H columns instead of the strip's 2K: the block of
// WB = (C-1) D + 64V input columns outputs WB - 2K (K=24, C=2: 452 of 500
// columns, 1.13x recompute against 1.23x for C = 1).
template <int K, int S, int V, int C>
struct Geo {
  static constexpr int W = kWave * V;                // one wave's window
  static constexpr int Hp = (Plan<K, S>::H + 1) / 2 * 2;
  static constexpr int D = C > 1 ? W - 2 * Hp : W;   // wave stride inside the block
  static constexpr int WB = (C - 1) * D + W;         // block row columns
  static constexpr int kStep = (WB - 2 * K) / V * V; // output columns per strip
  static_assert(C == 1 || (V == 4 && D % 4 == 0 && D > 2 * K / S), "bad column split");
};

// Waves per SIMD a block shape allows: the LDS (160 KiB per CU, 4 SIMDs)
// and a VGPR estimate, so a waves_per_eu cap never forces spills: fast5
// 3 rows x V cells x 2 dwords per level, stage 0's two-row prefetch, ~40 for
// addressing and temporaries; canonical also the carried y flux and the x
// fluxes (checked: no spills at any K, V, scripts/check_isa.py).
// arithmetic template ids (kAr*), ar_reg / ar_split: pipe_arith.h (host-safe)

template <int K, int S, int V, bool Canon, int C = 1>
constexpr int occupancy(int lds) {
  const int by_lds = (160 * 1024) / lds * S * C / 4;
  // (V = 5: 142-150 VGPRs measured at K = 20/24, the V <= 4 estimate would claim 1 wave)
  const int vgpr = Canon ? 8 * Plan<K, S>::H * V + 8 * V + 64
                         : (V == 5 ? 5 : 6) * Plan<K, S>::H * V + 8 * V + 40;
  const int by_vgpr = 512 / ((vgpr + 7) / 8 * 8);
  const int w = by_lds < by_vgpr ? by_lds : by_vgpr;
  return w < 1 ? 1 : (w > 8 ? 8 : w);
}

// Mirror rows of the factor ring: the H levels of a stage read the ring rows
// of H consecutive slots (descending); with the last H-1 slots mirrored in
// front of slot 0 the reads never wrap, so one base address and immediate
// ds_read offsets serve all levels (no per-level modulo and address VALU op:
// -3 % VALU, -50 % SALU instructions in the K=24 row loop). Only where the
// extra rows cost no occupancy.
template <int K, int S, int V, bool Canon, int C = 1>
constexpr int mirror_rows() {
  constexpr int H = Plan<K, S>::H, row = Geo<K, S, V, C>::WB * 8;
  constexpr int base = (ring_rows<K, S, V>() + 2 * (S > 1 ? S - 1 : 1)) * row;
  return occupancy<K, S, V, Canon, C>(base + (H - 1) * row) ==
                 occupancy<K, S, V, Canon, C>(base)
             ? H - 1
             : 0;
}

// LDS bytes of one block (ring + mirrors + double-buffered hand-off rows)
template <int K, int S, int V, bool Canon, int C = 1>
constexpr int lds_bytes() {
  return (ring_rows<K, S, V>() + mirror_rows<K, S, V, Canon, C>() + 2 * (S > 1 ? S - 1 : 1)) *
         Geo<K, S, V, C>::WB * 8;
}

template <int K, int S, int V, bool Canon, int C = 1>
constexpr int waves_per_simd() {
  return occupancy<K, S, V, Canon, C>(lds_bytes<K, S, V, Canon, C>());
}

// Register-resident factors (Ar = kArFast5Reg, "piper"): no factor ring. A
// stage keeps the factor rows of its H levels in registers (a shift register:
// level j+1 uses next row iteration the row level j uses now), and each stage
// hands the row it retires to the next stage through a double-buffered LDS
// row, like the T hand-off. LDS read bytes per cell update: the ring's one
// factor row per level -> one factor row per stage (H levels); LDS per
// block: 4 (S-1) rows.
#ifndef RMA_PIPE_U6
#define RMA_PIPE_U6 1
#endif
constexpr bool kPipeU6 = RMA_PIPE_U6;
#ifndef RMA_PIPE_U6_H6  // experiments only: unroll by 6 also at H = 6 (spills, see below)
#define RMA_PIPE_U6_H6 0
#endif
// Register factors: a factor row lives H iterations and a new one starts
// every iteration, so with the row loop unrolled by U < H the row started at
// phase p is still live when the next trip's phase-p row starts and the back
// edge has to move every row (20 v_mov_b64 per 3 rows at K=20: ~5 % of the
// VALU instructions). Unrolled by 6 >= H the rows keep their registers across
// the back edge (K=20: 2 moves per 6 rows in stages 1..3). Only H = 5 (K =
// 17..20): H = 6 (K >= 21) spills 39 VGPRs at K=24, and H = 4 (K = 13..16)
// takes 214 instead of 161 VGPRs at K=16 (2 instead of 3 waves per SIMD);
// K=20: 247 instead of 201 VGPRs, no spill, still 2 waves per SIMD.
template <int K, int S, int Ar>
constexpr bool pipe_u6() {
  return ar_reg(Ar) && kPipeU6 && Ar != kArFast5RegU3 &&
         (Plan<K, S>::H == 5 ||
          ((Ar == kArFast5RegW1 || Ar == kArFast5RegU6S || (RMA_PIPE_U6_H6 && Ar == kArFast5Reg)) &&
           Plan<K, S>::H == 6));
}
// LDS-DMA staging rows per array: one per phase of the unrolled row loop, so
// a row DMA'd at phase p is read at phase p of the next loop trip (across the
// back edge: a read of a slot DMA'd earlier in the same trip gets a vmcnt(0)
// from the compiler's LDS-DMA hazard check, which drains the prefetch)
template <int K, int S, int Ar>
constexpr int staging_rows() {
  return pipe_u6<K, S, Ar>() ? 6 : 3;
}
// T + factor hand-off rows (block-wide, WB columns), LDS-DMA staging (V = 2, 4;
// private to each column's stage-0 wave, W columns each)
template <int K, int S, int V, int Ar, int C = 1>
constexpr int lds_bytes_reg() {
  return (4 * (S > 1 ? S - 1 : 1) * Geo<K, S, V, C>::WB +
          (V == 2 || V == 4 ? 2 * staging_rows<K, S, Ar>() * Geo<K, S, V, C>::W * C : 0)) *
             8 +
         8;
}
template <int K, int S, int V, int Ar, int C>
constexpr int kernel_waves() {
  if constexpr (ar_reg(Ar)) {
    // + the H factor rows (measured 158 / 233 / 256 VGPRs at K = 12 / 20 / 24, V = 4)
    constexpr int H = Plan<K, S>::H;
    constexpr int vgpr = 8 * H * V + 8 * V + 40;
    constexpr int by_vgpr = 512 / ((vgpr + 7) / 8 * 8);
    constexpr int w = occupancy<K, S, V, false, C>(lds_bytes_reg<K, S, V, Ar, C>());
    if constexpr (Ar == kArFast5RegW1) return 1;
    return by_vgpr < 2 ? 2 : (by_vgpr < w ? by_vgpr : w);
  } else {
    return waves_per_simd<K, S, V, Ar == kArCanon, C>();
  }
}

template <bool kDpp = true>
__device__ __forceinline__ double from_next_lane(double v) {
  if constexpr (kDpp) {
    // wave_shl:1 (lane i <- lane i+1); bound_ctrl: lane 63 reads 0 (invalid column)
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x130, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
  } else {
    return __shfl_down(v, 1);  // ds_bpermute x2 (LDS pipe); lane 63: its own value
  }
}
template <bool kDpp = true>
__device__ __forceinline__ double from_prev_lane(double v) {
  if constexpr (kDpp) {
    // wave_shr:1 (lane i <- lane i-1); lane 0 reads 0 (invalid column)
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x138, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
  } else {
    return __shfl_up(v, 1);  // lane 0: its own value (an invalid column either way)
  }
}

// Direct-store halos of one stored row (DirectStores, kernels.h): the row's
// images in the neighbours in directions d = (i, j) (executor.h kDirI /
// kDirJ order) whose ranges hold it. dxm / dxp: the wave stores columns in the
// i = -1 / +1 ranges (uniform, per task). The lane masks are recomputed per
// row rather than held in registers across the row loop.
template <int V>
__device__ __forceinline__ void direct_row(const DirectStores& D, int row, int64_t nx, int x32,
                                           int64_t e, const double (&res)[V],
                                           const bool (&m)[V], bool dxm, bool dxp) {
  // e: element index of the lane's first cell, x32 its column
  const bool ym = row >= D.ym0 && row < D.ym1, yp = row >= D.yp0 && row < D.yp1;
  const int64_t sx = D.sx, sy = D.syr * nx;
  auto put = [&](int d, int64_t off, const bool (&mk)[V]) {
    if (D.dst[d]) store_row<V, true>(D.dst[d] + (e + off), res, mk);
  };
  if (ym) put(1, sy, m);   // (0, -1)
  if (yp) put(6, -sy, m);  // (0, +1)
  // the x-image columns, with their diagonal images in the y-image rows
  auto xside = [&](int dx, int dd0, int dd1, int64_t ox, int32_t a0, int32_t a1) {
    bool mk[V];
#pragma unroll
    for (int v = 0; v < V; ++v) mk[v] = m[v] && x32 + v >= a0 && x32 + v < a1;
    put(dx, ox, mk);
    if (ym) put(dd0, ox + sy, mk);
    if (yp) put(dd1, ox - sy, mk);
  };
  if (dxm) xside(3, 0, 5, sx, D.xm0, D.xm1);    // (-1, 0), (-1, -1), (-1, +1)
  if (dxp) xside(4, 2, 7, -sx, D.xp0, D.xp1);   // (+1, 0), (+1, -1), (+1, +1)
}

template <int K, int S, int V, int Ar, int C, bool Dir>
__device__ __forceinline__ void pipe_body(double* __restrict__ T2, const double* __restrict__ T,
                                          const double* __restrict__ iCp, int64_t nx, int64_t ny,
                                          const RectList& L, const StencilCoef& k, int chunk_rows,
                                          int remap, const DirectStores& DS) {
  using P = Plan<K, S>;
  constexpr bool Canon = Ar == kArCanon, kDpp = Ar != kArFast5Perm, kRegG = ar_reg(Ar);
  static_assert(!kRegG || (V != 5 && (C == 1 || V == 4)),
                "register factors: V <= 4; two column waves at V = 4 only");
  // register factors, 2 or 4 cells per lane: stage 0 prefetches T / 1/Cp three
  // rows ahead by LDS-DMA (global_load_lds_dwordx4 into three staging rows per
  // array) instead of two rows ahead into 4 rows of registers, which the
  // register factors need (K=24: 256 VGPRs + 6 spilled with the register
  // prefetch; with T one row ahead 251 VGPRs but the HBM latency shows: 92.7 vs
  // 81.6 ms per pass; with LDS-DMA 234 VGPRs). The row barrier is then a raw
  // s_barrier after lgkmcnt(0): __syncthreads() would also wait vmcnt(0) and
  // drain the prefetch every row.
  constexpr bool kGlds = kRegG && (V == 2 || V == 4);
  constexpr bool kU6 = pipe_u6<K, S, Ar>();
  constexpr int NST = staging_rows<K, S, Ar>();  // staging rows per array
  using G = Geo<K, S, V, C>;
  constexpr int H = P::H, HL = P::HL, R = ring_rows<K, S, V>();
  constexpr int M = kRegG ? 0 : mirror_rows<K, S, V, Canon, C>();
  constexpr bool kDelay = kDelayedRing<V>;
  static_assert(V != 5 || (C == 1 && Ar == kArFast5), "5 cells per lane: fast5, one column wave");
  constexpr int W = G::W, WB = G::WB, D = G::D;
  constexpr int kStep = G::kStep;  // output columns per strip (plan_strip_tasks, sw = WB)
  constexpr int NH = S > 1 ? S - 1 : 1;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = C > 1 ? wv / S : 0;
  // waves c*S .. c*S+S-1: column c, one per SIMD (waves are dealt to SIMDs in
  // order). Rotated maps: odd blocks (C = 1) / column 1 (C = 2) start at SIMD
  // 2, so no SIMD hosts two stage-0 waves
  const int stage = (Ar == kArFast5RegRot || Ar == kArFast5RegPrio)
                        ? (C > 1 ? (wv % S + 2 * col) % S : (wv + 2 * (int)(blockIdx.x & 1)) % S)
                        : wv % S;
  const int lane = threadIdx.x & (kWave - 1);
  if constexpr (Ar == kArFast5RegPrio || Ar == kArFast5RegPrioNR) {
    if (stage == 0) __builtin_amdgcn_s_setprio(2);  // wave-uniform
  }
  const int64_t sig_first = L.sig ? L.sig_blocks : 0;
  const int64_t b = remap ? xcd_remap_after(blockIdx.x, gridDim.x, sig_first) : (int64_t)blockIdx.x;
  int ri = 0;
  while (ri < L.n - 1 && b >= L.block_end[ri]) ++ri;
  const int64_t lb = b - (ri ? L.block_end[ri - 1] : 0);
  const int64_t strip = lb % L.strips[ri], chunk = lb / L.strips[ri];
  const Rect r = L.r[ri];
  const int64_t xs = L.xa[ri] + strip * kStep;
  const int64_t crows = L.crows[ri];  // == chunk_rows unless a fused pass's frame rect
  const int64_t ya = r.y0 + chunk * crows;
  const int64_t yb = min(r.y1, ya + crows);

  // the columns [lo, hi) of this wave's window it writes to the block rows
  // (the stage boundary with the neighbouring column wave at the window
  // offsets Hp and D + Hp, inside both waves' valid ranges)
  const int lo = col > 0 ? G::Hp : 0, hi = col < C - 1 ? D + G::Hp : W;
  const int64_t xw = xs + (int64_t)col * D;  // window origin
  const int64_t x = xw + (int64_t)lane * V;
  bool m[V], cin[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int p = lane * V + v, pb = col * D + p;
    m[v] = pb >= K && pb < K + kStep && p >= lo && p < hi && x + v >= r.x0 && x + v < r.x1;
    cin[v] = (x + v >= 1) && (x + v <= nx - 2);
  }
  const int64_t xl = min(max(x, (int64_t)0), nx - V);
  // 32-bit lane offsets from a uniform row pointer (SGPR base + VGPR offset
  // addressing instead of 64-bit VGPR address arithmetic); xso wraps only for
  // lanes left of the array, which never store (m[] false)
  const uint32_t xo = (uint32_t)xl, xso = (uint32_t)x;
  // byte offsets in 32 bits: uniform 64-bit row base + zero-extended 32-bit
  // offset is the SGPR-base + VGPR-offset (saddr) addressing form
  const uint32_t xob = xo * 8u, xsob = xso * 8u;
  auto at = [](const double* base, uint32_t boff) {
    return reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + boff);
  };
  const bool xin = xw >= 1 && xw + W - 1 <= nx - 2;  // no x-boundary cell in the window
  // direct-store halos (DirectStores): does this wave store into the x-image
  // ranges (a lane with a stored column there), do its rows meet the y ones
  bool dxm = false, dxp = false, dtask = false;
  if constexpr (Dir) {
    bool pm = false, pp = false;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      pm = pm || (m[v] && x + v >= DS.xm0 && x + v < DS.xm1);
      pp = pp || (m[v] && x + v >= DS.xp0 && x + v < DS.xp1);
    }
    dxm = __builtin_amdgcn_ballot_w64(pm) != 0;
    dxp = __builtin_amdgcn_ballot_w64(pp) != 0;
    const bool tym = ya < DS.ym1 && yb > DS.ym0, typ = ya < DS.yp1 && yb > DS.yp0;
    dtask = dxm || dxp || tym || typ;
  }

  // fast5 constants (the host guarantees fast5_ok); canonical uses k directly
  const double ax = (-k.mlam) * k.rdx * k.rdx;
  const double ay = (-k.mlam) * k.rdy * k.rdy;
  const double ry = Canon ? 0.0 : ay / ax;
  const double mkc = -2.0 * (1.0 + ry);
  const double gs = Canon ? 1.0 : k.dt * ax;

  // w[0]: the stage's input level; w[j]: local level j (j < levels); slots
  // rotate mod 3 with the row iteration (new row -> slot P, centre (P+2)%3,
  // up (P+1)%3). Canon carries the y face flux fy[j] instead of reading `up`.
  double w[H][3][V], fy[Canon ? H : 1][V], pT[V], pC[V], qT[V], qC[V];
#pragma unroll
  for (int j = 0; j < H; ++j)
#pragma unroll
    for (int v = 0; v < V; ++v) {
      w[j][0][v] = w[j][1][v] = w[j][2][v] = 0.0;
      fy[Canon ? j : 0][v] = 0.0;
    }
  // 32-bit row bookkeeping (host checks ny < 2^30): no 64-bit VALU compares
  const int ny32 = (int)ny, ya32 = (int)ya, yb32 = (int)yb;
  int i = ya32 - K;
  const int iend = yb32 + K - 3 + S;
  auto rowc = [&](int y) { return (int64_t)min(max(y, 0), ny32 - 1); };
  auto rowp = [&](const double* a, int y) { return at(a + rowc(y) * nx, xob); };
  if (stage == 0) {
    load_row<V>(w[0][2], rowp(T, i));
    if constexpr (!kGlds) {
      load_row<V>(pT, rowp(T, i + 1));
      load_row<V>(pC, rowp(iCp, i));
      load_row<V>(qT, rowp(T, i + 2));
      load_row<V>(qC, rowp(iCp, i + 1));
    }
  }
  // ring: physical row M + s holds slot s; rows [0, M) mirror slots [R-M, R).
  // Register factors: no ring; the factor hand-off rows follow the T hand-off
  // rows in `hand` ([2][NH][WB] each), and the LDS-DMA staging rows are an
  // array of their own (T rows 0..2, 1/Cp rows 3..5; referenced by kGlds code
  // only, so other instantiations allocate nothing for it): the compiler's
  // LDS-DMA hazard check then sees the hand-off writes and the DMA on distinct
  // objects and waits for no DMA before them
  constexpr int kRing = kRegG ? 1 : (R + M) * WB, kHand = kRegG ? 4 : 2;
  __shared__ double ring[kRing];
  __shared__ double hand[kHand][NH][WB];
  __shared__ double staging[kGlds ? 2 * NST * W * C : 1];  // per column wave
  if constexpr (!kRegG)
    for (int t = threadIdx.x; t < kRing; t += S * C * kWave) ring[t] = 0.0;
  for (int t = threadIdx.x; t < kHand * NH * WB; t += S * C * kWave) (&hand[0][0][0])[t] = 0.0;
  // register factors: gr[j-1] = the factor row of level j, shifted one level
  // per row iteration (level j+1 computes next iteration the row level j
  // computes now); the shift is SSA renaming, the loop back-edge costs the
  // register allocator a few row copies per 3 rows (the row loop stays
  // unrolled by 3: unrolling by 6 for static names raised the VGPR count of
  // the plain kernel from 213 to 270)
  double gr[kRegG ? H : 1][V];
#pragma unroll
  for (int q = 0; q < (kRegG ? H : 1); ++q)
#pragma unroll
    for (int v = 0; v < V; ++v) gr[q][v] = 0.0;
  auto gh = [&](int pb, int st) { return &hand[2 + pb][st][0]; };
  auto gshift = [&]() {
#pragma unroll
    for (int q = (kRegG ? H : 1) - 1; q > 0; --q)
#pragma unroll
      for (int v = 0; v < V; ++v) gr[q][v] = gr[q - 1][v];
  };
  __syncthreads();
  // LDS-DMA staging row of T (a = 0) / 1/Cp (a = 1) for relative row r (mod NST),
  // the column wave's own (only its stage-0 wave writes and reads it):
  // instruction h, lane l loads the cell pair 2l+h of the lane's window, which
  // lands at dbl2 slot h*64 + l (the one-window layout rds reads)
  auto stg = [&](int a, int r) { return &staging[((2 * col + a) * NST + r) * W]; };
  auto glds_row = [&](int a, int y, int r) {
    const double* rb = (a ? iCp : T) + rowc(y) * nx;
#pragma unroll
    for (int h = 0; h < V / 2; ++h)
      __builtin_amdgcn_global_load_lds(at(rb, xob + 16u * h), stg(a, r) + h * 2 * kWave, 16, 0, 0);
  };
  if constexpr (kGlds) {
    if (stage == 0) {  // rows i+1..i+NST of T and i..i+NST-1 of 1/Cp, in the order they are waited for
#pragma unroll
      for (int r = 0; r < NST; ++r) {
        glds_row(0, i + 1 + r, r);
        glds_row(1, i + r, r);
      }
    }
  }
  // LDS rows hold cell pairs interleaved by parity (pair p at dbl2 slot
  // (p & 1) * WB/4 + p/2): a wave window starting at an even pair (D % 4 == 0)
  // reads/writes each of its two pairs per lane as one contiguous 1 KiB
  // ds_read/write_b128, no bank conflicts (C = 1: slot h*64 + lane).
  constexpr int NPH = V == 4 ? WB / 4 : kWave;
  const int cq = col * (D / 4);
  auto rd2 = [&](const double* row, double (&out)[V]) {
    if constexpr (V == 1) {
      out[0] = row[lane];
    } else if constexpr (V == 5) {
#pragma unroll
      for (int v = 0; v < V; ++v) out[v] = row[v * kWave + lane];
    } else {
#pragma unroll
      for (int h = 0; h < V / 2; ++h) {
        const dbl2 t2 = reinterpret_cast<const dbl2*>(row)[h * NPH + cq + lane];
        out[2 * h] = t2.x;
        out[2 * h + 1] = t2.y;
      }
    }
  };
  auto rds = [&](const double* row, double (&out)[V]) {  // a staging row (V = 2, 4)
#pragma unroll
    for (int h = 0; h < V / 2; ++h) {
      const dbl2 t2 = reinterpret_cast<const dbl2*>(row)[h * kWave + lane];
      out[2 * h] = t2.x;
      out[2 * h + 1] = t2.y;
    }
  };
  auto wr2 = [&](double* row, const double (&in)[V]) {
    if constexpr (V == 1) {
      row[lane] = in[0];
    } else if constexpr (V == 5) {
#pragma unroll
      for (int v = 0; v < V; ++v) row[v * kWave + lane] = in[v];
    } else {
#pragma unroll
      for (int h = 0; h < V / 2; ++h) {
        dbl2 t2;
        t2.x = in[2 * h];
        t2.y = in[2 * h + 1];
        if (C == 1 || (lane * V + 2 * h >= lo && lane * V + 2 * h < hi))
          reinterpret_cast<dbl2*>(row)[h * NPH + cq + lane] = t2;
      }
    }
  };
  int slot0 = 0;  // ring slot of row i (stage 0's level-1 row)
  double gp[V];   // delayed ring: stage 0's factors of row i-1
#pragma unroll
  for (int v = 0; v < V; ++v) gp[v] = 0.0;
  int par = 0;
  const int lag = stage * (H + 1);  // rows behind stage 0
  // kArFast5RegMask: per local level, is any of this lane's cells inside the
  // level's valid cone (loop-invariant lane masks, kept in SGPR pairs)
  constexpr bool kMask = (Ar == kArFast5RegMask || Ar == kArFast5RegMaskCtl) && V == 4;  // other V: plain piper
  uint64_t amask[kMask ? H : 1];
#pragma unroll
  for (int j = 1; j <= (kMask ? H : 1); ++j) {
    const int l = stage * H + j;
    amask[j - 1] = __ballot(Ar == kArFast5RegMaskCtl || (lane * V + V > l && lane * V < W - l));
  }

  auto iter = [&](auto Pc, auto S0c, auto LASTc) {
    constexpr int Ps = decltype(Pc)::value;  // phase of the unrolled loop (staging slot)
    constexpr int Pr = Ps % 3;                // phase of the 3-row windows w
    constexpr bool S0 = decltype(S0c)::value;
    constexpr bool LAST = decltype(LASTc)::value;
    constexpr int NL = LAST ? HL : (S0 && Ar == kArDiagS0 ? H - 1 : H);  // levels of this stage
    constexpr int PC = (Pr + 2) % 3, PU = (Pr + 1) % 3;
    double g[V];
    if constexpr (S0) {
      // register factors: retire level H's row to stage 1 before row i's
      // factors exist (one factor row fewer live)
      if constexpr (kRegG && !LAST) wr2(gh(par, 0), gr[H - 1]);
      const bool rin1 = i >= 1 && i <= ny32 - 2;
      if constexpr (kGlds) {
        // NST (3, or 6 when unrolled by 6) rows ahead: the staging slot of this
        // iteration's rows (T i+1, 1/Cp i) is the unrolled phase (the loop
        // starts at phase 0), and their DMA (issued NST iterations ago, at this
        // phase of the previous loop trip) has landed when at most the NST-1
        // later iterations' 2 x V/2 instructions are outstanding. Same-phase
        // slots keep every DMA -> read pair across the loop back-edge, where the
        // compiler's LDS-DMA hazard check adds no vmcnt(0) (a read of a slot
        // DMA'd earlier in the same trip got one, whatever the counted wait
        // before it). The builtin (gfx9 encoding: vmcnt bits 3:0 and 15:14,
        // expcnt 6:4 and lgkmcnt 11:8 at their maxima = no wait) plus an empty
        // asm keeps the reads below the wait.
        constexpr int kVm = (NST - 1) * V;
        static_assert(kVm < 64, "vmcnt");
        __builtin_amdgcn_s_waitcnt(0x0F70 | (kVm & 15) | ((kVm >> 4) << 14));
        asm volatile("" ::: "memory");
        rds(stg(0, Ps), pT);
        rds(stg(1, Ps), pC);
      }
#pragma unroll
      for (int v = 0; v < V; ++v) w[0][Pr][v] = pT[v];
      if (rin1 && xin) {  // wave-uniform: no per-cell selects away from the x edges
#pragma unroll
        for (int v = 0; v < V; ++v) g[v] = Canon ? pC[v] : gs * pC[v];
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) g[v] = (rin1 && cin[v]) ? (Canon ? pC[v] : gs * pC[v]) : 0.0;
      }
      if constexpr (kRegG) {  // shift, take row i
        gshift();
#pragma unroll
        for (int v = 0; v < V; ++v) gr[0][v] = g[v];
      } else if constexpr (kDelay) {  // row i-1's factors, kept from the previous iteration
        const int sp = slot0 == 0 ? R - 1 : slot0 - 1;
        wr2(ring + (sp + M) * WB, gp);
        if constexpr (M > 0) {
          if (sp >= R - M) wr2(ring + (sp - (R - M)) * WB, gp);
        }
      } else {
        wr2(ring + (slot0 + M) * WB, g);
        if constexpr (M > 0) {
          if (slot0 >= R - M) wr2(ring + (slot0 - (R - M)) * WB, g);
        }
      }
      if constexpr (!kGlds) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          pT[v] = qT[v];
          pC[v] = qC[v];
        }
        load_row<V>(qT, rowp(T, i + 3));
        load_row<V>(qC, rowp(iCp, i + 2));
      }
    } else {
      rd2(&hand[par ^ 1][stage - 1][0], w[0][Pr]);
      if constexpr (kRegG) {
        if constexpr (!LAST) wr2(gh(par, stage), gr[H - 1]);
        gshift();
        rd2(gh(par ^ 1, stage - 1), gr[0]);
      }
    }
    int sbase = slot0 - (S0 ? 0 : lag);
    sbase = sbase < 0 ? sbase + R : sbase;
    const double* rbase = ring + (sbase + M) * WB;
    // NW (no mirrors, delayed ring): the stage's NL slots do not wrap this
    // iteration, so every level's row is one base + an immediate offset
    const double* rlow = ring + (sbase - (NL - 1)) * WB;
    auto levels = [&](auto NWc) {
    constexpr bool NW = decltype(NWc)::value;
    auto ring_row = [&](int j) {  // factor row of local level j (slot sbase - (j-1))
      if constexpr (NW) {
        return rlow + (NL - j) * WB;
      } else if constexpr (M > 0) {
        return rbase - (j - 1) * WB;  // j - 1 <= H - 1 = M: inside the mirrors
      } else {
        const int sl = sbase - (j - 1) < 0 ? sbase - (j - 1) + R : sbase - (j - 1);
        return (const double*)(ring + sl * WB);
      }
    };
    // factors read one level ahead (LDS latency under the previous level's
    // arithmetic); stage 0's level-1 factors are still in registers (with the
    // delayed ring also its level-2 factors: row i-1, gp)
    auto fetch = [&](int j, double (&out)[V]) {
      if (S0 && kDelay && j == 2) {
#pragma unroll
        for (int v = 0; v < V; ++v) out[v] = gp[v];
      } else {
        rd2(ring_row(j), out);
      }
    };
    double gn[V];
    if constexpr (kRegG) {
    } else if constexpr (S0) {
#pragma unroll
      for (int v = 0; v < V; ++v) gn[v] = g[v];
    } else {
      rd2(ring_row(1), gn);
    }
    constexpr bool kSP = Ar == kArFast5RegSP || Ar == kArFast5RegSP2;
    double tq[kSP ? V : 1];  // software pipelining: the next level's fma(mkc, c, L+R)
#pragma unroll
    for (int j = 1; j <= NL; ++j) {
      const int row = i - (S0 ? 0 : lag) - (j - 1);
      double gl[V];
      if constexpr (kRegG) {
#pragma unroll
        for (int v = 0; v < V; ++v) gl[v] = gr[j - 1][v];
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) gl[v] = gn[v];
        if (j < NL && Ar != kArDiagOneRow) fetch(j + 1, gn);
      }
      const double(&c)[V] = w[j - 1][PC];
      const double(&dn)[V] = w[j - 1][Pr];
      double res[V];
      uint64_t saved_exec = 0;
      if constexpr (!Canon) {
        const double(&up)[V] = w[j - 1][PU];
        const double rn = from_next_lane<kDpp>(c[0]);
        const double ln = from_prev_lane<kDpp>(c[V - 1]);
        if constexpr (kMask) {
          // the level's arithmetic in ONE asm statement under the cone's lane
          // mask (the compiler can place nothing of its own under the narrowed
          // EXEC); the lane moves above ran under the full EXEC (a neighbour
          // may skip the level). Same operations and order as below, per cell:
          // sx = L + R; t = fma(mkc, c, sx); t = fma(ry, U + D, t);
          // res = fma(g, t, c). Inactive lanes keep stale registers that no
          // valid output reads. s_nop 1: VALU write -> DPP read wait states.
          // In place where the input dies here: L + R of cell 0 / 3 into the lane
          // moves' registers, U + D into the oldest row `up` (dead after this level).
          double(&um)[V] = w[j - 1][PU];
          res[0] = ln;
          res[3] = rn;
          asm volatile(
              "s_and_saveexec_b64 %[sv], %[m]\n\t"
              "v_add_f64 %[r0], %[c1], %[r0]\n\t"
              "v_add_f64 %[r1], %[c2], %[c0]\n\t"
              "v_add_f64 %[r2], %[c3], %[c1]\n\t"
              "v_add_f64 %[r3], %[r3], %[c2]\n\t"
              "v_add_f64 %[u0], %[u0], %[d0]\n\t"
              "v_add_f64 %[u1], %[u1], %[d1]\n\t"
              "v_add_f64 %[u2], %[u2], %[d2]\n\t"
              "v_add_f64 %[u3], %[u3], %[d3]\n\t"
              "v_fma_f64 %[r0], %[mk], %[c0], %[r0]\n\t"
              "v_fma_f64 %[r1], %[mk], %[c1], %[r1]\n\t"
              "v_fma_f64 %[r2], %[mk], %[c2], %[r2]\n\t"
              "v_fma_f64 %[r3], %[mk], %[c3], %[r3]\n\t"
              "v_fma_f64 %[r0], %[ry], %[u0], %[r0]\n\t"
              "v_fma_f64 %[r1], %[ry], %[u1], %[r1]\n\t"
              "v_fma_f64 %[r2], %[ry], %[u2], %[r2]\n\t"
              "v_fma_f64 %[r3], %[ry], %[u3], %[r3]\n\t"
              "v_fma_f64 %[r0], %[g0], %[r0], %[c0]\n\t"
              "v_fma_f64 %[r1], %[g1], %[r1], %[c1]\n\t"
              "v_fma_f64 %[r2], %[g2], %[r2], %[c2]\n\t"
              "v_fma_f64 %[r3], %[g3], %[r3], %[c3]\n\t"
              "s_or_b64 exec, exec, %[sv]\n\t"
              "s_nop 1"
              : [r0] "+v"(res[0]), [r1] "=&v"(res[1]), [r2] "=&v"(res[2]), [r3] "+v"(res[3]),
                [u0] "+v"(um[0]), [u1] "+v"(um[1]), [u2] "+v"(um[2]), [u3] "+v"(um[3]),
                [sv] "=&s"(saved_exec)
              : [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]),
                [d0] "v"(dn[0]), [d1] "v"(dn[1]), [d2] "v"(dn[2]), [d3] "v"(dn[3]),
                [g0] "v"(gl[0]), [g1] "v"(gl[1]), [g2] "v"(gl[2]), [g3] "v"(gl[3]),
                [ry] "v"(ry), [mk] "v"(mkc), [m] "s"(amask[j - 1])
              : "scc");
        } else if constexpr (kSP) {
          auto partial = [&](const double(&cc)[V], double r_n, double l_n, double(&out)[V]) {
#pragma unroll
            for (int v = 0; v < V; ++v) {
              const double rv = v + 1 < V ? cc[v + 1] : r_n;
              const double lv = v > 0 ? cc[v - 1] : l_n;
              out[v] = __builtin_fma(mkc, cc[v], rv + lv);
            }
          };
          if (j == 1) partial(c, rn, ln, tq);
          double t[V];
#pragma unroll
          for (int v = 0; v < V; ++v) t[v] = tq[v];
          if (j < NL) {  // the next level's centre row: the previous row iteration's
            const double(&cn)[V] = w[j][PC];
            partial(cn, from_next_lane<kDpp>(cn[0]), from_prev_lane<kDpp>(cn[V - 1]), tq);
          }
#pragma unroll
          for (int v = 0; v < V; ++v) {
            t[v] = __builtin_fma(ry, up[v] + dn[v], t[v]);
            res[v] = __builtin_fma(gl[v], t[v], c[v]);
          }
          if constexpr (Ar == kArFast5RegSP) __builtin_amdgcn_sched_barrier(0);
        } else {
        double sx[V], sy[V], t[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const double rv = v + 1 < V ? c[v + 1] : rn;
          const double lv = v > 0 ? c[v - 1] : ln;
          sx[v] = rv + lv;
          sy[v] = up[v] + dn[v];
        }
        // the V cells' FMA chains interleaved (sched_barrier keeps them apart)
        if constexpr (Ar != kArFast5RegNoSB) __builtin_amdgcn_sched_barrier(0);
        if constexpr (ar_split(Ar)) {
          double u[V];
          if constexpr (Ar == kArFast6Reg) {
#pragma unroll
            for (int v = 0; v < V; ++v) {
              u[v] = __builtin_fma(-2.0, c[v], sx[v]);
              t[v] = __builtin_fma(-2.0, c[v], sy[v]);
            }
          } else {
#pragma unroll
            for (int v = 0; v < V; ++v) {
              const double d = c[v] + c[v];
              u[v] = sx[v] - d;
              t[v] = sy[v] - d;
            }
          }
          if constexpr (Ar != kArFast5RegNoSB) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int v = 0; v < V; ++v) t[v] = __builtin_fma(ry, t[v], u[v]);
        } else {
#pragma unroll
          for (int v = 0; v < V; ++v) t[v] = __builtin_fma(mkc, c[v], sx[v]);
          if constexpr (Ar != kArFast5RegNoSB) __builtin_amdgcn_sched_barrier(0);
          if constexpr (Ar == kArFast5RegIso) {
#pragma unroll
            for (int v = 0; v < V; ++v) t[v] = sy[v] + t[v];
          } else {
#pragma unroll
            for (int v = 0; v < V; ++v) t[v] = __builtin_fma(ry, sy[v], t[v]);
          }
        }
        if constexpr (Ar != kArFast5RegNoSB) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int v = 0; v < V; ++v) res[v] = __builtin_fma(gl[v], t[v], c[v]);
        }  // !kMask
      } else {
        // canonical: same expressions and rounding as rma/common.h
        const double rn = from_next_lane(c[0]);
        double qr[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const double rv = v + 1 < V ? c[v + 1] : rn;
          qr[v] = (k.mlam * (rv - c[v])) * k.rdx;  // qxR of cell v == qxL of cell v+1
        }
        const double ql0 = from_prev_lane(qr[V - 1]);
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const double qU = (k.mlam * (dn[v] - c[v])) * k.rdy;
          const double qD = fy[j - 1][v];  // qyU of the previous row
          fy[j - 1][v] = qU;
          const double qL = v == 0 ? ql0 : qr[v - 1];
          res[v] = c[v] + k.dt * (gl[v] * ((-(qr[v] - qL)) * k.rdx - (qU - qD) * k.rdy));
        }
      }
      (void)saved_exec;
      if (j < NL) {
        const int jj = j < NL ? j : NL - 1;
#pragma unroll
        for (int v = 0; v < V; ++v) w[jj][Pr][v] = res[v];
      } else if constexpr (!LAST) {
        wr2(&hand[par][S0 ? 0 : stage][0], res);
      } else if (row >= ya32 && row < yb32) {
        store_row<V, true>(const_cast<double*>(at(T2 + (int64_t)row * nx, xsob)), res, m);
        // direct-store halos: the same values into the neighbours' halos;
        // only tasks whose window or rows touch a halo image range (dtask,
        // uniform) test the row
        if constexpr (Dir) {
          if (dtask)
            direct_row<V>(DS, row, nx, (int)xso, (int64_t)row * nx + x, res, m, dxm, dxp);
        }
      }
    }
    };
    if constexpr (M == 0 && kDelay) {
      if (sbase >= NL - 1)
        levels(std::true_type{});
      else
        levels(std::false_type{});
    } else {
      levels(std::false_type{});
    }
    if constexpr (S0 && kDelay) {
#pragma unroll
      for (int v = 0; v < V; ++v) gp[v] = g[v];
    }
    slot0 = slot0 + 1 == R ? 0 : slot0 + 1;
    par ^= 1;
    if constexpr (kGlds) {  // no vmcnt(0): the staging DMA stays in flight across rows
      if constexpr (S0) {
        // the staging reads above are complete (lgkmcnt(0)) before the DMA of
        // T row i+1+NST / 1/Cp row i+NST overwrites the same slots
        __builtin_amdgcn_s_waitcnt(0xC07F);
        asm volatile("" ::: "memory");
        glds_row(0, i + 1 + NST, Ps);
        glds_row(1, i + NST, Ps);
      }
      if (Ar != kArDiagHalfBarrier || (Ps & 1))
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      __syncthreads();  // hand-off and ring rows visible; this iteration's reads done
    }
  };
  // one row loop per stage role (stage is wave-uniform; every copy passes the
  // same barriers): stage 0 carries the HBM prefetch registers, the others not
  // unrolled by 6 where the factor rows live 5 iterations (pipe_u6), else 3
  auto run = [&](auto S0c, auto LASTc) {
    for (;;) {
      iter(std::integral_constant<int, 0>{}, S0c, LASTc);
      if (++i > iend) break;
      iter(std::integral_constant<int, 1>{}, S0c, LASTc);
      if (++i > iend) break;
      iter(std::integral_constant<int, 2>{}, S0c, LASTc);
      if (++i > iend) break;
      if constexpr (kU6) {
        iter(std::integral_constant<int, 3>{}, S0c, LASTc);
        if (++i > iend) break;
        iter(std::integral_constant<int, 4>{}, S0c, LASTc);
        if (++i > iend) break;
        iter(std::integral_constant<int, 5>{}, S0c, LASTc);
        if (++i > iend) break;
      }
    }
  };
  if constexpr (S == 1) {
    run(std::true_type{}, std::true_type{});
  } else {
    if (stage == 0)
      run(std::true_type{}, std::false_type{});
    else if (stage == S - 1)
      run(std::false_type{}, std::true_type{});
    else if constexpr (S > 2)
      run(std::false_type{}, std::false_type{});
  }
  // the staging DMA issued past the last row must land before the block's LDS
  // is released to the next block on this CU
  if constexpr (kGlds) {
    if (stage == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (b < sig_first) signal_block_done(L.sig, L.sig_blocks);  // block-uniform
}

// Dir: the direct-store halo variant (DirectStores). A separate instantiation:
// the direct-store code costs the row loop registers and scheduling (~4 % per
// task measured when every task of a pass ran it, K = 20 then at one wave
// per SIMD), so the plain kernels carry none of it and the executor gives the
// Dir variant the frame launches only, which hold every image cell.
template <int K, int S, int V, int Ar, int C, bool Dir = false>
__global__ __launch_bounds__(kWave * S * C) __attribute__((amdgpu_waves_per_eu(
    kernel_waves<K, S, V, Ar, C>()))) void pipe_kernel(double* __restrict__ T2,
                                                      const double* __restrict__ T,
                                                      const double* __restrict__ iCp,
                                                      int64_t nx, int64_t ny, RectList L,
                                                      StencilCoef k, int chunk_rows,
                                                      int remap, DirectStores D) {
  pipe_body<K, S, V, Ar, C, Dir>(T2, T, iCp, nx, ny, L, k, chunk_rows, remap, D);
}

// direct-store variants exist for the production fast-math arithmetics
// (kArFast5 at every K, the register-factor kArFast5Reg) at one column wave
template <int V, int Ar, int C>
constexpr bool has_direct() {
  return C == 1 && V != 5 && (Ar == kArFast5 || Ar == kArFast5Reg || Ar == kArFast5RegNoSB);
}

struct PipeLaunch {
  double* T2;
  const double* T;
  const double* iCp;
  int64_t nx, ny;
  const Rect* rects;
  int nrects;
  StencilCoef k;
  int chunk_rows, remap;
  hipStream_t stream;
  uint64_t* sig = nullptr;  // fused pass: the first sig_rects rects signal (RectList::sig)
  int sig_rects = 0;
  int sig_chunk_rows = 0;   // ...with this many rows per task (0: chunk_rows)
  const DirectStores* direct = nullptr;  // direct-store halos (nullptr: none)
  int* occupancy = nullptr;  // non-null: launch nothing, store the blocks per CU of the
                             // plain kernel [0] and of its direct-store variant [1] (0: none)
};

// Plans the (strip, chunk) tasks with this instantiation's block width
// (Geo::WB, kStep), so host planning and kernel geometry cannot disagree.
template <int K, int S, int V, int Ar, int C = 1>
void launch(const PipeLaunch& a) {
  if (a.occupancy) {
    const int bs = kWave * S * C;
    a.occupancy[0] = a.occupancy[1] = 0;
    RMA_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &a.occupancy[0], pipe_kernel<K, S, V, Ar, C, false>, bs, 0));
    if constexpr (has_direct<V, Ar, C>())
      RMA_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &a.occupancy[1], pipe_kernel<K, S, V, Ar, C, true>, bs, 0));
    return;
  }
  int rows_buf[kMaxRects] = {};
  const int* rows = nullptr;
  if (a.sig_rects > 0 && a.sig_chunk_rows > 0) {  // lead rects with their own task rows
    for (int i = 0; i < a.sig_rects && i < kMaxRects; ++i) rows_buf[i] = a.sig_chunk_rows;
    rows = rows_buf;
  }
  RectList L;
  const int64_t blocks =
      plan_strip_tasks(L, a.rects, a.nrects, V, a.chunk_rows, K, Geo<K, S, V, C>::WB, rows);
  static_assert(Geo<K, S, V, C>::kStep == (Geo<K, S, V, C>::WB - 2 * K) / V * V, "strip step");
  if (L.n == 0) return;
  RMA_CHECK_ARG(blocks < (int64_t(1) << 31), "grid too large: " << blocks << " blocks");
  if (a.sig) {  // the signal rects' blocks (empty rects are not planned)
    int ns = 0;
    for (int i = 0; i < a.sig_rects; ++i) ns += a.rects[i].empty() ? 0 : 1;
    RMA_CHECK_ARG(ns > 0, "signalling launch without a non-empty signal rect");
    L.sig = a.sig;
    L.sig_blocks = L.block_end[ns - 1];
  }
  const dim3 grid((unsigned)blocks), block(kWave * S * C);
  if (a.direct && a.direct->on) {
    if constexpr (has_direct<V, Ar, C>()) {
      pipe_kernel<K, S, V, Ar, C, true><<<grid, block, 0, a.stream>>>(
          a.T2, a.T, a.iCp, a.nx, a.ny, L, a.k, a.chunk_rows, a.remap, *a.direct);
    } else {
      RMA_CHECK_ARG(false, "no direct-store variant of the pipelined kernel K=" << K << " S=" << S
                                << " V=" << V << " arithmetic " << Ar << " columns " << C);
    }
    return;
  }
  pipe_kernel<K, S, V, Ar, C><<<grid, block, 0, a.stream>>>(a.T2, a.T, a.iCp, a.nx, a.ny, L, a.k,
                                                           a.chunk_rows, a.remap, DirectStores{});
}

// Each stencil_pipe_{a,b,c}.hip unit instantiates a range of (K, S) of the
// default stage split and answers for it: returns false if it does not hold
// (K, S, V, arithmetic). Alternative splits, the ds_bpermute variant and the
// two-column blocks are in the lab library (csrc/lab/stencil_pipe_lab.hip).
bool dispatch_a(int K, int S, int V, int ar, const PipeLaunch& a);
bool dispatch_b(int K, int S, int V, int ar, const PipeLaunch& a);
bool dispatch_c(int K, int S, int V, int ar, const PipeLaunch& a);
// register-resident factors (stencil_pipe_r.hip): fast5, S = 4, K = 10..24
bool dispatch_r(int K, int S, int V, int ar, const PipeLaunch& a);
// ... K = 20 of it, compiled with another machine scheduler (stencil_pipe_r20.hip)
bool dispatch_r20(int K, int S, int V, int ar, const PipeLaunch& a);
// the executor's K = 24 kernel: piper without in-level sched_barriers, the
// same scheduler (stencil_pipe_r24.hip)
bool dispatch_r24(int K, int S, int V, int ar, const PipeLaunch& a);

}  // namespace pipe
}  // namespace rma

// (K, S, arithmetic) -> launch<K, S, V, Ar> for V in {1, 2, 4}
#define RMA_PIPE_CASE(KK, SS, CC)                                  \
  if (K == KK && S == SS && ar == CC) {                            \
    if (V == 4) launch<KK, SS, 4, CC>(a);                          \
    else if (V == 2) launch<KK, SS, 2, CC>(a);                     \
    else launch<KK, SS, 1, CC>(a);                                 \
    return true;                                                   \
  }
