// librma_lab.so, K-step unit: the superseded and experimental members of the
// overlapped-strip family (moved out of the core library in round 3):
//   0 / 1 / 2  canonical arithmetic with the 1/Cp window in registers or an
//              LDS ring, lane moves by ds_bpermute or DPP (3, the bitwise
//              default, stays in the core);
//   4 "fast"   reassociated fluxes, 7 fp64 ops per cell update;
//   5 "fast5"  5-point sum with one folded per-cell factor, 5 ops: the GPU
//              oracle of the pipelined kernel (pipe == fast5 bitwise,
//              tests/test_temporal_gpu.py);
//   6/7/8      "fast5p2/p4/p8": fast5 with the levels of one strip over 2/4/8
//              pipelined waves (fixed K), generalised by stencil_pipe.h.
// Measurements: profiles/SUMMARY_r1.md, profiles/pmc_pipe_r2.md.
#include "../kernels/stencil_kstep.h"

#include "../kernels/lab_hooks.h"

namespace rma {
namespace lab {
using namespace kstep;

// kernel=5 ("fast5"): the 5-point sum form with every constant folded into one
// per-cell coefficient, 5 fp64 operations per cell update (kFast: 7):
//   T2 = fma(g, fma(r, U + D, fma(-kc, c, R + L)), c)
//   g = dt*(lam/dx^2)/Cp (LDS ring, ZERO outside the interior), r = dy^-2/dx^-2,
//   kc = 2*(1 + r).
// No face fluxes are carried: a level keeps three rows (up, centre, down) in a
// 3-slot rotation (loop unrolled by three), the same register count as two
// rows + one flux row. Both lane moves read the centre row only, so they issue
// at the start of a level instead of in the middle of its dependency chain.
template <int K, int V, bool NT>
__device__ __forceinline__ void stencilk5_body(
    double* __restrict__ T2, const double* __restrict__ T, const double* __restrict__ iCp,
    int64_t nx, int64_t ny, const RectList& L, const StencilCoef& k, int chunk_rows, int remap) {
  constexpr int W = kWave * V;
  constexpr int kStep = (W - 2 * K) / V * V;  // output columns per strip (plan_rects)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = remap ? xcd_remap(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  int ri = 0;
  while (ri < L.n - 1 && b >= L.block_end[ri]) ++ri;
  int64_t strip, chunk;
  if (!locate_task(L, ri, b, wave, strip, chunk)) return;  // whole wave exits
  const Rect r = L.r[ri];
  const int64_t xs = L.xa[ri] + strip * kStep;
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

  const double ax = (-k.mlam) * k.rdx * k.rdx;  // lam/dx^2
  const double ay = (-k.mlam) * k.rdy * k.rdy;
  const double ry = ay / ax;                    // host guarantees ax != 0, ry finite
  const double mkc = -2.0 * (1.0 + ry);
  const double gs = k.dt * ax;

  // w[j][s]: level-j rows; at iteration t the new row goes to slot t%3, the
  // centre row is slot (t+2)%3 and the upper row slot (t+1)%3.
  // prefetch two rows ahead: (pT, pC) are consumed this iteration, (qT, qC)
  // arrive for the next one. With one row of prefetch the wait at the top of
  // an iteration also covered the previous iteration's (conditional) store:
  // its vmcnt count differs between paths, so the compiler waited for all.
  double w[K][3][V], pT[V], pC[V], qT[V], qC[V];
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int v = 0; v < V; ++v) w[j][s][v] = 0.0;
  int64_t i = ya - K;
  const int64_t iend = yb + K - 2;
  auto rowc = [&](int64_t y) { return min(max(y, (int64_t)0), ny - 1); };
  load_row<V>(w[0][2], T + rowc(i) * nx + xl);
  load_row<V>(pT, T + rowc(i + 1) * nx + xl);
  load_row<V>(pC, iCp + rowc(i) * nx + xl);
  load_row<V>(qT, T + rowc(i + 2) * nx + xl);
  load_row<V>(qC, iCp + rowc(i + 1) * nx + xl);

  __shared__ double ring[kWavesPerBlock * K * W];
  double* myring = ring + wave * K * W + lane * V;
  int slot = 0;
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int v = 0; v < V; ++v) myring[j * W + v] = 0.0;

  auto iter = [&](auto Pc) {
    constexpr int P = decltype(Pc)::value;       // new row
    constexpr int PC = (P + 2) % 3, PU = (P + 1) % 3;  // centre, up
    const bool rin1 = i >= 1 && i <= ny - 2;
#pragma unroll
    for (int v = 0; v < V; ++v) w[0][P][v] = pT[v];
    {
      double g[V];
#pragma unroll
      for (int v = 0; v < V; ++v) g[v] = (rin1 && cin[v]) ? gs * pC[v] : 0.0;
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
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
      pT[v] = qT[v];
      pC[v] = qC[v];
    }
    load_row<V>(qT, T + rowc(i + 3) * nx + xl);
    load_row<V>(qC, iCp + rowc(i + 2) * nx + xl);
#pragma unroll
    for (int j = 1; j <= K; ++j) {
      const int64_t row = i - (j - 1);
      double gl[V];
      {
        const int sl = slot - (j - 1) < 0 ? slot - (j - 1) + K : slot - (j - 1);
        const double* src = myring + sl * W;
        if constexpr (V == 1) {
          gl[0] = src[0];
        } else {
#pragma unroll
          for (int h = 0; h < V / 2; ++h) {
            const dbl2 t2 = reinterpret_cast<const dbl2*>(src)[h];
            gl[2 * h] = t2.x;
            gl[2 * h + 1] = t2.y;
          }
        }
      }
      const double(&up)[V] = w[j - 1][PU];
      const double(&c)[V] = w[j - 1][PC];
      const double(&dn)[V] = w[j - 1][P];
      const double rn = from_next_lane<true>(c[0]);      // lane 63: 0 (invalid column)
      const double ln = from_prev_lane<true>(c[V - 1]);  // lane 0: 0 (invalid column)
      double res[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const double rv = v + 1 < V ? c[v + 1] : rn;
        const double lv = v > 0 ? c[v - 1] : ln;
        const double sx = rv + lv;
        const double sy = up[v] + dn[v];
        res[v] = __builtin_fma(gl[v], __builtin_fma(ry, sy, __builtin_fma(mkc, c[v], sx)), c[v]);
      }
      if (j < K) {
        const int jj = j < K ? j : K - 1;
#pragma unroll
        for (int v = 0; v < V; ++v) w[jj][P][v] = res[v];
      } else if (row >= ya && row < yb) {
        store_row<V, NT>(T2 + row * nx + x, res, m);
      }
    }
    slot = slot + 1 == K ? 0 : slot + 1;
  };
  for (;;) {
    iter(std::integral_constant<int, 0>{});
    if (++i > iend) break;
    iter(std::integral_constant<int, 1>{});
    if (++i > iend) break;
    iter(std::integral_constant<int, 2>{});
    if (++i > iend) break;
  }
}

template <int K, int V, bool NT>
__global__ __launch_bounds__(kBlock) void stencilk5_kernel(
    double* __restrict__ T2, const double* __restrict__ T, const double* __restrict__ iCp,
    int64_t nx, int64_t ny, RectList L, StencilCoef k, int chunk_rows, int remap) {
  stencilk5_body<K, V, NT>(T2, T, iCp, nx, ny, L, k, chunk_rows, remap);
}

// kernel=6/7/8 ("fast5p2" / "fast5p4" / "fast5p8"): kernel 5's arithmetic with
// the K levels of ONE strip split over the S waves of a block (S = 2 / 4 / 8
// stages of H = K/S; fixed K in {8, 12, 16}, fast5p8 K in {8, 16}; the any-K
// generalisation is stencil_pipe.h, kernels 9/10)
// levels each). Stage s keeps only its own H three-row windows (K=16, S=4:
// 48 instead of 192 VGPRs of windows, so 5 waves per SIMD instead of 2 hide
// the fp64 and LDS latencies). Stage 0 streams T / 1/Cp from HBM and fills
// the per-strip 1/Cp ring; every other stage reads its input level from an
// LDS hand-off row written by the previous stage one iteration earlier; the
// last stage stores. One barrier per row iteration; stage s runs s(H+1) rows
// behind stage 0 (its new input row at iteration i is i + 1 - s(H+1)).
// Bitwise equal to kernel 5 (same operations per cell).
template <int K, int S, int V, bool NT>
__device__ __forceinline__ void stencilk5p_body(
    double* __restrict__ T2, const double* __restrict__ T, const double* __restrict__ iCp,
    int64_t nx, int64_t ny, const RectList& L, const StencilCoef& k, int chunk_rows, int remap) {
  static_assert(K % S == 0, "levels must split evenly over the stages");
  constexpr int H = K / S;
  constexpr int W = kWave * V;
  constexpr int kStep = (W - 2 * K) / V * V;
  constexpr int R = K + S - 1;  // ring rows: i (newest) .. i + 2 - K - S (oldest read)
  const int stage = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = remap ? xcd_remap(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  int ri = 0;
  while (ri < L.n - 1 && b >= L.block_end[ri]) ++ri;
  // one block = one strip task; every block is a task (the stages meet at barriers)
  const int64_t lb = b - (ri ? L.block_end[ri - 1] : 0);
  const int64_t strip = lb % L.strips[ri], chunk = lb / L.strips[ri];
  const Rect r = L.r[ri];
  const int64_t xs = L.xa[ri] + strip * kStep;
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
  // every cell of the strip inside the x range 1..nx-2 (so every cin is true)
  const bool xin = xs >= 1 && xs + W - 1 <= nx - 2;

  const double ax = (-k.mlam) * k.rdx * k.rdx;
  const double ay = (-k.mlam) * k.rdy * k.rdy;
  const double ry = ay / ax;
  const double mkc = -2.0 * (1.0 + ry);
  const double gs = k.dt * ax;

  // w[0]: the stage's input level (T for stage 0, level s*H otherwise),
  // w[j]: local level s*H + j, j < H; the level-(s+1)*H row is handed off
  double w[H][3][V], pT[V], pC[V], qT[V], qC[V];
#pragma unroll
  for (int j = 0; j < H; ++j)
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int v = 0; v < V; ++v) w[j][t][v] = 0.0;
  // row bookkeeping in 32 bits (the host checks ny < 2^31): gfx950 has no
  // 64-bit scalar compares, so int64 row tests became VALU v_cmp_*_i64 +
  // v_mov_b64 copies on every row iteration
  const int ny32 = (int)ny, ya32 = (int)ya, yb32 = (int)yb;
  int i = ya32 - K;
  const int iend = yb32 + K - 3 + S;
  auto rowc = [&](int y) { return (int64_t)min(max(y, 0), ny32 - 1); };
  if (stage == 0) {
    load_row<V>(w[0][2], T + rowc(i) * nx + xl);
    load_row<V>(pT, T + rowc(i + 1) * nx + xl);
    load_row<V>(pC, iCp + rowc(i) * nx + xl);
    load_row<V>(qT, T + rowc(i + 2) * nx + xl);
    load_row<V>(qC, iCp + rowc(i + 1) * nx + xl);
  }
  __shared__ double ring[R * W];
  __shared__ double hand[2][S > 1 ? S - 1 : 1][W];
  for (int t = threadIdx.x; t < R * W; t += S * kWave) ring[t] = 0.0;
  for (int t = threadIdx.x; t < 2 * (S > 1 ? S - 1 : 1) * W; t += S * kWave) (&hand[0][0][0])[t] = 0.0;
  __syncthreads();
  // LDS rows (ring and hand-off) are lane-interleaved: cell pair h of lane l
  // sits at dbl2 index h * 64 + l, so each ds_read/write_b128 covers 1 KiB
  // contiguously. The lane-major layout (lane l at l * V) strode 32 B per lane
  // at V = 4, a 2-way bank conflict on every access (SQ_LDS_BANK_CONFLICT =
  // half of SQ_LDS_IDX_ACTIVE, profiles/pmc_fast5_r1.md).
  auto rd2 = [&](const double* row, double (&out)[V]) {
    if constexpr (V == 1) {
      out[0] = row[lane];
    } else {
#pragma unroll
      for (int h = 0; h < V / 2; ++h) {
        const dbl2 t2 = reinterpret_cast<const dbl2*>(row)[h * kWave + lane];
        out[2 * h] = t2.x;
        out[2 * h + 1] = t2.y;
      }
    }
  };
  auto wr2 = [&](double* row, const double (&in)[V]) {
    if constexpr (V == 1) {
      row[lane] = in[0];
    } else {
#pragma unroll
      for (int h = 0; h < V / 2; ++h) {
        dbl2 t2;
        t2.x = in[2 * h];
        t2.y = in[2 * h + 1];
        reinterpret_cast<dbl2*>(row)[h * kWave + lane] = t2;
      }
    }
  };
  int slot0 = 0;  // ring slot of row i (stage 0's level-1 row)
  int par = 0;
  const int lag = stage * (H + 1);  // rows behind stage 0
  auto iter = [&](auto Pc, auto S0c) {
    constexpr int P = decltype(Pc)::value;
    constexpr bool S0 = decltype(S0c)::value;
    constexpr int PC = (P + 2) % 3, PU = (P + 1) % 3;
    double g[V];  // stage 0: the new ring row (its level-1 factors)
    if constexpr (S0) {
      const bool rin1 = i >= 1 && i <= ny32 - 2;
#pragma unroll
      for (int v = 0; v < V; ++v) w[0][P][v] = pT[v];
      // rin1 and xin are wave-uniform: strips away from the x edges take a
      // branch without the per-cell selects (2 v_cndmask_b32 per cell)
      if (rin1 && xin) {
#pragma unroll
        for (int v = 0; v < V; ++v) g[v] = gs * pC[v];
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) g[v] = (rin1 && cin[v]) ? gs * pC[v] : 0.0;
      }
      wr2(ring + slot0 * W, g);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        pT[v] = qT[v];
        pC[v] = qC[v];
      }
      load_row<V>(qT, T + rowc(i + 3) * nx + xl);
      load_row<V>(qC, iCp + rowc(i + 2) * nx + xl);
    } else {
      rd2(&hand[par ^ 1][stage - 1][0], w[0][P]);
    }
    // this stage's level-1 row is i - lag: its ring slot
    int sbase = slot0 - (S0 ? 0 : lag);
    sbase = sbase < 0 ? sbase + R : sbase;
    auto ring_row = [&](int j) {  // ring row of local level j
      const int sl = sbase - (j - 1) < 0 ? sbase - (j - 1) + R : sbase - (j - 1);
      return ring + sl * W;
    };
    // level factors read one level ahead, so the LDS latency of level j + 1's
    // read hides under level j's arithmetic; stage 0's level-1 factors are the
    // row it just wrote (still in registers)
    double gn[V];
    if constexpr (S0) {
#pragma unroll
      for (int v = 0; v < V; ++v) gn[v] = g[v];
    } else {
      rd2(ring_row(1), gn);
    }
#pragma unroll
    for (int j = 1; j <= H; ++j) {
      const int row = i - (S0 ? 0 : lag) - (j - 1);
      double gl[V];
#pragma unroll
      for (int v = 0; v < V; ++v) gl[v] = gn[v];
      if (j < H) rd2(ring_row(j + 1), gn);
      const double(&up)[V] = w[j - 1][PU];
      const double(&c)[V] = w[j - 1][PC];
      const double(&dn)[V] = w[j - 1][P];
      const double rn = from_next_lane<true>(c[0]);
      const double ln = from_prev_lane<true>(c[V - 1]);
      // the V cells' operation chains issued interleaved (sched_barrier keeps
      // the compiler from serialising each cell's dependent FMA chain):
      // 64.6 -> 64.2 ms per K=16 pass at 101376^2, same operations, bitwise
      double res[V], sx[V], sy[V], t[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const double rv = v + 1 < V ? c[v + 1] : rn;
        const double lv = v > 0 ? c[v - 1] : ln;
        sx[v] = rv + lv;
        sy[v] = up[v] + dn[v];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int v = 0; v < V; ++v) t[v] = __builtin_fma(mkc, c[v], sx[v]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int v = 0; v < V; ++v) t[v] = __builtin_fma(ry, sy[v], t[v]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int v = 0; v < V; ++v) res[v] = __builtin_fma(gl[v], t[v], c[v]);
      if (j < H) {
        const int jj = j < H ? j : H - 1;
#pragma unroll
        for (int v = 0; v < V; ++v) w[jj][P][v] = res[v];
      } else if (S0 ? S > 1 : stage < S - 1) {
        wr2(&hand[par][S0 ? 0 : stage][0], res);
      } else if (row >= ya32 && row < yb32) {
        store_row<V, NT>(T2 + (int64_t)row * nx + x, res, m);
      }
    }
    slot0 = slot0 + 1 == R ? 0 : slot0 + 1;
    par ^= 1;
    __syncthreads();  // hand-off rows and ring row visible; this iteration's reads done
  };
  // stage 0 and the other stages run separate copies of the row loop (the
  // stage is wave-uniform; both copies pass the same barriers). In one shared
  // loop the merge after the stage branch made every stage carry stage 0's
  // prefetch registers: 16 v_mov_b64 per row iteration on stages 1..S-1
  // (1 per cell update, ~11 % of their VALU instructions)
  auto run = [&](auto S0c) {
    for (;;) {
      iter(std::integral_constant<int, 0>{}, S0c);
      if (++i > iend) break;
      iter(std::integral_constant<int, 1>{}, S0c);
      if (++i > iend) break;
      iter(std::integral_constant<int, 2>{}, S0c);
      if (++i > iend) break;
    }
  };
  if (stage == 0)
    run(std::true_type{});
  else
    run(std::false_type{});
}

// Waves per SIMD: S=4 -> 3 (below), S=8 -> 4 (512-thread blocks, 75.8 KB LDS
// at V=4: 2 blocks per CU, VGPR budget 128), S=2 -> no cap.
// 3 waves per SIMD: the 51.2 KB LDS of a K=16, S=4 block allows 3 blocks per
// CU, so the VGPR budget is 168 (512 / 3, 8-register granules)
template <int K, int S, int V, bool NT>
__global__ __launch_bounds__(kWave * S) __attribute__((amdgpu_waves_per_eu(S == 8 ? 4 : S == 4 ? 3 : 1))) void stencilk5p_kernel(
    double* __restrict__ T2, const double* __restrict__ T, const double* __restrict__ iCp,
    int64_t nx, int64_t ny, RectList L, StencilCoef k, int chunk_rows, int remap) {
  stencilk5p_body<K, S, V, NT>(T2, T, iCp, nx, ny, L, k, chunk_rows, remap);
}

bool kstep(int K, double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
           const Rect* rects, int nrects, const StencilCoef& c, const StencilTuning& tune,
           stream_t stream) {
  if (tune.kernel == 3 || tune.kernel < 0 || tune.kernel > 8) return false;
  const kstep::KstepLaunch kl = kstep::check_launch(K, T2, T, iCp, nx, ny, rects, nrects, c, tune);
  const int V = kl.V, remap = kl.remap;
  RectList L;
  if (tune.kernel >= 6) {  // stage-pipelined fast5: 2, 4 or 8 waves per strip
    const int S = tune.kernel == 6 ? 2 : tune.kernel == 7 ? 4 : 8;
    RMA_CHECK_ARG(ny < (int64_t(1) << 30), "the stage-pipelined kernels index rows in 32 bits, ny = " << ny);
    RMA_CHECK_ARG(K == 8 || K == 16 || (K == 12 && S < 8),
                  "the stage-pipelined kernels run 8, 12 or 16 steps per pass, got " << K);
    const int64_t ntask = plan_strip_tasks(L, rects, nrects, V, tune.chunk_rows, K);
    if (L.n == 0) return true;
    RMA_CHECK_ARG(ntask < (int64_t(1) << 31), "grid too large: " << ntask << " blocks");
    const dim3 g((unsigned)ntask), blk(kWave * S);
    hipStream_t st = as_stream(stream);
    const bool nt1 = tune.nontemporal & 1;
#define RMA_TBKP(KK, SS)                                                                     \
  if (V == 4) {                                                                               \
    if (nt1) stencilk5p_kernel<KK, SS, 4, true><<<g, blk, 0, st>>>(T2, T, iCp, nx, ny, L, c,  \
                                                                    tune.chunk_rows, remap);  \
    else stencilk5p_kernel<KK, SS, 4, false><<<g, blk, 0, st>>>(T2, T, iCp, nx, ny, L, c,     \
                                                                 tune.chunk_rows, remap);     \
  } else if (V == 2) {                                                                        \
    if (nt1) stencilk5p_kernel<KK, SS, 2, true><<<g, blk, 0, st>>>(T2, T, iCp, nx, ny, L, c,  \
                                                                    tune.chunk_rows, remap);  \
    else stencilk5p_kernel<KK, SS, 2, false><<<g, blk, 0, st>>>(T2, T, iCp, nx, ny, L, c,     \
                                                                 tune.chunk_rows, remap);     \
  } else {                                                                                    \
    if (nt1) stencilk5p_kernel<KK, SS, 1, true><<<g, blk, 0, st>>>(T2, T, iCp, nx, ny, L, c,  \
                                                                    tune.chunk_rows, remap);  \
    else stencilk5p_kernel<KK, SS, 1, false><<<g, blk, 0, st>>>(T2, T, iCp, nx, ny, L, c,     \
                                                                 tune.chunk_rows, remap);     \
  }
    if (S == 2) {
      if (K == 8) { RMA_TBKP(8, 2) } else if (K == 12) { RMA_TBKP(12, 2) } else { RMA_TBKP(16, 2) }
    } else if (S == 4) {
      if (K == 8) { RMA_TBKP(8, 4) } else if (K == 12) { RMA_TBKP(12, 4) } else { RMA_TBKP(16, 4) }
    } else {
      if (K == 8) { RMA_TBKP(8, 8) } else { RMA_TBKP(16, 8) }
    }
#undef RMA_TBKP
    RMA_HIP_LAUNCH_CHECK();
    return true;
  }
  const int64_t total = plan_rects(L, rects, nrects, V, tune.chunk_rows, remap, false, K);
  if (L.n == 0) return true;
  RMA_CHECK_ARG(total < (int64_t(1) << 31), "grid too large: " << total << " blocks");
  const dim3 grid((unsigned)total), block(kBlock);
  hipStream_t s = as_stream(stream);
  const bool nts = tune.nontemporal & 1;
#define RMA_TBK(KK, VV, NTS)                                                                 \
  switch (tune.kernel) {                                                                       \
    case 1:                                                                                    \
      kstep::stencilk_ovl_kernel<KK, VV, NTS, true, false><<<grid, block, 0, s>>>(              \
          T2, T, iCp, nx, ny, L, c, tune.chunk_rows, remap);                                   \
      break;                                                                                   \
    case 2:                                                                                    \
      kstep::stencilk_ovl_kernel<KK, VV, NTS, false, true><<<grid, block, 0, s>>>(                     \
          T2, T, iCp, nx, ny, L, c, tune.chunk_rows, remap);                                   \
      break;                                                                                   \
    case 4:                                                                                    \
      kstep::stencilk_ovl_kernel<KK, VV, NTS, true, true, true><<<grid, block, 0, s>>>(                \
          T2, T, iCp, nx, ny, L, c, tune.chunk_rows, remap);                                   \
      break;                                                                                   \
    case 5:                                                                                    \
      stencilk5_kernel<KK, VV, NTS><<<grid, block, 0, s>>>(T2, T, iCp, nx, ny, L, c,           \
                                                            tune.chunk_rows, remap);          \
      break;                                                                                   \
    default:                                                                                   \
      kstep::stencilk_ovl_kernel<KK, VV, NTS, false, false><<<grid, block, 0, s>>>(                    \
          T2, T, iCp, nx, ny, L, c, tune.chunk_rows, remap);                                   \
  }
#define RMA_TBK_V(KK)                                   \
  if (V == 4) {                                         \
    if (nts) { RMA_TBK(KK, 4, true); } else { RMA_TBK(KK, 4, false); } \
  } else if (V == 2) {                                  \
    if (nts) { RMA_TBK(KK, 2, true); } else { RMA_TBK(KK, 2, false); } \
  } else {                                              \
    if (nts) { RMA_TBK(KK, 1, true); } else { RMA_TBK(KK, 1, false); } \
  }
  // 12 / 16 levels: fast5 only, V <= 2 (register budget)
#define RMA_TBK_DEEP(KK, VV, NTS)                                                           \
  stencilk5_kernel<KK, VV, NTS><<<grid, block, 0, s>>>(T2, T, iCp, nx, ny, L, c,              \
                                                       tune.chunk_rows, remap);
#define RMA_TBK_DEEP_V(KK)                                                                  \
  if (V == 2) {                                                                               \
    if (nts) { RMA_TBK_DEEP(KK, 2, true) } else { RMA_TBK_DEEP(KK, 2, false) }                \
  } else {                                                                                    \
    if (nts) { RMA_TBK_DEEP(KK, 1, true) } else { RMA_TBK_DEEP(KK, 1, false) }                \
  }
  switch (K) {
    case 2: RMA_TBK_V(2) break;
    case 3: RMA_TBK_V(3) break;
    case 4: RMA_TBK_V(4) break;
    case 6: RMA_TBK_V(6) break;
    case 8: RMA_TBK_V(8) break;
    case 12: RMA_TBK_DEEP_V(12) break;
    default: RMA_TBK_DEEP_V(16) break;
  }
#undef RMA_TBK_DEEP_V
#undef RMA_TBK_DEEP
#undef RMA_TBK_V
#undef RMA_TBK
  RMA_HIP_LAUNCH_CHECK();
  return true;
}

}  // namespace lab

namespace {
// installs the lab kernels in the core's dispatchers when this library is loaded
struct Register {
  Register() {
    LabHooks h;
    h.kstep = &lab::kstep;
    h.pipe = &lab::pipe;
    h.onestep = &lab::onestep;
    set_lab_hooks(h);
  }
} g_register;
}  // namespace

}  // namespace rma
