// rocm_mpi_amd native core — kernel launch API (host side).
//
// Every GPU entry point enqueues work on the given HIP stream (passed as an
// opaque pointer so this header stays HIP-free for the pybind11 layer) and
// returns immediately. The *_cpu twins are bit-identical host implementations
// used for CPU-only runs (the reference's "ap 256² single-rank CPU array path",
// BASELINE.json configs[0]) and as the numerics oracle in tests.
#pragma once

#include <cstddef>
#include <cstdint>

#include "rma/common.h"

namespace rma {

using stream_t = void*;  // hipStream_t

// ---------------------------------------------------------------------------
// Fused 5-point stencil (K4 of SURVEY.md §2.3; reference
// scripts/diffusion_2D_perf.jl:3-13). Updates every cell of every rect in ONE
// launch: T2[r] = f(T, iCp)[r]. The split boundary/interior steps of
// perf_hide (K5, scripts/diffusion_2D_perf_hide.jl:15-29) are the same launch
// with the frame rects / interior rect, so the arithmetic is shared bitwise.
// ---------------------------------------------------------------------------
constexpr int kMaxRects = 8;

// Direct-store halos (pipelined K-step kernels only): cells of the output rect
// that are a neighbour's halo are ALSO stored straight into the neighbour's
// output field -- its own tile in the same process (loopback ranks), a mapped
// peer tile (IPC) or this tile's own periodic images. Replaces the pack /
// send / receive / unpack of an exchange (DiffusionExecutor::set_direct).
// Direction d = 0..7 is (i, j) = (kDirI[d], kDirJ[d]) of executor.h. A stored
// cell (x, y) also goes to dst[d] when dst[d] is set, x lies in the i-range
// (i = -1: [xm0, xm1), +1: [xp0, xp1), 0: any) and y in the j-range (same with
// ym / yp), at element index (y * nx + x) - i * sx - j * syr * nx: every rank
// has the same nx x ny tile, the neighbour's origin sx = nx - olx columns /
// syr = ny - oly rows away. Eight fixed ranges rather than a list of rects:
// the kernel decides per task (which ranges its window and rows touch) and per
// row with a few scalar compares; a list walked per row costs a scalar load
// chain per entry and doubled the K = 24 pass at 8192^2. Passed by value (a
// kernel argument).
struct DirectStores {
  int on = 0;  // any dst set
  int32_t xm0 = 0, xm1 = 0, xp0 = 0, xp1 = 0;
  int32_t ym0 = 0, ym1 = 0, yp0 = 0, yp1 = 0;
  int64_t sx = 0, syr = 0;
  double* dst[8] = {};
};

struct StencilTuning {
  int chunk_rows = 4;      // rows marched by one wave-task
  int nontemporal = 3;     // bit 0: NT T2 stores; bit 1: NT 1/Cp loads; bit 2: NT T loads
  int kernel = 0;          // 0 = register march (default), 1 = LDS-tiled
  int unroll = 4;          // rows per march iteration whose loads are issued together
  int vec = 2;             // cells per lane (2: one 16-B access per row, 4: two)
  int xcd_remap = -1;      // 1: each XCD takes a contiguous 1/8 of the tasks; 0: chunk rows
                           // padded to 8-block multiples (same-XCD neighbours); -1: by size
  int stages = 0;          // pipelined K-step kernels 9/10: waves per strip (0: default)
  int cols = 0;            // pipelined kernels: column waves per stage (0: default, 1, 2)
  // Frame-first fused pass (pipelined kernels only): signal != nullptr makes
  // the first signal_rects rects' tasks dispatch first (never XCD-remapped)
  // and count their completion in signal[0] (device memory, zero); the last
  // one resets it and stores 1 into signal[1] with system-scope release. A
  // flag_wait_gpu(signal + 1, 1, ...) on another stream then orders work after
  // those rects without waiting for the rest of the launch.
  // Without signal, signal_rects > 0 only gives the first rects their own
  // rows per task (the direct-store one-launch pass: shorter edge tasks).
  uint64_t* signal = nullptr;
  int signal_rects = 0;
  int signal_chunk_rows = 0;  // rows per task of the signal rects (0: chunk_rows)
  // direct-store halos of this launch (pipelined kernels; nullptr: none)
  const DirectStores* direct = nullptr;
};

void stencil_rects_gpu(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                       const Rect* rects, int nrects, const StencilCoef& c,
                       const StencilTuning& tune, stream_t stream);
void stencil_rects_cpu(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                       const Rect* rects, int nrects, const StencilCoef& c);

// Two steps per pass (temporal blocking, stencil_tb.hip): T2[r] = f(f(T))[r],
// where the intermediate step is f(T) on the interior [1,nx-1)x[1,ny-1) and T
// elsewhere. Bitwise equal to two one-step launches. T2 != T; unroll 2 or 4;
// no column mode (every rect is marched in 64*V-cell strips).
void stencil2_rects_gpu(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                        const Rect* rects, int nrects, const StencilCoef& c,
                        const StencilTuning& tune, stream_t stream);
void stencil2_rects_cpu(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                        const Rect* rects, int nrects, const StencilCoef& c);

// K steps per pass (K = 2, 3, 4, 6, 8: stencil_kstep.hip kernel 3; others: csrc/lab): T2[r] = f^K(T)[r], the
// intermediate levels being f on the interior and T elsewhere; face fluxes
// shared between neighbouring cells (same rounding). Bitwise equal to K
// one-step launches.
void stencilk_rects_gpu(int K, double* T2, const double* T, const double* iCp, int64_t nx,
                        int64_t ny, const Rect* rects, int nrects, const StencilCoef& c,
                        const StencilTuning& tune, stream_t stream);
void stencilk_rects_cpu(int K, double* T2, const double* T, const double* iCp, int64_t nx,
                        int64_t ny, const Rect* rects, int nrects, const StencilCoef& c);
// StencilTuning::kernel of the K-step launcher: 0 march, 1 LDS 1/Cp ring, 2 DPP,
// 3 LDS ring + DPP (bitwise default), 4 fast (reassociated fluxes, 7 fp64 ops
// per cell update), 5 fast5 (5-point sum, constants folded into one per-cell
// factor, 5 ops). 4 and 5 are not bitwise equal to the canonical update.
// fast5_ok: kernel 5 divides by lam/dx^2, so it needs lam != 0.
bool fast5_ok(const StencilCoef& c);
//   9 pipe  (fast5 arithmetic) / 10 pipec (canonical) / 11 pipeb (fast5, lane
//     moves by ds_bpermute; K = 16, 20, 24 only): stage-pipelined strips
//     for ANY K in 1..kPipeMaxK (stencil_pipe.h); stencilk_rects_gpu routes
//     kernels 9/10 here. stages = waves per strip (0: pipe_default_stages).
//     pipe is bitwise equal to kernel 5 and to stencilk5_rects_cpu; pipec to K
//     one-step launches and stencilk_rects_cpu.
constexpr int kPipeMaxK = 24;
int pipe_default_stages(int K);
bool pipe_has(int K, int stages, int arith = 0);
// Column waves per stage: 2 = blocks of 2 x stages waves over ~500 columns
// (V = 4 only, fast5 K = 16/20/24, csrc/lab/stencil_pipe_lab.hip, an experiment: slower
// than 1); pipe_has_cols says whether (K, S, arith, cols) is instantiated,
// pipe_default_cols is what a tuning of cols = 0 runs.
bool pipe_has_cols(int K, int stages, int arith, int cols);
int pipe_default_cols(int K, int stages, int arith);
// Cells per lane the pipelined kernel runs for a requested tuning.vec: 5
// (fast5, K = 16..20, nx % 5 == 0: lanes never straddle the array edge; 8-B
// aligned accesses), else 4 / 2 with 16-B aligned arrays and nx % 4 / % 2,
// else 1. The executor's frame geometry uses the same answer.
int pipe_vec(int K, int stages, int arith, int64_t nx, int requested, bool aligned16);
// Blocks per CU of the core pipelined kernel (occ[0]) and of its direct-store
// variant (occ[1]; 0 when it has none; both 0 outside the core library) for
// (K, stages, arith, V): the
// executor prices direct-store passes with it (DiffusionExecutor::set_direct).
void stencil_pipe_occupancy(int K, int stages, int arith, int V, int occ[2]);
// arith: 0 fast5, 1 canonical, 2 fast5 with ds_bpermute lane moves (kernel 11)
void stencil_pipe_rects_gpu(int K, int stages, int arith, double* T2, const double* T,
                            const double* iCp, int64_t nx, int64_t ny, const Rect* rects,
                            int nrects, const StencilCoef& c, const StencilTuning& tune,
                            stream_t stream);
// CPU twins of the fast5 arithmetic (one step / K steps, same operations and
// rounding as kernels 5-9: std::fma, -ffp-contract=off); the intermediate
// levels are updated on the interior only, like stencilk_rects_cpu.
void stencil5_rects_cpu(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                        const Rect* rects, int nrects, const StencilCoef& c);
void stencilk5_rects_cpu(int K, double* T2, const double* T, const double* iCp, int64_t nx,
                         int64_t ny, const Rect* rects, int nrects, const StencilCoef& c);
// the split fast-math form (kernels 14 / 15), see stencil_pipe.h kArFast6Reg
void stencil6_rects_cpu(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                        const Rect* rects, int nrects, const StencilCoef& c);
void stencilk6_rects_cpu(int K, double* T2, const double* T, const double* iCp, int64_t nx,
                         int64_t ny, const Rect* rects, int nrects, const StencilCoef& c);

// Width (in cells) of one wave's x-strip in the march kernel; perf_hide rounds
// its x-frame so the interior rect starts on a strip boundary.
int stencil_vec(int64_t nx, const StencilTuning& tune);
int stencil_strip_cells(int64_t nx, const StencilTuning& tune);

// ---------------------------------------------------------------------------
// kp: the three-kernel formulation (K1-K3; scripts/diffusion_2D_kp.jl:16-54).
// QX, QY, D are full (ny, nx) buffers indexed like T (see kp.hip):
//   QX[y][x] = reference qx[y-1][x]   (rows 1..ny-2, cols 0..nx-2)
//   QY[y][x] = reference qy[y][x-1]   (rows 0..ny-2, cols 1..nx-2)
//   D [y][x] = reference dTdt[y-1][x-1] (interior)
// The GPU versions use 16-byte accesses for even nx and aligned buffers and a
// scalar path otherwise.
// ---------------------------------------------------------------------------
void flux_gpu(double* QX, double* QY, const double* T, int64_t nx, int64_t ny, double mlam,
              double rdx, double rdy, stream_t stream);
void residual_gpu(double* D, const double* QX, const double* QY, const double* iCp, int64_t nx,
                  int64_t ny, double rdx, double rdy, stream_t stream);
void update_gpu(double* T, const double* D, int64_t nx, int64_t ny, double dt, stream_t stream);
void flux_cpu(double* QX, double* QY, const double* T, int64_t nx, int64_t ny, double mlam,
              double rdx, double rdy);
void residual_cpu(double* D, const double* QX, const double* QY, const double* iCp, int64_t nx,
                  int64_t ny, double rdx, double rdy);
void update_cpu(double* T, const double* D, int64_t nx, int64_t ny, double dt);
bool kp_native_layout_ok(int64_t nx);

// ---------------------------------------------------------------------------
// Initial conditions (K9/K10). Device-side so a 288 GB tile never touches the
// host.
// ---------------------------------------------------------------------------
// Geometry of a local tile inside the implicit global grid: global coordinate
// of local cell ix is x = (gx0 + ix)*dx + xoff, wrapped into [0, nxg*dx) when
// periodic (ImplicitGlobalGrid x_g semantics).
struct TileGeom {
  int64_t gx0, gy0;    // global index of local cell (0,0)
  int64_t nxg, nyg;    // global grid size
  double dx, dy;
  double xoff, yoff;   // staggering offsets 0.5*(n - size(A))*d
  int periodx, periody;
};

// T = exp(-(x+dx/2-lx/2)^2 - (y+dy/2-ly/2)^2)   (ap.jl:28)
void init_gaussian_gpu(double* T, int64_t nx, int64_t ny, const TileGeom& g, double lx, double ly,
                       stream_t stream);
void init_gaussian_cpu(double* T, int64_t nx, int64_t ny, const TileGeom& g, double lx, double ly);
// Counter-based uniform [lo,hi) keyed by the GLOBAL cell index, so every
// decomposition of the same global grid sees the same field (bitwise) and the
// overlap cells of neighbouring ranks agree.
void init_random_gpu(double* A, int64_t nx, int64_t ny, const TileGeom& g, uint64_t seed,
                     double lo, double hi, stream_t stream);
void init_random_cpu(double* A, int64_t nx, int64_t ny, const TileGeom& g, uint64_t seed,
                     double lo, double hi);
void fill_gpu(double* A, int64_t n, double value, stream_t stream);

// ---------------------------------------------------------------------------
// Halo pack / unpack (K7/K8): strided 2D block copy. Both sides have a
// contiguous inner dimension of n_k elements; outer rows are dst_ld / src_ld
// elements apart. Element size in bytes: 2, 4, 8 or 16.
// ---------------------------------------------------------------------------
void copy2d_gpu(void* dst, int64_t dst_ld, const void* src, int64_t src_ld, int64_t n_o,
                int64_t n_k, int elem_bytes, stream_t stream);
void copy2d_cpu(void* dst, int64_t dst_ld, const void* src, int64_t src_ld, int64_t n_o,
                int64_t n_k, int elem_bytes);
// Up to kCopy2dBatch independent copies of one element size in ONE launch
// (the halo engine issues all packs of a dimension, then all its unpacks, as
// one batch each). Empty copies are skipped.
constexpr int kCopy2dBatch = 8;
struct Copy2d {
  void* dst;
  int64_t dst_ld;
  const void* src;
  int64_t src_ld, n_o, n_k;
};
void copy2d_batch_gpu(const Copy2d* copies, int n, int elem_bytes, stream_t stream);
void copy2d_batch_cpu(const Copy2d* copies, int n, int elem_bytes);

// ---------------------------------------------------------------------------
// Streaming roofline probes (same-box HBM ceiling for the T_eff comparison):
//   copy : b[i] = a[i]              (1 read + 1 write)
//   triad: c[i] = a[i] + s*b[i]     (2 reads + 1 write = the stencil's mix)
// 16-byte vector accesses, grid-stride.
// ---------------------------------------------------------------------------
void stream_copy_gpu(double* b, const double* a, int64_t n, int nt, int blocks, stream_t stream);
void stream_triad_gpu(double* c, const double* a, const double* b, double s, int64_t n, int nt,
                      int blocks, stream_t stream);

// ---------------------------------------------------------------------------
// Stream-ordered flags in host-registered shared memory (flags.hip; the HIP
// IPC transport's stream mode): wait until *flag == want (bounded: after
// timeout_s the kernel stores `code` into *err and exits), or store value
// with system-scope release. One 64-lane workgroup each; graph-capturable.
// ---------------------------------------------------------------------------
void flag_wait_gpu(const uint64_t* flag, uint64_t want, double timeout_s, uint32_t* err,
                   uint32_t code, stream_t stream);
void flag_write_gpu(uint64_t* flag, uint64_t value, stream_t stream);
// Direct-store halo passes: wait until every flags[i] with bit i of mask set
// is >= want (bounded, as flag_wait_gpu); store value into every non-null
// dst[i] (system-scope release), i < 8. One 64-lane workgroup each.
void flags_wait_ge_gpu(const uint64_t* flags, uint32_t mask, uint64_t want, double timeout_s,
                       uint32_t* err, uint32_t code, stream_t stream);
struct FlagTargets {
  uint64_t* dst[8] = {};
};
void flags_write_gpu(const FlagTargets& t, uint64_t value, stream_t stream);

// ---------------------------------------------------------------------------
// Reductions for verification / NaN guards. Result is written
// to out (device memory, 1 double). workspace must hold reduce_workspace_doubles().
// ---------------------------------------------------------------------------
enum ReduceOp : int { kSum = 0, kMax = 1, kMin = 2, kMaxAbs = 3, kNonFinite = 4 };
int64_t reduce_workspace_doubles();
void reduce_gpu(const double* A, int64_t n, int op, double* out, double* workspace,
                stream_t stream);
double reduce_cpu(const double* A, int64_t n, int op);
// One pass over a field: out3 = {non-finite count, min, max of the finite cells}
// (device memory; workspace: field_stats_workspace_doubles()). The full-field
// check of a timed run (bench.py).
int64_t field_stats_workspace_doubles();
void field_stats_gpu(const double* A, int64_t n, double* out3, double* workspace,
                     stream_t stream);
void field_stats_cpu(const double* A, int64_t n, double* out3);

}  // namespace rma
