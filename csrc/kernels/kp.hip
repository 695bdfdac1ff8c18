// Kernel-programming formulation: Flux / Residual / Update as three launches.
// Reference: scripts/diffusion_2D_kp.jl:16-54 (launched with (32,8) groups and a
// host wait after each, :88-90). Here they are stream-ordered (no host waits)
// and compute exactly the canonical expression of rma/common.h, so kp == perf
// bitwise.
//
// MI355X layout choice: the face fluxes and the residual live in full (ny,nx)
// buffers indexed like T ("in place staggering"), so every array shares T's
// row pitch and 16-byte alignment:
//   QX[y][x] = flux between cells x and x+1 of row y    (reference qx[y-1][x])
//   QY[y][x] = flux between rows y and y+1 of column x  (reference qy[y][x-1])
//   D [y][x] = dT/dt of interior cell (x,y)             (reference dTdt[y-1][x-1])
// Each thread then updates two cells with 16-byte loads/stores (one wave row
// = 1 KiB per access), blocks are rows of 512 cells padded to multiples of 8
// per row so that a row and the row below share an XCD's L2, and the outputs
// are streamed with non-temporal stores. kp is 10 array passes per step by
// construction (vs 3 for the fused kernel); the target is that traffic at the
// HBM roofline.
#include <hip/hip_runtime.h>

#include "rma/hip_check.h"
#include "rma/kernels.h"

namespace rma {
namespace {

constexpr int kThreads = 256;
constexpr int kCellsPerBlock = 2 * kThreads;
typedef double dbl2 __attribute__((ext_vector_type(2)));

struct RowGrid {
  int64_t nx, ny;
  int64_t row0;           // first row handled
  int64_t bpr;            // blocks per row (padded to a multiple of 8)
  int64_t bpr_used;       // blocks per row that have cells
};

RowGrid make_grid(int64_t nx, int64_t ny, int64_t row0, int64_t rows) {
  RowGrid g;
  g.nx = nx;
  g.ny = ny;
  g.row0 = row0;
  g.bpr_used = (nx + kCellsPerBlock - 1) / kCellsPerBlock;
  g.bpr = (g.bpr_used + 7) / 8 * 8;
  (void)rows;
  return g;
}

__device__ __forceinline__ bool locate(const RowGrid& g, int64_t& y, int64_t& x) {
  const int64_t b = blockIdx.x;
  const int64_t bx = b % g.bpr;
  if (bx >= g.bpr_used) return false;
  y = g.row0 + b / g.bpr;
  x = bx * kCellsPerBlock + 2 * (int64_t)threadIdx.x;
  return x < g.nx;
}

// VEC: 16-byte accesses (even nx, aligned buffers); otherwise two scalar
// accesses (odd nx / unaligned views), same arithmetic.
template <bool VEC>
__device__ __forceinline__ dbl2 ld2(const double* p) {
  if constexpr (VEC) {
    return *reinterpret_cast<const dbl2*>(p);
  } else {
    dbl2 t;
    t.x = p[0];
    t.y = p[1];
    return t;
  }
}

template <bool NT>
__device__ __forceinline__ void st1(double* p, double v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <bool NT, bool VEC>
__device__ __forceinline__ void st2(double* p, double a, double b, bool ma, bool mb) {
  if (VEC && ma && mb) {
    dbl2 t;
    t.x = a;
    t.y = b;
    if constexpr (NT) __builtin_nontemporal_store(t, reinterpret_cast<dbl2*>(p));
    else *reinterpret_cast<dbl2*>(p) = t;
  } else {
    if (ma) st1<NT>(p, a);
    if (mb) st1<NT>(p + 1, b);
  }
}

// rows y in [0, ny-1): QY[y][x] for x in [1, nx-1); rows y in [1, ny-1): QX[y][x], x in [0, nx-1)
template <bool NT, bool VEC>
__global__ __launch_bounds__(kThreads) void flux_kernel(double* __restrict__ QX,
                                                        double* __restrict__ QY,
                                                        const double* __restrict__ T, RowGrid g,
                                                        double mlam, double rdx, double rdy) {
  int64_t y, x;
  if (!locate(g, y, x)) return;
  const int64_t nx = g.nx;
  const double* r0 = T + y * nx;
  const double* r1 = r0 + nx;  // y+1 < ny always (y <= ny-2)
  // (odd nx: the last pair x = nx-1 has no second cell; clamp its loads)
  const int64_t xl = VEC ? x : (x + 1 < nx ? x : x - 1);
  const dbl2 a0 = ld2<VEC>(r0 + xl);
  const dbl2 b0 = ld2<VEC>(r1 + xl);
  const dbl2 a = (VEC || xl == x) ? a0 : dbl2{a0.y, a0.y};
  const dbl2 b = (VEC || xl == x) ? b0 : dbl2{b0.y, b0.y};
  // QY[y][x..x+1] = (mlam*(T[y+1][.] - T[y][.]))*rdy, columns 1..nx-2
  st2<NT, VEC>(QY + y * nx + x, (mlam * (b.x - a.x)) * rdy, (mlam * (b.y - a.y)) * rdy,
               x >= 1 && x <= nx - 2, x + 1 <= nx - 2);
  if (y >= 1) {  // QX[y][x..x+1] = (mlam*(T[y][.+1] - T[y][.]))*rdx, columns 0..nx-2
    const double a2 = (x + 2 < nx) ? r0[x + 2] : 0.0;
    st2<NT, VEC>(QX + y * nx + x, (mlam * (a.y - a.x)) * rdx, (mlam * (a2 - a.y)) * rdx,
                 x <= nx - 2, x + 1 <= nx - 2);
  }
}

// interior rows y in [1, ny-1), columns x in [1, nx-1)
template <bool NT, bool VEC>
__global__ __launch_bounds__(kThreads) void residual_kernel(double* __restrict__ D,
                                                            const double* __restrict__ QX,
                                                            const double* __restrict__ QY,
                                                            const double* __restrict__ iCp,
                                                            RowGrid g, double rdx, double rdy) {
  int64_t y, x;
  if (!locate(g, y, x)) return;
  const int64_t nx = g.nx;
  if (!VEC && x + 1 >= nx) return;  // odd nx: the last pair holds only the boundary cell
  const int64_t o = y * nx + x;
  const dbl2 qx = ld2<VEC>(QX + o);
  const double qxm = (x >= 1) ? QX[o - 1] : 0.0;
  const dbl2 qy = ld2<VEC>(QY + o);
  const dbl2 qym = ld2<VEC>(QY + o - nx);
  const dbl2 ic = ld2<VEC>(iCp + o);
  const double d0 = ic.x * (-((qx.x - qxm) * rdx + (qy.x - qym.x) * rdy));
  const double d1 = ic.y * (-((qx.y - qx.x) * rdx + (qy.y - qym.y) * rdy));
  st2<NT, VEC>(D + o, d0, d1, x >= 1 && x <= nx - 2, x + 1 <= nx - 2);
}

template <bool NT, bool VEC>
__global__ __launch_bounds__(kThreads) void update_kernel(double* __restrict__ T,
                                                          const double* __restrict__ D,
                                                          RowGrid g, double dt) {
  int64_t y, x;
  if (!locate(g, y, x)) return;
  const int64_t nx = g.nx;
  if (!VEC && x + 1 >= nx) return;  // odd nx: the last pair holds only the boundary cell
  const int64_t o = y * nx + x;
  const dbl2 t = ld2<VEC>(T + o);
  const dbl2 d = ld2<VEC>(D + o);
  st2<NT, VEC>(T + o, t.x + dt * d.x, t.y + dt * d.y, x >= 1 && x <= nx - 2, x + 1 <= nx - 2);
}

bool vec_ok(const void* a, const void* b, const void* c, int64_t nx) {
  return nx % 2 == 0 && ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                          reinterpret_cast<uintptr_t>(c)) & 15) == 0;
}

dim3 blocks(const RowGrid& g, int64_t rows) {
  const int64_t n = g.bpr * rows;
  RMA_CHECK_ARG(n < (int64_t(1) << 31), "grid too large");
  return dim3((unsigned)n);
}

}  // namespace

bool kp_native_layout_ok(int64_t nx) { return nx % 2 == 0; }

void flux_gpu(double* QX, double* QY, const double* T, int64_t nx, int64_t ny, double mlam,
              double rdx, double rdy, stream_t stream) {
  RMA_CHECK_ARG(nx >= 3 && ny >= 3, "grid too small");
  const RowGrid g = make_grid(nx, ny, 0, ny - 1);
  hipStream_t s = as_stream(stream);
  if (vec_ok(QX, QY, T, nx))
    flux_kernel<true, true><<<blocks(g, ny - 1), kThreads, 0, s>>>(QX, QY, T, g, mlam, rdx, rdy);
  else
    flux_kernel<true, false><<<blocks(g, ny - 1), kThreads, 0, s>>>(QX, QY, T, g, mlam, rdx, rdy);
  RMA_HIP_LAUNCH_CHECK();
}

void residual_gpu(double* D, const double* QX, const double* QY, const double* iCp, int64_t nx,
                  int64_t ny, double rdx, double rdy, stream_t stream) {
  RMA_CHECK_ARG(nx >= 3 && ny >= 3, "grid too small");
  const RowGrid g = make_grid(nx, ny, 1, ny - 2);
  hipStream_t s = as_stream(stream);
  if (vec_ok(D, QX, QY, nx) && vec_ok(iCp, iCp, iCp, nx))
    residual_kernel<true, true><<<blocks(g, ny - 2), kThreads, 0, s>>>(D, QX, QY, iCp, g, rdx,
                                                                      rdy);
  else
    residual_kernel<true, false><<<blocks(g, ny - 2), kThreads, 0, s>>>(D, QX, QY, iCp, g, rdx,
                                                                       rdy);
  RMA_HIP_LAUNCH_CHECK();
}

void update_gpu(double* T, const double* D, int64_t nx, int64_t ny, double dt, stream_t stream) {
  RMA_CHECK_ARG(nx >= 3 && ny >= 3, "grid too small");
  const RowGrid g = make_grid(nx, ny, 1, ny - 2);
  hipStream_t s = as_stream(stream);
  if (vec_ok(T, D, T, nx))
    update_kernel<false, true><<<blocks(g, ny - 2), kThreads, 0, s>>>(T, D, g, dt);
  else
    update_kernel<false, false><<<blocks(g, ny - 2), kThreads, 0, s>>>(T, D, g, dt);
  RMA_HIP_LAUNCH_CHECK();
}

}  // namespace rma
