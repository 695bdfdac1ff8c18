// Kernel-programming formulation: Flux / Residual / Update as three launches.
// Reference: scripts/diffusion_2D_kp.jl:16-54 (launched with (32,8) groups and a
// host wait after each, :88-90). Here they are stream-ordered (no host waits),
// use 64-wide wave rows (block 64x4) and compute exactly the canonical
// expression of rma/common.h, so kp == perf bitwise.
#include <hip/hip_runtime.h>

#include "rma/hip_check.h"
#include "rma/kernels.h"

namespace rma {
namespace {

constexpr int kBX = 64, kBY = 4;

__global__ __launch_bounds__(kBX* kBY) void flux_kernel(double* __restrict__ qx,
                                                         double* __restrict__ qy,
                                                         const double* __restrict__ T, int64_t nx,
                                                         int64_t ny, double mlam, double rdx,
                                                         double rdy) {
  const int64_t i = (int64_t)blockIdx.x * kBX + threadIdx.x;
  const int64_t j = (int64_t)blockIdx.y * kBY + threadIdx.y;
  // qx: (ny-2) x (nx-1);  qx[j][i] = (mlam*(T[j+1][i+1]-T[j+1][i]))*rdx
  if (i < nx - 1 && j < ny - 2) {
    const double* r = T + (j + 1) * nx;
    qx[j * (nx - 1) + i] = (mlam * (r[i + 1] - r[i])) * rdx;
  }
  // qy: (ny-1) x (nx-2);  qy[j][i] = (mlam*(T[j+1][i+1]-T[j][i+1]))*rdy
  if (i < nx - 2 && j < ny - 1) {
    qy[j * (nx - 2) + i] = (mlam * (T[(j + 1) * nx + i + 1] - T[j * nx + i + 1])) * rdy;
  }
}

__global__ __launch_bounds__(kBX* kBY) void residual_kernel(double* __restrict__ dTdt,
                                                             const double* __restrict__ qx,
                                                             const double* __restrict__ qy,
                                                             const double* __restrict__ iCp,
                                                             int64_t nx, int64_t ny, double rdx,
                                                             double rdy) {
  const int64_t i = (int64_t)blockIdx.x * kBX + threadIdx.x;
  const int64_t j = (int64_t)blockIdx.y * kBY + threadIdx.y;
  if (i < nx - 2 && j < ny - 2) {
    const double ddx = (qx[j * (nx - 1) + i + 1] - qx[j * (nx - 1) + i]) * rdx;
    const double ddy = (qy[(j + 1) * (nx - 2) + i] - qy[j * (nx - 2) + i]) * rdy;
    dTdt[j * (nx - 2) + i] = iCp[(j + 1) * nx + i + 1] * (-(ddx + ddy));
  }
}

__global__ __launch_bounds__(kBX* kBY) void update_kernel(double* __restrict__ T,
                                                           const double* __restrict__ dTdt,
                                                           int64_t nx, int64_t ny, double dt) {
  const int64_t i = (int64_t)blockIdx.x * kBX + threadIdx.x;
  const int64_t j = (int64_t)blockIdx.y * kBY + threadIdx.y;
  if (i < nx - 2 && j < ny - 2) {
    double* p = T + (j + 1) * nx + i + 1;
    *p = *p + dt * dTdt[j * (nx - 2) + i];
  }
}

dim3 grid_for(int64_t nx, int64_t ny) {
  const int64_t gx = (nx + kBX - 1) / kBX, gy = (ny + kBY - 1) / kBY;
  RMA_CHECK_ARG(gy <= 65535 && gx < (1LL << 31), "grid too large for kp kernels: " << nx << "x" << ny);
  return dim3((unsigned)gx, (unsigned)gy);
}

}  // namespace

void flux_gpu(double* qx, double* qy, const double* T, int64_t nx, int64_t ny, double mlam,
              double rdx, double rdy, stream_t stream) {
  RMA_CHECK_ARG(nx >= 3 && ny >= 3, "grid too small");
  flux_kernel<<<grid_for(nx, ny), dim3(kBX, kBY), 0, as_stream(stream)>>>(qx, qy, T, nx, ny, mlam,
                                                                         rdx, rdy);
  RMA_HIP_LAUNCH_CHECK();
}

void residual_gpu(double* dTdt, const double* qx, const double* qy, const double* iCp, int64_t nx,
                  int64_t ny, double rdx, double rdy, stream_t stream) {
  RMA_CHECK_ARG(nx >= 3 && ny >= 3, "grid too small");
  residual_kernel<<<grid_for(nx, ny), dim3(kBX, kBY), 0, as_stream(stream)>>>(dTdt, qx, qy, iCp, nx,
                                                                             ny, rdx, rdy);
  RMA_HIP_LAUNCH_CHECK();
}

void update_gpu(double* T, const double* dTdt, int64_t nx, int64_t ny, double dt, stream_t stream) {
  RMA_CHECK_ARG(nx >= 3 && ny >= 3, "grid too small");
  update_kernel<<<grid_for(nx, ny), dim3(kBX, kBY), 0, as_stream(stream)>>>(T, dTdt, nx, ny, dt);
  RMA_HIP_LAUNCH_CHECK();
}

}  // namespace rma
