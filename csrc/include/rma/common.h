// rocm_mpi_amd native core — shared types and error handling.
//
// Everything in the native layer works on raw device/host pointers plus explicit
// shapes; the Python layer owns the memory (torch tensors) and validates shapes
// before any launch. Layout convention: a 2D field is stored
// row-major as (ny, nx) with x fastest, i.e. identical in memory to the
// reference's Julia column-major A[ix,iy] (scripts/diffusion_2D_perf.jl:3-13).
#pragma once

#include <cstdint>
#include <sstream>
#include <stdexcept>
#include <string>

namespace rma {

// Error raised for any HIP / RCCL / argument failure. The message carries the
// rank (if known) so that a multi-rank failure points at the offending process
// ("check every HIP/RCCL return code, mapping errors to
// exceptions with rank id").
struct Error : public std::runtime_error {
  explicit Error(const std::string& m) : std::runtime_error(m) {}
};

int current_rank_for_errors();           // -1 if unknown
void set_rank_for_errors(int rank);

[[noreturn]] void throw_error(const char* what, const char* file, int line, const std::string& detail);

#define RMA_CHECK_ARG(cond, msg)                                                     \
  do {                                                                               \
    if (!(cond)) {                                                                   \
      std::ostringstream _oss;                                                       \
      _oss << msg;                                                                   \
      ::rma::throw_error("invalid argument: " #cond, __FILE__, __LINE__, _oss.str()); \
    }                                                                                \
  } while (0)

// Half-open rectangle of cells [x0,x1) x [y0,y1) to update.
struct Rect {
  int64_t x0, x1, y0, y1;
  bool empty() const { return x1 <= x0 || y1 <= y0; }
  int64_t cells() const { return empty() ? 0 : (x1 - x0) * (y1 - y0); }
};

// Coefficients of the explicit-Euler 5-point diffusion update. The canonical
// per-cell expression (identical in every variant, bitwise) is
//   qxR = (mlam*(T[y][x+1]-T[y][x]))*rdx    qxL = (mlam*(T[y][x]-T[y][x-1]))*rdx
//   qyU = (mlam*(T[y+1][x]-T[y][x]))*rdy    qyD = (mlam*(T[y][x]-T[y-1][x]))*rdy
//   T2  = T + dt*( iCp*( (-(qxR-qxL))*rdx - (qyU-qyD)*rdy ) )
// with mlam = -lam, rdx = 1/dx, rdy = 1/dy and iCp = 1/Cp stored as an array
// (the reference multiplies by Cp in perf.jl:8 but divides in ap.jl:40 /
// kp.jl:37; we standardise on a precomputed 1/Cp array which keeps the
// 3-array T_eff traffic). All native code is compiled
// with -ffp-contract=off so this is bit-reproducible against NumPy/torch.
struct StencilCoef {
  double mlam;  // -lam
  double rdx;   // 1/dx
  double rdy;   // 1/dy
  double dt;
};

}  // namespace rma
