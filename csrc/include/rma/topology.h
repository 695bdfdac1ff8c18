// Cartesian process topology (host-only, no communication needed).
//
// Re-implements the MPI pieces ImplicitGlobalGrid.init_global_grid relies on
// (Dims_create, Cart_create, Cart_coords, Cart_shift): the
// reference scripts only see the result (me, dims, nprocs, coords, comm_cart)
// at scripts/diffusion_2D_ap.jl:17. Ordering follows MPI's row-major Cartesian
// convention: rank = (c0*d1 + c1)*d2 + c2, so for dims (2,2,1) rank 1 is at
// coords (0,1,0).
#pragma once

#include <array>
#include <cstdint>
#include <vector>

namespace rma {

constexpr int kProcNull = -1;

// MPI_Dims_create semantics: entries of dims that are > 0 are fixed; zeros are
// filled so that prod(dims) == nprocs with the free entries as balanced as
// possible and in non-increasing order. Throws if impossible.
std::array<int, 3> dims_create(int nprocs, std::array<int, 3> dims);

class CartTopology {
 public:
  CartTopology(int nprocs, std::array<int, 3> dims, std::array<int, 3> periods);

  int nprocs() const { return nprocs_; }
  const std::array<int, 3>& dims() const { return dims_; }
  const std::array<int, 3>& periods() const { return periods_; }

  std::array<int, 3> coords(int rank) const;
  int rank_of(std::array<int, 3> coords) const;  // wraps periodic dims; kProcNull if outside
  // Cart_shift by +-1 along dim: {source(lo side), dest(hi side)}
  std::array<int, 2> shift(int rank, int dim) const;
  // neighbours[dim][0] = low side, [1] = high side (kProcNull at open edges)
  std::array<std::array<int, 2>, 3> neighbors(int rank) const;
  // the x-y diagonal neighbours (x-1,y-1), (x+1,y-1), (x-1,y+1), (x+1,y+1)
  // (kProcNull outside an open edge), for the merged halo exchange
  std::array<int, 4> diagonals(int rank) const;

 private:
  int nprocs_;
  std::array<int, 3> dims_;
  std::array<int, 3> periods_;
};

// The implicit global grid of one rank (ImplicitGlobalGrid init_global_grid,
// SURVEY.md C16/C17), host-only: what the C ABI (capi.cpp) and the Python
// layer compute before any GPU or communicator exists.
struct GridDesc {
  int nprocs = 1, me = 0;
  std::array<int, 3> nxyz{1, 1, 1}, dims{1, 1, 1}, periods{0, 0, 0}, overlaps{2, 2, 2},
      hw{1, 1, 1}, coords{0, 0, 0};
  std::array<int64_t, 3> nxyz_g{1, 1, 1};
  std::array<std::array<int, 2>, 3> neighbors{{{-1, -1}, {-1, -1}, {-1, -1}}};
};
// Null dims / periods / overlaps / halowidths mean IGG's defaults (auto, open,
// 2, overlap/2). Validates every argument (throws rma::Error).
GridDesc make_grid_desc(int nx, int ny, int nz, const int dims[3], const int periods[3],
                        const int overlaps[3], const int halowidths[3], int nprocs, int rank);
// IGG x_g / y_g / z_g: global coordinate of local index ix (0-based) of an
// array of size size_A along d (staggered arrays are offset by half a cell).
double grid_coord(const GridDesc& g, int d, int64_t ix, double dd, int64_t size_A);

}  // namespace rma
