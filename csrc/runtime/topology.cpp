#include "rma/topology.h"

#include <algorithm>

#include "rma/common.h"

namespace rma {

std::array<int, 3> dims_create(int nprocs, std::array<int, 3> dims) {
  RMA_CHECK_ARG(nprocs >= 1, "nprocs=" << nprocs);
  int fixed = 1;
  std::vector<int> free_idx;
  for (int d = 0; d < 3; ++d) {
    RMA_CHECK_ARG(dims[d] >= 0, "dims[" << d << "]=" << dims[d] << " must be >= 0");
    if (dims[d] > 0)
      fixed *= dims[d];
    else
      free_idx.push_back(d);
  }
  RMA_CHECK_ARG(nprocs % fixed == 0,
                "nprocs=" << nprocs << " not divisible by the product of fixed dims " << fixed);
  int rest = nprocs / fixed;
  if (free_idx.empty()) {
    RMA_CHECK_ARG(rest == 1, "prod(dims)=" << fixed << " != nprocs=" << nprocs);
    return dims;
  }
  // prime factors, largest first, each to the currently smallest free slot
  std::vector<int> primes;
  for (int p = 2; (int64_t)p * p <= rest; ++p)
    while (rest % p == 0) {
      primes.push_back(p);
      rest /= p;
    }
  if (rest > 1) primes.push_back(rest);
  std::sort(primes.rbegin(), primes.rend());
  std::vector<int> slot(free_idx.size(), 1);
  for (int p : primes) {
    auto it = std::min_element(slot.begin(), slot.end());
    *it *= p;
  }
  std::sort(slot.rbegin(), slot.rend());  // non-increasing, as MPI_Dims_create
  for (size_t i = 0; i < free_idx.size(); ++i) dims[free_idx[i]] = slot[i];
  return dims;
}

CartTopology::CartTopology(int nprocs, std::array<int, 3> dims, std::array<int, 3> periods)
    : nprocs_(nprocs), dims_(dims), periods_(periods) {
  RMA_CHECK_ARG(dims[0] >= 1 && dims[1] >= 1 && dims[2] >= 1, "dims must be >= 1");
  RMA_CHECK_ARG(dims[0] * dims[1] * dims[2] == nprocs,
                "prod(dims)=" << dims[0] * dims[1] * dims[2] << " != nprocs=" << nprocs);
}

std::array<int, 3> CartTopology::coords(int rank) const {
  RMA_CHECK_ARG(rank >= 0 && rank < nprocs_, "rank " << rank << " out of range");
  std::array<int, 3> c;
  c[2] = rank % dims_[2];
  c[1] = (rank / dims_[2]) % dims_[1];
  c[0] = rank / (dims_[2] * dims_[1]);
  return c;
}

int CartTopology::rank_of(std::array<int, 3> c) const {
  for (int d = 0; d < 3; ++d) {
    if (c[d] < 0 || c[d] >= dims_[d]) {
      if (!periods_[d]) return kProcNull;
      c[d] = ((c[d] % dims_[d]) + dims_[d]) % dims_[d];
    }
  }
  return (c[0] * dims_[1] + c[1]) * dims_[2] + c[2];
}

std::array<int, 2> CartTopology::shift(int rank, int dim) const {
  RMA_CHECK_ARG(dim >= 0 && dim < 3, "dim=" << dim);
  auto lo = coords(rank), hi = coords(rank);
  lo[dim] -= 1;
  hi[dim] += 1;
  return {rank_of(lo), rank_of(hi)};
}

std::array<std::array<int, 2>, 3> CartTopology::neighbors(int rank) const {
  return {shift(rank, 0), shift(rank, 1), shift(rank, 2)};
}

std::array<int, 4> CartTopology::diagonals(int rank) const {
  std::array<int, 4> out{};
  const auto c = coords(rank);
  for (int k = 0; k < 4; ++k) {
    auto d = c;
    d[0] += (k & 1) ? 1 : -1;
    d[1] += (k & 2) ? 1 : -1;
    out[k] = rank_of(d);
  }
  return out;
}

GridDesc make_grid_desc(int nx, int ny, int nz, const int dims[3], const int periods[3],
                        const int overlaps[3], const int halowidths[3], int nprocs, int rank) {
  RMA_CHECK_ARG(nprocs >= 1 && rank >= 0 && rank < nprocs, "rank " << rank << " of " << nprocs);
  RMA_CHECK_ARG(nx >= 1 && ny >= 1 && nz >= 1, "local sizes " << nx << "x" << ny << "x" << nz);
  GridDesc g;
  g.nxyz = {nx, ny, nz};
  g.nprocs = nprocs;
  g.me = rank;
  std::array<int, 3> din{0, 0, 0};
  for (int d = 0; d < 3; ++d) {
    din[d] = dims ? dims[d] : 0;
    g.periods[d] = periods ? (periods[d] ? 1 : 0) : 0;
    g.overlaps[d] = overlaps ? overlaps[d] : 2;
    g.hw[d] = halowidths ? halowidths[d] : std::max(1, g.overlaps[d] / 2);
    RMA_CHECK_ARG(din[d] >= 0, "dims[" << d << "] = " << din[d]);
    if (g.nxyz[d] == 1) {
      RMA_CHECK_ARG(din[d] <= 1 && !g.periods[d],
                    "dimension " << d << " has local size 1: it cannot be split or periodic");
      din[d] = 1;
    } else {
      RMA_CHECK_ARG(g.hw[d] >= 1 && g.overlaps[d] >= 2 * g.hw[d],
                    "dim " << d << ": overlap " << g.overlaps[d] << " must be >= 2*halowidth "
                           << g.hw[d]);
      RMA_CHECK_ARG(g.nxyz[d] >= g.overlaps[d] + g.hw[d],
                    "dim " << d << ": local size " << g.nxyz[d] << " < overlap + halowidth");
    }
  }
  g.dims = dims_create(nprocs, din);
  const CartTopology topo(nprocs, g.dims, g.periods);
  g.coords = topo.coords(rank);
  g.neighbors = topo.neighbors(rank);
  for (int d = 0; d < 3; ++d)
    g.nxyz_g[d] = g.nxyz[d] == 1 ? 1
                                 : (int64_t)g.dims[d] * (g.nxyz[d] - g.overlaps[d]) +
                                       (g.periods[d] ? 0 : g.overlaps[d]);
  return g;
}

double grid_coord(const GridDesc& g, int d, int64_t ix, double dd, int64_t size_A) {
  RMA_CHECK_ARG(d >= 0 && d < 3, "dim " << d);
  const double x0 = 0.5 * (double)(g.nxyz[d] - size_A) * dd;
  double x = (double)((int64_t)g.coords[d] * (g.nxyz[d] - g.overlaps[d]) + ix) * dd + x0;
  if (g.periods[d]) {
    const int64_t n = g.nxyz_g[d];
    x = x - dd;
    if (x > (double)(n - 1) * dd) x = x - (double)n * dd;
    if (x < 0) x = x + (double)n * dd;
  }
  return x;
}

}  // namespace rma
