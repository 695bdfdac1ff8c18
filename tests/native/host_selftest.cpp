// Host-side self test of the native core, built with AddressSanitizer and
// UndefinedBehaviorSanitizer (tests/test_native_host_asan.py). Covers the pure
// host code: topology, CPU stencil / kp twins, pack/unpack, reductions,
// argument validation (exceptions instead of out-of-bounds access).
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "rma/kernels.h"
#include "rma/topology.h"

#define EXPECT(c)                                                   \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "FAILED %s at line %d\n", #c, __LINE__); \
      return 1;                                                     \
    }                                                               \
  } while (0)

int main() {
  using namespace rma;
  // topology
  EXPECT((dims_create(8, {0, 0, 1}) == std::array<int, 3>{4, 2, 1}));
  EXPECT((dims_create(12, {0, 0, 0}) == std::array<int, 3>{3, 2, 2}));
  bool threw = false;
  try {
    dims_create(6, {4, 0, 1});
  } catch (const Error&) {
    threw = true;
  }
  EXPECT(threw);
  CartTopology t(8, {4, 2, 1}, {1, 0, 0});
  for (int r = 0; r < 8; ++r) {
    EXPECT(t.rank_of(t.coords(r)) == r);
    auto nb = t.neighbors(r);
    EXPECT(nb[0][0] >= 0 && nb[0][1] >= 0);  // periodic x
    EXPECT(nb[2][0] == kProcNull);
  }
  // stencil CPU twin vs kp CPU twin (bitwise)
  const int64_t nx = 37, ny = 29;
  std::vector<double> T(nx * ny), iCp(nx * ny), T2(nx * ny, 0.0);
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> u(0, 1);
  for (auto& v : T) v = u(g);
  for (auto& v : iCp) v = 0.5 + u(g);
  StencilCoef c{-1.3, 27.0, 24.0, 3e-4};
  Rect r{1, nx - 1, 1, ny - 1};
  stencil_rects_cpu(T2.data(), T.data(), iCp.data(), nx, ny, &r, 1, c);
  std::vector<double> QX(nx * ny), QY(nx * ny), D(nx * ny), Tk(T);
  flux_cpu(QX.data(), QY.data(), Tk.data(), nx, ny, c.mlam, c.rdx, c.rdy);
  residual_cpu(D.data(), QX.data(), QY.data(), iCp.data(), nx, ny, c.rdx, c.rdy);
  update_cpu(Tk.data(), D.data(), nx, ny, c.dt);
  for (int64_t y = 1; y < ny - 1; ++y)
    for (int64_t x = 1; x < nx - 1; ++x) EXPECT(Tk[y * nx + x] == T2[y * nx + x]);
  // invalid rects are rejected before any access
  threw = false;
  Rect bad{0, nx, 1, ny - 1};
  try {
    stencil_rects_cpu(T2.data(), T.data(), iCp.data(), nx, ny, &bad, 1, c);
  } catch (const Error&) {
    threw = true;
  }
  EXPECT(threw);
  // pack / unpack of a strided column
  std::vector<double> col(ny), back(nx * ny, -1.0);
  copy2d_cpu(col.data(), 1, T.data() + 3, nx, ny, 1, 8);
  copy2d_cpu(back.data() + 5, nx, col.data(), 1, ny, 1, 8);
  for (int64_t y = 0; y < ny; ++y) EXPECT(back[y * nx + 5] == T[y * nx + 3]);
  // reductions
  EXPECT(reduce_cpu(T.data(), nx * ny, kMaxAbs) <= 1.0);
  T[11] = NAN;
  EXPECT(reduce_cpu(T.data(), nx * ny, kNonFinite) == 1.0);
  std::puts("host selftest OK");
  return 0;
}
