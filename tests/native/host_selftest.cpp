// Host-side self test of the native core, built with AddressSanitizer and
// UndefinedBehaviorSanitizer (tests/test_native_host_asan.py). Covers the pure
// host code: topology and the C ABI's grid description, CPU stencil / kp /
// fast5 twins, pack/unpack, reductions, the executor's pass geometry and pass
// planner (plan.cpp), the halo exchange plan (halo_plan.cpp) executed on host
// memory for several fake ranks of one process (periodic self neighbours,
// minimal tiles, staggered n+1 fields, 2K overlaps, 3D), parallel_for
// exception propagation, and argument validation (exceptions instead of
// out-of-bounds access).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <random>
#include <stdexcept>
#include <vector>

#include "rma/halo_plan.h"
#include "rma/kernels.h"
#include "rma/parallel_for.h"
#include "rma/plan.h"
#include "rma/topology.h"

#define EXPECT(c)                                                   \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "FAILED %s at line %d\n", #c, __LINE__); \
      return 1;                                                     \
    }                                                               \
  } while (0)

namespace {
using namespace rma;

template <typename F>
bool throws(F&& f) {
  try {
    f();
  } catch (const Error&) {
    return true;
  }
  return false;
}

// N fake ranks of a Cartesian grid, each owning a local tile of a global
// field; one halo exchange executed from the plan on host memory (copy2d_cpu
// for copies / packs / unpacks, per-pair FIFO queues matching sends and
// receives in order, like RCCL). Afterwards every tile must equal its window
// of the global field. cross: the order of HaloExchanger::exchange_cross
// (packs of every dimension, ONE group with all sends and receives, unpacks):
// every cell must match except corners (cells in two dimensions' halos).
// merged: plan_exchange_merged (x and y in one group, corner blocks to the
// diagonal ranks), executed like cross; every cell, corners included, must match.
int halo_case(std::array<int, 3> dims, std::array<int, 3> periods, std::array<int, 3> n,
              std::array<int, 3> ol, std::array<int, 3> hw, int stagger_x, bool via_comm,
              bool cross = false, bool merged = false) {
  const bool one_group = cross || merged;
  const int P = dims[0] * dims[1] * dims[2];
  CartTopology topo(P, dims, periods);
  std::array<int64_t, 3> ng;
  for (int d = 0; d < 3; ++d)
    ng[d] = n[d] == 1 ? 1 : (int64_t)dims[d] * (n[d] - ol[d]) + (periods[d] ? 0 : ol[d]);
  // field 0: n; field 1: staggered along x (size n+stagger_x, overlap ol+stagger_x)
  auto gval = [&](int f, int64_t gx, int64_t gy, int64_t gz) {
    return 1000.0 * f + gx + 1e3 * (gy + 1) + 1e6 * (gz + 1);
  };
  struct Tile {
    std::array<std::vector<double>, 2> a;
    std::array<std::array<int64_t, 3>, 2> size;
  };
  std::vector<Tile> tiles(P);
  std::vector<std::vector<HaloField>> fields(P);
  auto gidx = [&](int r, int f, int d, int64_t i) {
    const int64_t c = topo.coords(r)[d];
    const int64_t nd = n[d] + (f == 1 && d == 0 ? stagger_x : 0);
    const int64_t ngd = ng[d] + (f == 1 && d == 0 && !periods[d] ? stagger_x : 0);
    int64_t g = c * (n[d] - ol[d]) + i;
    if (periods[d]) g = ((g % ngd) + ngd) % ngd;
    (void)nd;
    return g;
  };
  for (int r = 0; r < P; ++r) {
    for (int f = 0; f < 2; ++f) {
      auto& sz = tiles[r].size[f];
      sz = {n[0] + (f == 1 ? stagger_x : 0), n[1], n[2]};
      tiles[r].a[f].assign(sz[0] * sz[1] * sz[2], -7.0);
      const auto nb = topo.neighbors(r);
      for (int64_t z = 0; z < sz[2]; ++z)
        for (int64_t y = 0; y < sz[1]; ++y)
          for (int64_t x = 0; x < sz[0]; ++x) {
            // halo planes start as garbage, every other cell holds the global value
            const int64_t ix[3] = {x, y, z};
            bool halo = false;
            for (int d = 0; d < 3; ++d) {
              const int64_t s = sz[d], h = hw[d];
              const int64_t old = ol[d] + (s - n[d]);
              const bool hh = s > 1 && old >= 2 * h && s >= old + h;
              if (!hh) continue;
              if (nb[d][0] >= 0 && ix[d] < h) halo = true;
              if (nb[d][1] >= 0 && ix[d] >= s - h) halo = true;
            }
            if (!halo)
              tiles[r].a[f][(z * sz[1] + y) * sz[0] + x] =
                  gval(f, gidx(r, f, 0, x), gidx(r, f, 1, y), gidx(r, f, 2, z));
          }
      HaloField hf;
      hf.ptr = tiles[r].a[f].data();
      hf.size = sz;
      hf.elem_bytes = 8;
      for (int d = 0; d < 3; ++d) {
        hf.ol[d] = ol[d] + (sz[d] - n[d]);
        hf.hw[d] = hw[d];
      }
      fields[r].push_back(hf);
    }
  }
  std::vector<HaloPlan> plans(P);
  std::vector<std::vector<std::vector<double>>> bufs(P);
  for (int r = 0; r < P; ++r) {
    plans[r] = merged ? plan_exchange_merged(fields[r], topo.neighbors(r), topo.diagonals(r), r,
                                             via_comm)
                      : plan_exchange(fields[r], topo.neighbors(r), r, via_comm, 7);
    for (size_t b : plans[r].slot_bytes) bufs[r].push_back(std::vector<double>(b / 8, -9.0));
  }
  std::vector<std::vector<void*>> slots(P);
  for (int r = 0; r < P; ++r)
    for (auto& b : bufs[r]) slots[r].push_back(b.data());
  auto at = [&](int r, int f, const PlaneView& v) {
    return reinterpret_cast<char*>(fields[r][f].ptr) + v.offset * 8;
  };
  // dimension by dimension on every rank (the plans list the same dims)
  std::map<std::pair<int, int>, std::deque<std::vector<char>>> wire;
  if (one_group) {
    for (int r = 0; r < P; ++r) {
      if (!merged && plans[r].dims.size() != plans[0].dims.size()) return 101;
      if (merged && plans[r].dims.size() > 1) return 106;
      for (const HaloDimPlan& dp : plans[r].dims)
        for (const CopyBatch& b : batch_copies(dim_copies(dp, fields[r], slots[r], 0)))
          copy2d_batch_cpu(b.copies.data(), (int)b.copies.size(), b.elem_bytes);
    }
    for (int r = 0; r < P; ++r)  // the one group: every dimension's sends, then receives
      for (const HaloDimPlan& dp : plans[r].dims)
        for (const auto& m : dp.sends) {
          const char* src = m.slot >= 0 ? reinterpret_cast<const char*>(bufs[r][m.slot].data())
                                        : at(r, m.field, m.view);
          wire[{r, m.peer}].emplace_back(src, src + m.bytes);
        }
    for (int r = 0; r < P; ++r)
      for (const HaloDimPlan& dp : plans[r].dims)
        for (const auto& m : dp.recvs) {
          auto& q = wire[{m.peer, r}];
          if (q.empty()) return 102;
          if (q.front().size() != m.bytes) return 103;
          char* dst = m.slot >= 0 ? reinterpret_cast<char*>(bufs[r][m.slot].data())
                                  : at(r, m.field, m.view);
          std::memcpy(dst, q.front().data(), m.bytes);
          q.pop_front();
        }
    for (int r = 0; r < P; ++r)
      for (const HaloDimPlan& dp : plans[r].dims)
        for (const CopyBatch& b : batch_copies(dim_copies(dp, fields[r], slots[r], 1)))
          copy2d_batch_cpu(b.copies.data(), (int)b.copies.size(), b.elem_bytes);
  }
  for (size_t k = 0; !one_group && k < plans[0].dims.size(); ++k) {
    for (int r = 0; r < P; ++r) {
      if (plans[r].dims.size() != plans[0].dims.size()) return 101;
      const HaloDimPlan& dp = plans[r].dims[k];
      // the engine's batches (halo.cpp), executed by the CPU twin
      for (const CopyBatch& b : batch_copies(dim_copies(dp, fields[r], slots[r], 0)))
        copy2d_batch_cpu(b.copies.data(), (int)b.copies.size(), b.elem_bytes);
      for (const auto& m : dp.sends) {
        const char* src = m.slot >= 0 ? reinterpret_cast<const char*>(bufs[r][m.slot].data())
                                      : at(r, m.field, m.view);
        wire[{r, m.peer}].emplace_back(src, src + m.bytes);
      }
    }
    for (int r = 0; r < P; ++r) {
      const HaloDimPlan& dp = plans[r].dims[k];
      for (const auto& m : dp.recvs) {
        auto& q = wire[{m.peer, r}];
        if (q.empty()) return 102;
        if (q.front().size() != m.bytes) return 103;
        char* dst = m.slot >= 0 ? reinterpret_cast<char*>(bufs[r][m.slot].data())
                                : at(r, m.field, m.view);
        std::memcpy(dst, q.front().data(), m.bytes);
        q.pop_front();
      }
      for (const CopyBatch& b : batch_copies(dim_copies(dp, fields[r], slots[r], 1)))
        copy2d_batch_cpu(b.copies.data(), (int)b.copies.size(), b.elem_bytes);
    }
  }
  for (auto& kv : wire)
    if (!kv.second.empty()) return 104;
  for (int r = 0; r < P; ++r)
    for (int f = 0; f < 2; ++f) {
      const auto& sz = tiles[r].size[f];
      const auto nb = topo.neighbors(r);
      for (int64_t z = 0; z < sz[2]; ++z)
        for (int64_t y = 0; y < sz[1]; ++y)
          for (int64_t x = 0; x < sz[0]; ++x) {
            if (cross) {  // corners: in the halo of two or more dimensions
              const int64_t ix[3] = {x, y, z};
              int nh = 0;
              for (int d = 0; d < 3; ++d) {
                const int64_t s = sz[d], h = hw[d], old = ol[d] + (s - n[d]);
                if (!(s > 1 && old >= 2 * h && s >= old + h)) continue;
                nh += (nb[d][0] >= 0 && ix[d] < h) || (nb[d][1] >= 0 && ix[d] >= s - h);
              }
              if (nh >= 2) continue;
            }
            const double want = gval(f, gidx(r, f, 0, x), gidx(r, f, 1, y), gidx(r, f, 2, z));
            if (tiles[r].a[f][(z * sz[1] + y) * sz[0] + x] != want) {
              std::fprintf(stderr, "halo mismatch rank %d field %d at (%ld,%ld,%ld)\n", r, f,
                           (long)x, (long)y, (long)z);
              return 105;
            }
          }
    }
  return 0;
}
}  // namespace

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
  // copy batching: plan order per element size, <= kCopy2dBatch per batch
  {
    std::vector<std::pair<int, Copy2d>> q;
    std::vector<std::vector<uint32_t>> bufs(2 * kCopy2dBatch + 3, std::vector<uint32_t>(8, 0));
    for (int i = 0; i < 2 * kCopy2dBatch + 3; ++i) {
      for (auto& v : bufs[i]) v = (uint32_t)i;
      // one 4-byte copy in every third slot, 8-byte copies otherwise
      const int eb = i % 3 == 1 ? 4 : 8;
      q.push_back({eb, {bufs[i].data() + 4, 1, bufs[i].data(), 1, 4 * 4 / eb, 1}});
    }
    const std::vector<CopyBatch> bs = batch_copies(q);
    size_t total = 0;
    int prev8 = -1;
    for (const CopyBatch& b : bs) {
      EXPECT(!b.copies.empty() && (int)b.copies.size() <= kCopy2dBatch);
      total += b.copies.size();
      for (const Copy2d& c : b.copies) {
        EXPECT((b.elem_bytes == 4) == ((static_cast<const uint32_t*>(c.src))[0] % 3 == 1));
        if (b.elem_bytes == 8) {  // plan order kept within an element size
          const int idx = (int)(static_cast<const uint32_t*>(c.src))[0];
          EXPECT(idx > prev8);
          prev8 = idx;
        }
      }
      copy2d_batch_cpu(b.copies.data(), (int)b.copies.size(), b.elem_bytes);
    }
    EXPECT(total == q.size());
    for (auto& b : bufs)
      for (int k = 4; k < 8; ++k) EXPECT(b[k] == b[0]);
    EXPECT(throws([&] { copy2d_batch_cpu(nullptr, kCopy2dBatch + 1, 8); }));
  }
  // reductions
  EXPECT(reduce_cpu(T.data(), nx * ny, kMaxAbs) <= 1.0);
  T[11] = NAN;
  EXPECT(reduce_cpu(T.data(), nx * ny, kNonFinite) == 1.0);
  // fast5 CPU twin: K passes == K one-step passes, finite, differs from canonical
  {
    std::vector<double> a(nx * ny), b(nx * ny), k3(nx * ny);
    for (auto& v : T) v = u(g);
    stencil5_rects_cpu(a.data(), T.data(), iCp.data(), nx, ny, &r, 1, c);
    for (int64_t i = 0; i < nx * ny; ++i)
      if (!(i % nx == 0 || i % nx == nx - 1 || i / nx == 0 || i / nx == ny - 1)) continue;
      else a[i] = T[i];
    stencil5_rects_cpu(b.data(), a.data(), iCp.data(), nx, ny, &r, 1, c);
    stencilk5_rects_cpu(2, k3.data(), T.data(), iCp.data(), nx, ny, &r, 1, c);
    for (int64_t y = 1; y < ny - 1; ++y)
      for (int64_t x = 1; x < nx - 1; ++x) EXPECT(k3[y * nx + x] == b[y * nx + x]);
    EXPECT(throws([&] { stencil5_rects_cpu(b.data(), T.data(), iCp.data(), nx, ny, &r, 1,
                                           StencilCoef{0.0, 27.0, 24.0, 3e-4}); }));
  }
  // executor pass geometry (plan.cpp)
  {
    std::vector<Rect> fr;
    Rect in;
    split_rect({1, 99, 1, 49}, 4, 3, fr, in);
    EXPECT(fr.size() == 4 && in.x0 == 5 && in.x1 == 95 && in.y0 == 4 && in.y1 == 46);
    int64_t cells = in.cells();
    for (auto& q : fr) cells += q.cells();
    EXPECT(cells == 98 * 48);
    split_rect({1, 9, 1, 9}, 5, 1, fr, in);  // frame swallows the rect
    EXPECT(fr.size() == 1 && in.empty());
    split_rect({1, 1, 1, 9}, 1, 1, fr, in);  // empty rect
    EXPECT(fr.empty() && in.empty());
    EXPECT(throws([&] { split_rect({1, 9, 1, 9}, -1, 1, fr, in); }));
    const Neighbors none{{{-1, -1}, {-1, -1}, {-1, -1}}}, all{{{1, 1}, {2, 2}, {-1, -1}}},
        self{{{0, 0}, {0, 0}, {-1, -1}}}, xhi_ylo{{{-1, 3}, {4, -1}, {-1, -1}}},
        xlo{{{5, -1}, {-1, -1}, {-1, -1}}};
    // per-side frames: only sides with a neighbour
    split_rect_sides({1, 99, 1, 49}, 0, 4, 3, 0, fr, in);
    EXPECT(fr.size() == 2 && in.x0 == 1 && in.x1 == 95 && in.y0 == 4 && in.y1 == 49);
    split_rect_sides({1, 99, 1, 49}, 0, 0, 0, 0, fr, in);
    EXPECT(fr.empty() && in.x0 == 1 && in.x1 == 99 && in.y0 == 1 && in.y1 == 49);
    {
      const auto sd = frame_sides(xhi_ylo);
      EXPECT(!sd[0][0] && sd[0][1] && sd[1][0] && !sd[1][1]);
      const auto sn = frame_sides(none);
      EXPECT(!sn[0][0] && !sn[0][1] && !sn[1][0] && !sn[1][1]);
    }
    Rect o = owned_rect(100, 60, 16, all);
    EXPECT(o.x0 == 16 && o.x1 == 84 && o.y0 == 16 && o.y1 == 44);
    o = owned_rect(100, 60, 16, none);
    EXPECT(o.x0 == 1 && o.x1 == 99 && o.y0 == 1 && o.y1 == 59);
    EXPECT(throws([&] { owned_rect(20, 60, 10, all); }));  // minimal tile: nothing owned
    for (int K = 1; K <= 24; ++K) {
      for (const Neighbors* nb : {&none, &all, &self, &xhi_ylo, &xlo})
        for (int variant = 0; variant < 4; ++variant) {
        // variant 0: ol-wide frame strips on a small tile; 1, 2: frames of
        // whole pipelined tasks (aligned) on tiles large enough for them; 3:
        // tasks taller than 1024 rows: whole strip columns + ol-K-row bands
        const int64_t n0 = variant == 0 ? 2 * (2 * 24) + 8 : 2000 + 17 * variant;
        const int vec = variant == 2 ? 2 : 4;
        const int64_t tw = (64 * vec - 2 * K) / vec * vec, th = variant == 3 ? 2048 : 64 * variant;
        PassGeom pg = pass_geometry(n0, n0 + 3, K, *nb, true, 1, 1, 48, 48,
                                    variant ? tw : 0, variant ? th : 0, vec);
        if (variant && variant < 3 && nb != &none && K >= 1) {
          EXPECT(pg.aligned == (tw >= 48 - pg.out.x0 && th >= 48 - pg.out.y0));
        }
        if (variant == 3 && nb != &none) {
          EXPECT(pg.aligned == (tw >= 48 - pg.out.x0));
          if (pg.aligned)
            for (auto& q : pg.frame_wide) EXPECT(q.y1 - q.y0 == std::max<int64_t>(1, 48 - pg.out.y0));
        }
        if (pg.aligned) {  // every frame strip is one strip column of the grid
          for (auto& q : pg.frame_tall) {
            const int64_t xa = (q.x0 - K) - ((((q.x0 - K) % vec) + vec) % vec);
            EXPECT(q.x1 <= xa + K + tw && q.x1 > q.x0);
          }
          if ((*nb)[0][0] >= 0) EXPECT(((pg.interior.x0 - K) % vec + vec) % vec == 0);
        }
        int64_t c2 = pg.interior.cells();
        for (auto& q : pg.frame) {
          c2 += q.cells();
          EXPECT(q.x0 >= pg.out.x0 && q.x1 <= pg.out.x1 && q.y0 >= pg.out.y0 && q.y1 <= pg.out.y1);
        }
        EXPECT(c2 == pg.out.cells());
        // the shape split partitions the frame: wide strips are not taller than wide
        EXPECT(pg.frame_wide.size() + pg.frame_tall.size() == pg.frame.size());
        int64_t c3 = 0;
        for (auto& q : pg.frame_wide) {
          c3 += q.cells();
          EXPECT(q.x1 - q.x0 >= q.y1 - q.y0);
        }
        for (auto& q : pg.frame_tall) {
          c3 += q.cells();
          EXPECT(q.x1 - q.x0 < q.y1 - q.y0);
        }
        EXPECT(c3 + pg.interior.cells() == pg.out.cells());
        if (nb != &none && !pg.frame.empty() && !pg.interior.empty()) {
          // the frame holds the send planes [ol-hw, ol) of the sides with a
          // neighbour; an open side belongs to the interior launch
          const int64_t nxx = n0, nyy = n0 + 3;
          const Neighbors& b = *nb;
          EXPECT(b[0][0] >= 0 ? pg.interior.x0 >= 48 : pg.interior.x0 == pg.out.x0);
          EXPECT(b[0][1] >= 0 ? pg.interior.x1 <= nxx - 48 : pg.interior.x1 == pg.out.x1);
          EXPECT(b[1][0] >= 0 ? pg.interior.y0 >= 48 : pg.interior.y0 == pg.out.y0);
          EXPECT(b[1][1] >= 0 ? pg.interior.y1 <= nyy - 48 : pg.interior.y1 == pg.out.y1);
        }
        }
    }
  }
  // pass planner
  {
    const auto cf = default_pass_costs(24, true), cc = default_pass_costs(24, false);
    EXPECT(cf.size() == 25 && cc.size() == 25);
    for (int64_t nsteps : {0, 1, 2, 5, 19, 20, 21, 47, 1000, 5000, 100003}) {
      for (const auto* cost : {&cf, &cc}) {
        const auto p = plan_passes(nsteps, *cost);
        int64_t sum = 0;
        for (int k : p) {
          EXPECT(k >= 1 && k <= 24);
          sum += k;
        }
        EXPECT(sum == nsteps);
        for (size_t i = 1; i < p.size(); ++i) EXPECT(p[i] <= p[i - 1]);
      }
    }
    EXPECT(plan_passes(20, cf) == std::vector<int>{20});
    // tile classes: nearest measured table in log(cells); 0 = the 288 GB tile
    EXPECT(default_pass_costs(24, true, 101376.0 * 101376.0) == cf);
    EXPECT(default_pass_costs(24, true, 4096.0 * 4096.0) != cf);
    EXPECT(default_pass_costs(24, true, 4000.0 * 4000.0) ==
           default_pass_costs(24, true, 4096.0 * 4096.0));
    EXPECT(default_pass_costs(24, true, 64.0 * 64.0) ==
           default_pass_costs(24, true, 4096.0 * 4096.0));  // below the smallest class
    EXPECT(default_pass_costs(24, true, 2e11) == cf);       // above the largest
    {  // a cheaper table entry changes the plan of that class only
      auto c4 = default_pass_costs(24, true, 4096.0 * 4096.0);
      c4[10] = 0.01;
      EXPECT(plan_passes(20, c4) == (std::vector<int>{10, 10}));
      EXPECT(plan_passes(20, cf) == std::vector<int>{20});
    }
    EXPECT(default_pass_costs(12, false, 16384.0 * 16384.0).size() == 13);
    EXPECT(throws([&] { default_pass_costs(25, true); }));
    EXPECT(throws([&] { default_pass_costs(0, true); }));
    // DP optimality against brute force on small n
    std::function<double(int)> best = [&](int m) -> double {
      if (m == 0) return 0.0;
      double b = 1e300;
      for (int k = 1; k <= std::min(m, 24); ++k) b = std::min(b, best(m - k) + cf[k]);
      return b;
    };
    for (int m = 1; m <= 30; ++m) {
      double sum = 0;
      for (int k : plan_passes(m, cf)) sum += cf[k];
      EXPECT(std::fabs(sum - best(m)) < 1e-9);
    }
    auto c2 = cf;
    apply_cost_overrides(c2, "20:9.5,3:0.5");
    EXPECT(c2[20] == 9.5 && c2[3] == 0.5);
    EXPECT(plan_passes(20, c2)[0] != 20);
    EXPECT(throws([&] { apply_cost_overrides(c2, "30:1.0"); }));
    EXPECT(throws([&] { apply_cost_overrides(c2, "5"); }));
    EXPECT(throws([&] { apply_cost_overrides(c2, "5:-1"); }));
    EXPECT(throws([&] { plan_passes(-1, cf); }));
  }
  // halo exchange plans executed on host memory
  EXPECT(halo_case({2, 2, 1}, {0, 0, 0}, {12, 10, 1}, {2, 2, 2}, {1, 1, 1}, 1, false) == 0);
  EXPECT(halo_case({4, 2, 1}, {0, 0, 0}, {40, 36, 1}, {32, 32, 2}, {16, 16, 1}, 1, false) == 0);
  EXPECT(halo_case({2, 1, 1}, {1, 1, 0}, {10, 9, 1}, {4, 4, 2}, {2, 2, 1}, 0, false) == 0);
  EXPECT(halo_case({1, 1, 1}, {1, 1, 0}, {10, 9, 1}, {4, 4, 2}, {2, 2, 1}, 0, false) == 0);
  EXPECT(halo_case({1, 1, 1}, {1, 1, 0}, {10, 9, 1}, {4, 4, 2}, {2, 2, 1}, 0, true) == 0);
  EXPECT(halo_case({2, 2, 1}, {1, 0, 0}, {6, 6, 1}, {2, 2, 2}, {1, 1, 1}, 1, true) == 0);  // minimal
  EXPECT(halo_case({2, 1, 2}, {0, 0, 1}, {8, 7, 6}, {2, 2, 2}, {1, 1, 1}, 0, false) == 0);  // 3D
  // exchange_cross order (one group for all dimensions; corners not checked)
  EXPECT(halo_case({2, 2, 1}, {0, 0, 0}, {12, 10, 1}, {2, 2, 2}, {1, 1, 1}, 1, false, true) == 0);
  EXPECT(halo_case({2, 1, 1}, {1, 1, 0}, {10, 9, 1}, {4, 4, 2}, {2, 2, 1}, 0, false, true) == 0);
  EXPECT(halo_case({1, 1, 1}, {1, 1, 0}, {10, 9, 1}, {4, 4, 2}, {2, 2, 1}, 0, true, true) == 0);
  EXPECT(halo_case({2, 2, 1}, {1, 1, 0}, {6, 6, 1}, {2, 2, 2}, {1, 1, 1}, 1, true, true) == 0);
  EXPECT(halo_case({4, 2, 1}, {1, 1, 0}, {9, 8, 1}, {2, 2, 2}, {1, 1, 1}, 0, false, true) == 0);
  // merged x+y exchange (one group, corner blocks to the diagonals): every
  // cell incl. corners == the global field, open / periodic / mixed grids,
  // self neighbours by copy and through the transport, staggered fields,
  // width-K halos (2K overlaps) and a 4x2 grid of width-16 halos
  EXPECT(halo_case({2, 2, 1}, {0, 0, 0}, {12, 10, 1}, {2, 2, 2}, {1, 1, 1}, 1, false, false, true) == 0);
  EXPECT(halo_case({4, 2, 1}, {0, 0, 0}, {40, 36, 1}, {32, 32, 2}, {16, 16, 1}, 1, false, false, true) == 0);
  EXPECT(halo_case({4, 2, 1}, {1, 1, 0}, {9, 8, 1}, {2, 2, 2}, {1, 1, 1}, 0, false, false, true) == 0);
  EXPECT(halo_case({2, 1, 1}, {1, 1, 0}, {10, 9, 1}, {4, 4, 2}, {2, 2, 1}, 0, false, false, true) == 0);
  EXPECT(halo_case({1, 1, 1}, {1, 1, 0}, {10, 9, 1}, {4, 4, 2}, {2, 2, 1}, 0, false, false, true) == 0);
  EXPECT(halo_case({1, 1, 1}, {1, 1, 0}, {10, 9, 1}, {4, 4, 2}, {2, 2, 1}, 0, true, false, true) == 0);
  EXPECT(halo_case({2, 2, 1}, {1, 1, 0}, {6, 6, 1}, {2, 2, 2}, {1, 1, 1}, 1, true, false, true) == 0);
  EXPECT(halo_case({2, 2, 1}, {1, 0, 0}, {6, 6, 1}, {2, 2, 2}, {1, 1, 1}, 1, false, false, true) == 0);
  EXPECT(halo_case({3, 2, 1}, {0, 1, 0}, {20, 18, 1}, {8, 8, 2}, {4, 4, 1}, 1, false, false, true) == 0);
  EXPECT(halo_case({1, 3, 1}, {0, 0, 0}, {12, 14, 1}, {4, 4, 2}, {2, 2, 1}, 0, false, false, true) == 0);
  EXPECT(halo_case({3, 1, 1}, {0, 0, 0}, {12, 14, 1}, {4, 4, 2}, {2, 2, 1}, 0, false, false, true) == 0);
  {  // 3D fields are refused
    HaloField f3;
    f3.ptr = &f3;
    f3.size = {8, 8, 4};
    EXPECT(throws([&] {
      plan_exchange_merged({f3}, {{{1, 1}, {1, 1}, {-1, -1}}}, {1, 1, 1, 1}, 0, false);
    }));
  }
  {
    HaloField f;
    EXPECT(throws([&] { plan_exchange({f}, {{{1, 1}, {-1, -1}, {-1, -1}}}, 0, false, 7); }));
    double x = 0;
    f.ptr = &x;
    f.elem_bytes = 3;
    EXPECT(throws([&] { plan_exchange({f}, {{{1, 1}, {-1, -1}, {-1, -1}}}, 0, false, 7); }));
  }
  // grid description of the C ABI (make_grid_desc / grid_coord)
  {
    const int ol[3] = {4, 4, 2}, hw[3] = {2, 2, 1}, per[3] = {1, 0, 0};
    GridDesc gd = make_grid_desc(20, 12, 1, nullptr, per, ol, hw, 8, 5);
    EXPECT((gd.dims == std::array<int, 3>{4, 2, 1}));
    EXPECT(gd.nxyz_g[0] == 4 * 16 && gd.nxyz_g[1] == 2 * 8 + 4 && gd.nxyz_g[2] == 1);
    EXPECT(gd.neighbors[0][0] >= 0 && gd.neighbors[0][1] >= 0);
    EXPECT(grid_coord(gd, 1, 0, 0.5, 12) >= 0.0);
    EXPECT(throws([&] { make_grid_desc(20, 12, 1, nullptr, per, ol, hw, 8, 8); }));  // rank
    EXPECT(throws([&] { make_grid_desc(5, 12, 1, nullptr, per, ol, hw, 2, 0); }));   // n < ol+hw
    const int bad_hw[3] = {3, 2, 1};
    EXPECT(throws([&] { make_grid_desc(20, 12, 1, nullptr, per, ol, bad_hw, 2, 0); }));
    const int per_z[3] = {0, 0, 1};
    EXPECT(throws([&] { make_grid_desc(20, 12, 1, nullptr, per_z, ol, hw, 2, 0); }));
    const int dims_bad[3] = {3, 0, 1};
    EXPECT(throws([&] { make_grid_desc(20, 12, 1, dims_bad, per, ol, hw, 8, 0); }));
  }
  // parallel_for: an exception on a worker (or the caller) reaches the caller
  {
    bool caught = false;
    try {
      parallel_for(0, 1 << 16, 1, [](int64_t i) {
        if (i == 40000) throw std::runtime_error("boom");
      });
    } catch (const std::runtime_error&) {
      caught = true;
    }
    EXPECT(caught);
    std::vector<int> hit(1 << 12, 0);
    parallel_for(0, 1 << 12, 1, [&](int64_t i) { hit[i] += 1; });
    for (int h : hit) EXPECT(h == 1);
  }
  std::puts("host selftest OK");
  return 0;
}
