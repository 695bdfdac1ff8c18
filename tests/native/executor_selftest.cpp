// The native time loop (csrc/runtime/executor.cpp DiffusionExecutor) on P rank
// threads over the loopback transport, against a host stand-in of the HIP
// runtime (tests/native/hip_stub) with the kernels replaced by their CPU
// twins, so it builds with a host compiler under ThreadSanitizer and
// AddressSanitizer (tests/test_native_host_threads.py).
//
// Each case decomposes one global grid over dims[0] x dims[1] rank threads
// (open or periodic), runs n steps of perf or perf_hide with K-step passes
// (canonical K = 1; fast-math K = 4, 8, 24: split frame / interior launches and
// the frame-first fused pass, whose frame flag the stub raises when the launch
// "completes") and requires every tile to equal its window of the same grid
// run by ONE rank, bitwise: the executor's pass plan, frame / interior
// geometry, stream / event ordering and exchanges, with the sanitizers
// watching the threads meet in the loopback hub. Reference:
// /root/reference/scripts/diffusion_2D_perf_hide.jl:63-101 (the overlapped
// time loop this executor implements), diffusion_2D_perf.jl:22-58.
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>  // the host stub

#include "rma/executor.h"
#include "rma/halo.h"
#include "rma/kernels.h"
#include "rma/loopback.h"
#include "rma/topology.h"

namespace rma {
// the stub runs stream work at enqueue time: every launch is its CPU twin
void copy2d_batch_gpu(const Copy2d* copies, int n, int elem_bytes, stream_t) {
  copy2d_batch_cpu(copies, n, elem_bytes);
}
void flag_wait_gpu(const uint64_t* flag, uint64_t want, double timeout_s, uint32_t* err,
                   uint32_t code, stream_t) {
  auto* f = reinterpret_cast<const std::atomic<uint64_t>*>(flag);
  const auto t0 = std::chrono::steady_clock::now();
  while (f->load(std::memory_order_acquire) != want) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
      __atomic_store_n(err, code, __ATOMIC_RELEASE);
      return;
    }
    std::this_thread::yield();
  }
}
void flag_write_gpu(uint64_t* flag, uint64_t value, stream_t) {
  reinterpret_cast<std::atomic<uint64_t>*>(flag)->store(value, std::memory_order_release);
}
std::atomic<long> g_signals{0};
std::atomic<long> g_direct_launches{0};
void flags_wait_ge_gpu(const uint64_t* flags, uint32_t mask, uint64_t want, double timeout_s,
                       uint32_t* err, uint32_t code, stream_t) {
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 8; ++i) {
    if (!((mask >> i) & 1u)) continue;
    auto* f = reinterpret_cast<const std::atomic<uint64_t>*>(flags + i);
    while (f->load(std::memory_order_acquire) < want) {
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
        __atomic_store_n(err, code, __ATOMIC_RELEASE);
        return;
      }
      std::this_thread::yield();
    }
  }
}
void flags_write_gpu(const FlagTargets& t, uint64_t value, stream_t) {
  for (uint64_t* p : t.dst)
    if (p) reinterpret_cast<std::atomic<uint64_t>*>(p)->store(value, std::memory_order_release);
}
void stencil_rects_gpu(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                       const Rect* rects, int nrects, const StencilCoef& c, const StencilTuning& t,
                       stream_t) {
  if (t.signal) throw std::runtime_error("a signalling one-step launch (fused one-step passes "
                                         "were removed)");
  stencil_rects_cpu(T2, T, iCp, nx, ny, rects, nrects, c);
}
void stencil2_rects_gpu(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                        const Rect* rects, int nrects, const StencilCoef& c, const StencilTuning&,
                        stream_t) {
  stencil2_rects_cpu(T2, T, iCp, nx, ny, rects, nrects, c);
}
void stencilk_rects_gpu(int K, double* T2, const double* T, const double* iCp, int64_t nx,
                        int64_t ny, const Rect* rects, int nrects, const StencilCoef& c,
                        const StencilTuning& t, stream_t) {
  // fast5 family: kernel 5 and the pipelined kernels except 10 (canonical)
  const bool fast = t.kernel == 5 || (t.kernel >= 9 && t.kernel != 10);
  // like the GPU kernel, read only the cells the rects depend on (each rect
  // grown by K, clamped to the tile): the CPU twin on that box, whose own
  // edge cells stay fixed over the K levels, gives the rect cells bitwise (the
  // dependency cone of K levels ends K cells out). Reading the whole tile
  // would race with a neighbour's direct stores into halos no launch reads.
  for (int i = 0; i < nrects; ++i) {
    const Rect& r = rects[i];
    if (r.empty()) continue;
    const int64_t bx0 = std::max<int64_t>(0, r.x0 - K), bx1 = std::min<int64_t>(nx, r.x1 + K);
    const int64_t by0 = std::max<int64_t>(0, r.y0 - K), by1 = std::min<int64_t>(ny, r.y1 + K);
    const int64_t bw = bx1 - bx0, bh = by1 - by0;
    std::vector<double> a((size_t)(bw * bh)), ic((size_t)(bw * bh)), o((size_t)(bw * bh));
    for (int64_t y = 0; y < bh; ++y)
      for (int64_t x = 0; x < bw; ++x) {
        a[(size_t)(y * bw + x)] = T[(by0 + y) * nx + bx0 + x];
        ic[(size_t)(y * bw + x)] = iCp[(by0 + y) * nx + bx0 + x];
      }
    const Rect lr{r.x0 - bx0, r.x1 - bx0, r.y0 - by0, r.y1 - by0};
    if (fast)
      stencilk5_rects_cpu(K, o.data(), a.data(), ic.data(), bw, bh, &lr, 1, c);
    else
      stencilk_rects_cpu(K, o.data(), a.data(), ic.data(), bw, bh, &lr, 1, c);
    for (int64_t y = r.y0; y < r.y1; ++y)
      for (int64_t x = r.x0; x < r.x1; ++x) T2[y * nx + x] = o[(size_t)((y - by0) * bw + x - bx0)];
  }
  if (t.direct) {  // direct-store halos: the launched cells' images into the peers' fields
    if (t.kernel < 9) throw std::runtime_error("direct stores on a non-pipelined kernel");
    const DirectStores& D = *t.direct;
    auto in = [](int64_t a, int s, int64_t m0, int64_t m1, int64_t p0, int64_t p1) {
      return s == 0 || (s < 0 ? a >= m0 && a < m1 : a >= p0 && a < p1);
    };
    for (int d = 0; d < 8; ++d) {
      if (!D.dst[d]) continue;
      const int di = DiffusionExecutor::kDirI[d], dj = DiffusionExecutor::kDirJ[d];
      const int64_t off = -di * D.sx - dj * D.syr * nx;
      for (int i = 0; i < nrects; ++i) {
        const Rect& r = rects[i];
        for (int64_t y = r.y0; y < r.y1; ++y) {
          if (!in(y, dj, D.ym0, D.ym1, D.yp0, D.yp1)) continue;
          for (int64_t x = r.x0; x < r.x1; ++x)
            if (in(x, di, D.xm0, D.xm1, D.xp0, D.xp1)) D.dst[d][y * nx + x + off] = T2[y * nx + x];
        }
      }
    }
    ++g_direct_launches;
  }
  if (t.signal) {  // the launch's frame blocks are done: raise the flag (stencil_device.h)
    if (t.kernel < 9) throw std::runtime_error("signal on a non-pipelined kernel");
    reinterpret_cast<std::atomic<uint64_t>*>(t.signal + 1)->store(1, std::memory_order_release);
    ++g_signals;
  }
}
// the direct-store kernel variants' occupancy (set_direct's planner pricing):
// depth 20 at half the plain kernel's, as the register-capped GPU build
void stencil_pipe_occupancy(int K, int, int, int, int occ[2]) {
  occ[0] = 2;
  occ[1] = K == 20 ? 1 : 2;
}
void flux_gpu(double* QX, double* QY, const double* T, int64_t nx, int64_t ny, double mlam,
              double rdx, double rdy, stream_t) {
  flux_cpu(QX, QY, T, nx, ny, mlam, rdx, rdy);
}
void residual_gpu(double* D, const double* QX, const double* QY, const double* iCp, int64_t nx,
                  int64_t ny, double rdx, double rdy, stream_t) {
  residual_cpu(D, QX, QY, iCp, nx, ny, rdx, rdy);
}
void update_gpu(double* T, const double* D, int64_t nx, int64_t ny, double dt, stream_t) {
  update_cpu(T, D, nx, ny, dt);
}
}  // namespace rma

using namespace rma;

// The executor's process-wide stream pool (executor.cpp g_pool) keeps its
// streams for the life of the process by design (reused by later executors,
// never destroyed during HIP teardown): not a leak to report.
extern "C" const char* __lsan_default_suppressions() {
  return "leak:hipStreamCreateWithPriority\n";
}

namespace {

std::atomic<int> g_fail{0};

#define CHECK(cond, ...)                  \
  do {                                    \
    if (!(cond)) {                        \
      std::fprintf(stderr, "FAIL: ");     \
      std::fprintf(stderr, __VA_ARGS__);  \
      std::fprintf(stderr, "\n");         \
      ++g_fail;                           \
    }                                     \
  } while (0)

uint64_t mix(uint64_t z) {  // splitmix64
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// a value keyed by the GLOBAL cell (wrapped on periodic dims): every
// decomposition of the grid sees the same field, overlaps agree
double cell_value(int64_t gx, int64_t gy, int64_t nxg, int64_t nyg, uint64_t seed, double lo,
                  double hi) {
  gx = ((gx % nxg) + nxg) % nxg;
  gy = ((gy % nyg) + nyg) % nyg;
  const uint64_t h = mix(seed ^ mix((uint64_t)(gy * nxg + gx)));
  return lo + (hi - lo) * (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

struct Case {
  const char* name;
  std::array<int, 3> dims, periods;
  int64_t nx, ny;  // per-rank tile (with overlaps)
  int K;           // max steps per pass (1: canonical one-step, > 1 fast-math)
  Mode mode;
  int nt;
  const char* fused;  // RMA_EXEC_FUSED for the multi-rank run ("" = auto)
  int chunk = 0;      // K-step rows per task (ExecParams::chunk_rows2; 0: the table)
  bool direct = false;  // direct-store halos between the rank threads (set_direct)
  bool host_wait = false;  // ...with host-side count waits (the loopback mode)
};

struct TileResult {
  std::array<int, 3> coords;
  std::vector<double> T;
  int64_t fused_passes, passes;
};

// runs the case's grid on dims[0] x dims[1] rank threads; returns every tile
std::vector<TileResult> run_ranks(const Case& c, std::array<int, 3> dims, int64_t nx, int64_t ny,
                                  bool direct = false) {
  const int P = dims[0] * dims[1] * dims[2];
  // direct-store halos: every rank's fields and pass-count words, published
  // before any rank runs (a one-shot barrier)
  std::vector<std::array<double*, 2>> fields((size_t)P);
  std::vector<std::array<uint64_t, 8>> counts((size_t)P);
  for (auto& a : counts) a.fill(0);
  std::atomic<int> published{0};
  const int64_t ol = std::max(2, 2 * c.K);
  const int64_t nxg = c.periods[0] ? dims[0] * (nx - ol) : dims[0] * (nx - ol) + ol;
  const int64_t nyg = c.periods[1] ? dims[1] * (ny - ol) : dims[1] * (ny - ol) + ol;
  CartTopology topo(P, dims, c.periods);
  auto hub = std::make_shared<LoopbackHub>(P, 60.0);
  std::vector<TileResult> out((size_t)P);
  std::vector<std::thread> th;
  for (int r = 0; r < P; ++r) {
    th.emplace_back([&, r] {
      try {
        const auto co = topo.coords(r);
        auto ep = std::make_unique<LoopbackEndpoint>(hub, r);
        auto hx = std::make_unique<HaloExchanger>(ep.get(), r, topo.neighbors(r));
        hx->set_diagonals(topo.diagonals(r));
        const int64_t gx0 = co[0] * (nx - ol), gy0 = co[1] * (ny - ol);
        std::vector<double> T((size_t)(nx * ny)), T2((size_t)(nx * ny)), iCp((size_t)(nx * ny));
        for (int64_t y = 0; y < ny; ++y)
          for (int64_t x = 0; x < nx; ++x) {
            T[(size_t)(y * nx + x)] = cell_value(gx0 + x, gy0 + y, nxg, nyg, 11, 0.0, 1.0);
            iCp[(size_t)(y * nx + x)] = cell_value(gx0 + x, gy0 + y, nxg, nyg, 29, 0.5, 1.5);
          }
        T2 = T;
        fields[(size_t)r] = {T.data(), T2.data()};
        published.fetch_add(1, std::memory_order_acq_rel);
        while (published.load(std::memory_order_acquire) < P) std::this_thread::yield();
        ExecParams p;
        p.mode = c.mode;
        const double dx = 10.0 / (double)nxg, dy = 10.0 / (double)nyg;
        p.coef = StencilCoef{-1.0, 1.0 / dx, 1.0 / dy, std::min(dx * dx, dy * dy) / 4.1};
        p.temporal = c.K;
        p.olx = p.oly = ol;
        p.fast_math = c.K > 1 ? 1 : 0;
        p.chunk_rows2 = c.chunk;
        TileResult& res = out[(size_t)r];
        {
          DiffusionExecutor ex(T.data(), T2.data(), iCp.data(), nx, ny, p, hx.get());
          if (direct) {
            std::array<DiffusionExecutor::DirectPeer, 8> peers{};
            const auto nb = topo.neighbors(r);
            const auto dg = topo.diagonals(r);
            for (int d = 0; d < 8; ++d) {
              const int i = DiffusionExecutor::kDirI[d], j = DiffusionExecutor::kDirJ[d];
              int q = -1;
              if (j == 0) q = nb[0][i > 0];
              else if (i == 0) q = nb[1][j > 0];
              else if (nb[0][i > 0] >= 0 && nb[1][j > 0] >= 0) q = dg[(j > 0) * 2 + (i > 0)];
              if (q < 0) continue;
              peers[d].rank = q;
              peers[d].T = fields[(size_t)q][0];
              peers[d].T2 = fields[(size_t)q][1];
              // the peer counts our passes in its word of direction 7 - d
              peers[d].flag = q == r ? nullptr : &counts[(size_t)q][(size_t)(7 - d)];
            }
            ex.set_direct(peers, counts[(size_t)r].data(), c.host_wait);
          }
          ex.run(c.nt, nullptr);
          (void)hipDeviceSynchronize();
          res.fused_passes = ex.fused_passes();
          res.passes = ex.passes_done();
          res.T = ex.parity() ? T2 : T;
        }
        res.coords = co;
        hx.reset();
        ep.reset();
      } catch (const std::exception& e) {
        std::fprintf(stderr, "FAILED %s rank %d: %s\n", c.name, r, e.what());
        ++g_fail;
      }
    });
  }
  for (auto& t : th) t.join();
  return out;
}

int run_case(const Case& c) {
  const int fails0 = g_fail.load();
  const int64_t ol = std::max(2, 2 * c.K);
  if (*c.fused)
    setenv("RMA_EXEC_FUSED", c.fused, 1);
  else
    unsetenv("RMA_EXEC_FUSED");
  const auto multi = run_ranks(c, c.dims, c.nx, c.ny, c.direct);
  // the same global grid on one rank: its tile is the global grid plus the
  // overlap cells (periodic: wrapped by the self exchange)
  const int64_t nx1 = c.dims[0] * (c.nx - ol) + ol, ny1 = c.dims[1] * (c.ny - ol) + ol;
  setenv("RMA_EXEC_FUSED", "0", 1);
  const auto one = run_ranks(c, {1, 1, 1}, nx1, ny1);
  unsetenv("RMA_EXEC_FUSED");
  if (g_fail.load() != fails0) return 1;
  long fused = 0;
  for (const TileResult& t : multi) {
    fused += t.fused_passes;
    const int64_t gx0 = t.coords[0] * (c.nx - ol), gy0 = t.coords[1] * (c.ny - ol);
    for (int64_t y = 0; y < c.ny; ++y)
      for (int64_t x = 0; x < c.nx; ++x) {
        const double a = t.T[(size_t)(y * c.nx + x)];
        const double b = one[0].T[(size_t)((gy0 + y) * nx1 + gx0 + x)];
        if (std::memcmp(&a, &b, sizeof a) != 0) {
          CHECK(false, "%s: tile (%d,%d) cell (%lld,%lld) %.17g != %.17g", c.name, t.coords[0],
                t.coords[1], (long long)x, (long long)y, a, b);
          return 1;
        }
      }
  }
  const bool want_fused = std::string(c.fused) == "1" && !c.direct;
  CHECK(!want_fused || fused > 0, "%s: no fused pass ran", c.name);
  CHECK(std::string(c.fused) != "0" || fused == 0, "%s: fused passes with RMA_EXEC_FUSED=0",
        c.name);
  std::printf("%s OK (%zu ranks, %lld passes on rank 0, %ld fused)\n", c.name, multi.size(),
              (long long)multi[0].passes, fused);
  return g_fail.load() != fails0;
}

}  // namespace

int main() {
  const Case cases[] = {
      {"perf_hide K=1 2x2 open", {2, 2, 1}, {0, 0, 0}, 40, 36, 1, Mode::kHide, 13, ""},
      {"perf K=1 3x1 periodic-x", {3, 1, 1}, {1, 0, 0}, 30, 28, 1, Mode::kPerf, 11, ""},
      {"perf_hide K=1 2x2 periodic", {2, 2, 1}, {1, 1, 0}, 40, 36, 1, Mode::kHide, 13, ""},
      {"perf_hide K=4 2x2 periodic", {2, 2, 1}, {1, 1, 0}, 48, 44, 4, Mode::kHide, 19, ""},
      {"perf_hide K=8 2x1 split", {2, 1, 1}, {0, 0, 0}, 800, 120, 8, Mode::kHide, 21, "0"},
      {"perf_hide K=8 2x1 fused", {2, 1, 1}, {0, 0, 0}, 800, 120, 8, Mode::kHide, 21, "1"},
      {"perf_hide K=8 2x2 fused", {2, 2, 1}, {0, 1, 0}, 760, 400, 8, Mode::kHide, 17, "1"},
      // 64-row tasks: the table's 16 rows at this height are shorter than the
      // 2K - 1 rows an aligned band must hold, so the frame would not be aligned
      {"perf_hide K=24 2x1 fused", {2, 1, 1}, {0, 0, 0}, 700, 400, 24, Mode::kHide, 50, "1", 64},
      {"perf_hide K=24 2x2 auto", {2, 2, 1}, {1, 1, 0}, 700, 400, 24, Mode::kHide, 48, "", 64},
      {"perf K=8 1x2 periodic-y", {1, 2, 1}, {0, 1, 0}, 64, 60, 8, Mode::kPerf, 17, ""},
      // direct-store halos (set_direct): the neighbours' halos stored by the
      // frame tasks, pass counts instead of the exchange; split and fused passes
      {"direct perf_hide K=8 2x2 open split", {2, 2, 1}, {0, 0, 0}, 760, 400, 8, Mode::kHide, 17,
       "0", 0, true},
      {"direct perf_hide K=8 2x2 periodic fused", {2, 2, 1}, {1, 1, 0}, 760, 400, 8, Mode::kHide,
       19, "1", 0, true},
      {"direct perf_hide K=24 3x1 periodic-x", {3, 1, 1}, {1, 0, 0}, 700, 400, 24, Mode::kHide, 50,
       "", 64, true},
      {"direct perf K=4 2x2 periodic-y", {2, 2, 1}, {0, 1, 0}, 64, 60, 4, Mode::kPerf, 13, "",
       0, true},
      {"direct perf_hide K=6 1x1 periodic self", {1, 1, 1}, {1, 1, 0}, 90, 70, 6, Mode::kHide, 25,
       "", 0, true},
      // the same with the host waiting for the counts (ranks of one process)
      {"direct host-wait perf_hide K=8 2x2 open split", {2, 2, 1}, {0, 0, 0}, 760, 400, 8,
       Mode::kHide, 17, "0", 0, true, true},
      {"direct host-wait perf_hide K=8 2x2 periodic fused", {2, 2, 1}, {1, 1, 0}, 760, 400, 8,
       Mode::kHide, 19, "1", 0, true, true},
      {"direct host-wait perf K=4 2x2 periodic-y", {2, 2, 1}, {0, 1, 0}, 64, 60, 4, Mode::kPerf,
       13, "", 0, true, true},
  };
  for (const Case& c : cases)
    if (run_case(c)) return 1;
  // random fused-pass geometries (fixed seed): dims, periods, depth, rows per
  // task, steps; tiles wide and tall enough for aligned frames
  std::mt19937 rng(20251018u);
  static std::vector<std::string> names;
  names.reserve(8);
  for (int i = 0; i < 6; ++i) {
    const std::array<int, 3> dimsets[4] = {{2, 1, 1}, {1, 2, 1}, {2, 2, 1}, {3, 1, 1}};
    Case c{};
    c.dims = dimsets[rng() % 4];
    c.periods = {(int)(rng() % 2), (int)(rng() % 2), 0};
    c.K = 8 + (int)(rng() % 17);                          // 8..24
    c.nx = 3 * (256 - 2 * c.K) + 2 * c.K + 8 + (int64_t)(rng() % 64);
    c.chunk = 32 + 16 * (int)(rng() % 3);                 // 32, 48, 64
    c.ny = 3 * c.chunk + 4 * c.K + (int64_t)(rng() % 80);
    c.mode = Mode::kHide;
    c.nt = c.K + 1 + (int)(rng() % (2 * c.K));
    c.fused = "1";
    names.push_back("random fused " + std::to_string(i) + " dims " + std::to_string(c.dims[0]) +
                    "x" + std::to_string(c.dims[1]) + " per " + std::to_string(c.periods[0]) +
                    std::to_string(c.periods[1]) + " K=" + std::to_string(c.K) + " tile " +
                    std::to_string(c.nx) + "x" + std::to_string(c.ny) + " rows " +
                    std::to_string(c.chunk) + " nt " + std::to_string(c.nt));
    c.name = names.back().c_str();
    if (run_case(c)) return 1;
  }
  std::printf("frame flags raised %ld, direct-store launches %ld\n", g_signals.load(),
              g_direct_launches.load());
  CHECK(rma_stub::live_events() == 0, "events leaked: %ld", rma_stub::live_events().load());
  if (g_fail.load()) return 1;
  std::printf("executor selftest OK\n");
  return 0;
}
