// C ABI implementation (see rma/capi.h).
#include "rma/capi.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstring>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "rma/comm.h"
#include "rma/executor.h"
#include "rma/halo.h"
#include "rma/hip_check.h"
#include "rma/kernels.h"
#include "rma/topology.h"

struct rma_grid : rma::GridDesc {  // host part: topology.cpp make_grid_desc
  int device = 0;
  std::unique_ptr<rma::CartTopology> topo;
  std::unique_ptr<rma::RcclComm> comm;
  std::unique_ptr<rma::HaloExchanger> halo;
  std::chrono::steady_clock::time_point t0;
  // executors hold raw pointers to `halo`: they pin the grid. finalize with
  // executors alive defers the teardown to the last rma_executor_destroy (a
  // GC'd host such as the Julia shim may finalize objects in any order), and
  // rma_grid_self_via_rccl refuses to swap the exchanger under them.
  int live_executors = 0;
  bool finalized = false;
};

namespace {
thread_local std::string g_err;

template <typename F>
int guard(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return 1;
  }
}

double coord(const rma_grid* g, int d, int64_t ix, double dd, int64_t size_A) {
  return rma::grid_coord(*g, d, ix, dd, size_A);
}
}  // namespace

extern "C" {

const char* rma_last_error(void) { return g_err.c_str(); }

int rma_unique_id(char out[128]) {
  return guard([&] {
    const std::string id = rma::RcclComm::unique_id();
    RMA_CHECK_ARG(id.size() <= 128, "unique id too large");
    std::memset(out, 0, 128);
    std::memcpy(out, id.data(), id.size());
  });
}

int rma_init_global_grid(int nx, int ny, int nz, const int dims[3], const int periods[3],
                         const int overlaps[3], const int halowidths[3], int nprocs, int rank,
                         const char* unique_id, int device, rma_grid** out_grid, int* out_me,
                         int out_dims[3], int out_coords[3]) {
  return guard([&] {
    RMA_CHECK_ARG(out_grid != nullptr, "out_grid is NULL");
    auto g = std::make_unique<rma_grid>();
    static_cast<rma::GridDesc&>(*g) =
        rma::make_grid_desc(nx, ny, nz, dims, periods, overlaps, halowidths, nprocs, rank);
    g->device = device;
    g->topo = std::make_unique<rma::CartTopology>(nprocs, g->dims, g->periods);
    RMA_HIP_CHECK(hipSetDevice(device));
    if (nprocs > 1) {
      RMA_CHECK_ARG(unique_id != nullptr, "unique_id required when nprocs > 1");
      // non-blocking init with a timeout (RMA_COMM_TIMEOUT s, default 300)
      // unless RMA_RCCL_BLOCKING=1
      const char* tb = std::getenv("RMA_RCCL_BLOCKING");
      const char* to = std::getenv("RMA_COMM_TIMEOUT");
      const double init_timeout = (tb && tb[0] == '1') ? 0.0 : (to ? std::atof(to) : 300.0);
      g->comm = std::make_unique<rma::RcclComm>(nprocs, rank, std::string(unique_id, 128), device,
                                                init_timeout);
    }
    rma::set_rank_for_errors(rank);
    g->halo = std::make_unique<rma::HaloExchanger>(g->comm.get(), rank, g->topo->neighbors(rank));
    g->halo->set_diagonals(g->topo->diagonals(rank));
    if (out_me) *out_me = rank;
    for (int d = 0; d < 3; ++d) {
      if (out_dims) out_dims[d] = g->dims[d];
      if (out_coords) out_coords[d] = g->coords[d];
    }
    *out_grid = g.release();
  });
}

namespace {
void destroy_grid(rma_grid* g) {
  g->halo.reset();
  g->comm.reset();
  delete g;
}
}  // namespace

int rma_finalize_global_grid(rma_grid* g) {
  return guard([&] {
    if (!g) return;
    RMA_CHECK_ARG(!g->finalized, "grid finalized twice");
    g->finalized = true;
    if (g->live_executors == 0) destroy_grid(g);
  });
}

int64_t rma_nx_g(const rma_grid* g) { return g->nxyz_g[0]; }
int64_t rma_ny_g(const rma_grid* g) { return g->nxyz_g[1]; }
int64_t rma_nz_g(const rma_grid* g) { return g->nxyz_g[2]; }
double rma_x_g(const rma_grid* g, int64_t ix, double dx, int64_t s) { return coord(g, 0, ix, dx, s); }
double rma_y_g(const rma_grid* g, int64_t iy, double dy, int64_t s) { return coord(g, 1, iy, dy, s); }
double rma_z_g(const rma_grid* g, int64_t iz, double dz, int64_t s) { return coord(g, 2, iz, dz, s); }

int rma_neighbors(const rma_grid* g, int out[6]) {
  return guard([&] {
    const auto nb = g->topo->neighbors(g->me);
    for (int d = 0; d < 3; ++d) {
      out[2 * d] = nb[d][0];
      out[2 * d + 1] = nb[d][1];
    }
  });
}

int rma_update_halo(rma_grid* g, int nfields, void* const* fields, const int64_t* sizes,
                    const int* elem_bytes, void* stream) {
  return guard([&] {
    std::vector<rma::HaloField> fs;
    for (int i = 0; i < nfields; ++i) {
      rma::HaloField f;
      f.ptr = fields[i];
      f.elem_bytes = elem_bytes ? elem_bytes[i] : 8;
      for (int d = 0; d < 3; ++d) {
        f.size[d] = sizes[3 * i + d];
        // staggered arrays: overlap of this array = ol + (size(A) - n)
        f.ol[d] = g->overlaps[d] + (f.size[d] - g->nxyz[d]);
        f.hw[d] = g->hw[d];
      }
      fs.push_back(f);
    }
    g->halo->exchange(fs, stream, 7);
  });
}

int rma_gather(rma_grid* g, const void* sendbuf, void* recvbuf, size_t bytes, int root,
               void* stream) {
  return guard([&] {
    if (g->comm) {
      g->comm->gather(sendbuf, recvbuf, bytes, root, stream);
    } else {
      RMA_HIP_CHECK(hipMemcpyAsync(recvbuf, sendbuf, bytes, hipMemcpyDefault,
                                   rma::as_stream(stream)));
    }
  });
}

int rma_tic(rma_grid* g, void* stream) {
  return guard([&] {
    if (g->comm)
      g->comm->barrier(stream, 300.0);
    else
      RMA_HIP_CHECK(hipStreamSynchronize(rma::as_stream(stream)));
    g->t0 = std::chrono::steady_clock::now();
  });
}

int rma_toc(rma_grid* g, void* stream, double* seconds) {
  return guard([&] {
    if (g->comm)
      g->comm->barrier(stream, 300.0);
    else
      RMA_HIP_CHECK(hipStreamSynchronize(rma::as_stream(stream)));
    *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - g->t0).count();
  });
}

int rma_diffusion_step(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                       const double coef[4], void* stream) {
  return guard([&] {
    const rma::Rect r{1, nx - 1, 1, ny - 1};
    const rma::StencilCoef c{coef[0], coef[1], coef[2], coef[3]};
    rma::stencil_rects_gpu(T2, T, iCp, nx, ny, &r, 1, c, rma::StencilTuning{}, stream);
  });
}

namespace {
rma::TileGeom geom(const rma_grid* g, int64_t nx, int64_t ny, double dx, double dy) {
  rma::TileGeom t;
  t.gx0 = (int64_t)g->coords[0] * (g->nxyz[0] - g->overlaps[0]);
  t.gy0 = (int64_t)g->coords[1] * (g->nxyz[1] - g->overlaps[1]);
  t.nxg = g->nxyz_g[0];
  t.nyg = g->nxyz_g[1];
  t.dx = dx;
  t.dy = dy;
  t.xoff = 0.5 * (double)(g->nxyz[0] - nx) * dx;
  t.yoff = 0.5 * (double)(g->nxyz[1] - ny) * dy;
  t.periodx = g->periods[0];
  t.periody = g->periods[1];
  return t;
}
}  // namespace

struct rma_executor {
  std::unique_ptr<rma::DiffusionExecutor> ex;
  rma_grid* grid = nullptr;  // pinned: live_executors counts this executor
};

int rma_init_gaussian(rma_grid* g, double* T, int64_t nx, int64_t ny, double dx, double dy,
                      double lx, double ly, void* stream) {
  return guard([&] { rma::init_gaussian_gpu(T, nx, ny, geom(g, nx, ny, dx, dy), lx, ly, stream); });
}

int rma_init_random(rma_grid* g, double* A, int64_t nx, int64_t ny, double dx, double dy,
                    uint64_t seed, void* stream) {
  return guard(
      [&] { rma::init_random_gpu(A, nx, ny, geom(g, nx, ny, dx, dy), seed, 0.0, 1.0, stream); });
}

int rma_fill(double* A, int64_t n, double value, void* stream) {
  return guard([&] { rma::fill_gpu(A, n, value, stream); });
}

int rma_executor_create_k(rma_grid* g, int mode, double* T, double* T2, const double* iCp,
                          int64_t nx, int64_t ny, const double coef[4], int64_t bwx, int64_t bwy,
                          int steps_per_pass, double* qx, double* qy, double* dTdt,
                          rma_executor** out) {
  return rma_executor_create_kf(g, mode, T, T2, iCp, nx, ny, coef, bwx, bwy, steps_per_pass, 0,
                                qx, qy, dTdt, out);
}

int rma_executor_create_kf(rma_grid* g, int mode, double* T, double* T2, const double* iCp,
                           int64_t nx, int64_t ny, const double coef[4], int64_t bwx,
                           int64_t bwy, int steps_per_pass, int fast_math, double* qx,
                           double* qy, double* dTdt, rma_executor** out) {
  return rma_executor_create_g(g, mode, T, T2, iCp, nx, ny, coef, bwx, bwy, steps_per_pass,
                               fast_math, 0, qx, qy, dTdt, out);
}

// the one place the C ABI builds ExecParams (every create_* lands here)
int rma_executor_create_g(rma_grid* g, int mode, double* T, double* T2, const double* iCp,
                          int64_t nx, int64_t ny, const double coef[4], int64_t bwx, int64_t bwy,
                          int steps_per_pass, int fast_math, int graph_steps, double* qx,
                          double* qy, double* dTdt, rma_executor** out) {
  return guard([&] {
    RMA_CHECK_ARG(g && out && mode >= 0 && mode <= 2, "bad executor arguments");
    RMA_CHECK_ARG(!g->finalized, "grid already finalized");
    RMA_CHECK_ARG(mode != 2 || (qx && qy && dTdt),
                  "kp mode (2) needs the qx, qy and dTdt device buffers");
    rma::ExecParams p;
    p.mode = static_cast<rma::Mode>(mode);
    p.coef = {coef[0], coef[1], coef[2], coef[3]};
    p.bwx = bwx;
    p.bwy = bwy;
    p.temporal = steps_per_pass;
    p.olx = g->overlaps[0];
    p.oly = g->overlaps[1];
    p.tune2 = rma::default_tune_k(steps_per_pass, ny);
    p.fast_math = fast_math ? 1 : 0;
    p.use_graph = graph_steps > 0 ? 1 : 0;
    p.graph_steps = graph_steps > 0 ? graph_steps : 0;
    auto e = std::make_unique<rma_executor>();
    e->ex = std::make_unique<rma::DiffusionExecutor>(T, T2, iCp, nx, ny, p, g->halo.get(), qx, qy,
                                                     dTdt);
    e->grid = g;
    ++g->live_executors;
    *out = e.release();
  });
}

int rma_grid_self_via_rccl(rma_grid* g) {
  return guard([&] {
    RMA_CHECK_ARG(g != nullptr, "grid is NULL");
    RMA_CHECK_ARG(g->nprocs == 1, "self via RCCL is for a single-rank grid");
    // executors hold the current exchanger: replacing it would leave them a
    // dangling pointer
    RMA_CHECK_ARG(g->live_executors == 0,
                  "rma_grid_self_via_rccl: " << g->live_executors
                                             << " executor(s) still use this grid's halo exchanger; "
                                                "call it before creating executors");
    if (!g->comm) {
      const std::string uid = rma::RcclComm::unique_id();
      const char* tb = std::getenv("RMA_RCCL_BLOCKING");
      const double init_timeout = (tb && tb[0] == '1') ? 0.0 : 300.0;
      g->comm = std::make_unique<rma::RcclComm>(1, 0, uid, g->device, init_timeout);
    }
    g->halo = std::make_unique<rma::HaloExchanger>(g->comm.get(), 0, g->topo->neighbors(0));
    g->halo->set_diagonals(g->topo->diagonals(0));
    g->halo->set_self_via_transport(true);
  });
}

int rma_executor_create(rma_grid* g, int mode, double* T, double* T2, const double* iCp,
                        int64_t nx, int64_t ny, const double coef[4], int64_t bwx, int64_t bwy,
                        double* qx, double* qy, double* dTdt, rma_executor** out) {
  return rma_executor_create_k(g, mode, T, T2, iCp, nx, ny, coef, bwx, bwy, 1, qx, qy, dTdt, out);
}

int rma_executor_run(rma_executor* e, int64_t nsteps, void* stream) {
  return guard([&] { e->ex->run(nsteps, stream); });
}

int rma_executor_parity(const rma_executor* e) { return e->ex->parity(); }

int rma_executor_check(const rma_executor* e, int64_t* out_fused) {
  return guard([&] {
    if (out_fused) *out_fused = e->ex->fused_passes();
    e->ex->check_error();
  });
}

int rma_executor_destroy(rma_executor* e) {
  return guard([&] {
    if (!e) return;
    rma_grid* g = e->grid;
    delete e;
    if (g && --g->live_executors == 0 && g->finalized) destroy_grid(g);
  });
}

}  // extern "C"
