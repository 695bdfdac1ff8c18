/* C ABI of the native core — ImplicitGlobalGrid-compatible names.
 *
 * For non-Python hosts (a Julia `ccall` shim: julia/ImplicitGlobalGridMI355X.jl,
 * C/C++/Fortran drivers: examples/diffusion_2D_perf_hide.cpp). Mirrors the IGG
 * calls the reference scripts make: init_global_grid,
 * update_halo!, gather!, nx_g/ny_g, x_g/y_g, tic/toc, finalize_global_grid.
 *
 * Bootstrap is the caller's: rank 0 calls rma_unique_id() and the 128 bytes
 * reach every rank by whatever the host uses (MPI.Bcast in Julia, a file, a
 * TCP store); world size 1 needs no id (pass NULL).
 * All functions return 0 on success, non-zero on error; rma_last_error()
 * gives the message (thread-local). Device pointers / streams are opaque.
 */
#ifndef RMA_CAPI_H
#define RMA_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rma_grid rma_grid;

const char* rma_last_error(void);
int rma_unique_id(char out[128]);

/* nxyz: local sizes (halo incl.); dims: 0 = let Dims_create choose; periods;
 * overlaps (default 2) and halowidths (default 1) per dim. out_* may be NULL. */
int rma_init_global_grid(int nx, int ny, int nz, const int dims[3], const int periods[3],
                         const int overlaps[3], const int halowidths[3], int nprocs, int rank,
                         const char* unique_id, int device, rma_grid** out_grid, int* out_me,
                         int out_dims[3], int out_coords[3]);
/* Executors created on a grid pin it: with executors still alive the teardown
 * is deferred to the last rma_executor_destroy (any order is safe). */
int rma_finalize_global_grid(rma_grid* g);

int64_t rma_nx_g(const rma_grid* g);
int64_t rma_ny_g(const rma_grid* g);
int64_t rma_nz_g(const rma_grid* g);
/* global coordinate of 0-based local index ix of an array of extent size_A (IGG x_g(ix+1,...)) */
double rma_x_g(const rma_grid* g, int64_t ix, double dx, int64_t size_A);
double rma_y_g(const rma_grid* g, int64_t iy, double dy, int64_t size_A);
double rma_z_g(const rma_grid* g, int64_t iz, double dz, int64_t size_A);
int rma_neighbors(const rma_grid* g, int out[6]);

/* update_halo!: nfields device arrays, sizes[3*i..] = (nx_A, ny_A, nz_A) with x
 * fastest; elem_bytes per field. Enqueued on `stream` (asynchronous). */
int rma_update_halo(rma_grid* g, int nfields, void* const* fields, const int64_t* sizes,
                    const int* elem_bytes, void* stream);
/* gather!: root receives nprocs*bytes (rank-major) from every rank's buffer. */
int rma_gather(rma_grid* g, const void* sendbuf, void* recvbuf, size_t bytes, int root,
               void* stream);
/* barrier-synchronised timers */
int rma_tic(rma_grid* g, void* stream);
int rma_toc(rma_grid* g, void* stream, double* seconds);

/* the fused 5-point diffusion step of the reference (perf.jl) on one tile:
 * T2[interior] = f(T, iCp); coef = {-lam, 1/dx, 1/dy, dt}. */
int rma_diffusion_step(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                       const double coef[4], void* stream);

/* device-side initial conditions of a local tile of the global grid */
int rma_init_gaussian(rma_grid* g, double* T, int64_t nx, int64_t ny, double dx, double dy,
                      double lx, double ly, void* stream);
int rma_init_random(rma_grid* g, double* A, int64_t nx, int64_t ny, double dx, double dy,
                    uint64_t seed, void* stream);
int rma_fill(double* A, int64_t n, double value, void* stream);

/* native time-loop executor: mode 0 = perf (fused), 1 = perf_hide (boundary on a
 * high-priority stream + halo exchange overlapped with the interior), 2 = kp
 * (needs qx, qy, dTdt). Enqueues n steps after the work on `stream`. */
typedef struct rma_executor rma_executor;
int rma_executor_create(rma_grid* g, int mode, double* T, double* T2, const double* iCp,
                        int64_t nx, int64_t ny, const double coef[4], int64_t bwx, int64_t bwy,
                        double* qx, double* qy, double* dTdt, rma_executor** out);
// Same with temporal blocking: at most `steps_per_pass` (1..24) time steps per
// kernel pass (rma_executor_run plans passes of 1..steps_per_pass steps) (needs a grid created with overlaps >= 2*steps_per_pass and
// halowidths = steps_per_pass along every dimension with a neighbour).
int rma_executor_create_k(rma_grid* g, int mode, double* T, double* T2, const double* iCp,
                          int64_t nx, int64_t ny, const double coef[4], int64_t bwx, int64_t bwy,
                          int steps_per_pass, double* qx, double* qy, double* dTdt,
                          rma_executor** out);
// Same with `fast_math` != 0: every pass uses the 5-point-sum arithmetic (5 fp64
// operations per cell update instead of 14; rounding-level, not bitwise, equal to
// the canonical update; the bench default). Both arithmetics run any depth 1..24.
int rma_executor_create_kf(rma_grid* g, int mode, double* T, double* T2, const double* iCp,
                           int64_t nx, int64_t ny, const double coef[4], int64_t bwx,
                           int64_t bwy, int steps_per_pass, int fast_math, double* qx,
                           double* qy, double* dTdt, rma_executor** out);
// Same with `graph_steps` > 0: steps are replayed from a hipGraph capturing
// `graph_steps` steps (the host enqueue cost of a step drops to a graph launch);
// needs a capturable halo transport (RCCL: RMA_DIAG=rccl_graph, see README).
int rma_executor_create_g(rma_grid* g, int mode, double* T, double* T2, const double* iCp,
                          int64_t nx, int64_t ny, const double coef[4], int64_t bwx, int64_t bwy,
                          int steps_per_pass, int fast_math, int graph_steps, double* qx,
                          double* qy, double* dTdt, rma_executor** out);
/* Single-rank grid: route the periodic self-neighbours through a 1-rank RCCL
 * communicator (send/recv to itself) instead of local copies -- the GPU-direct
 * P2P path on one GPU (tests, probes). Call before creating executors: it
 * fails while an executor of this grid is alive. */
int rma_grid_self_via_rccl(rma_grid* g);
int rma_executor_run(rma_executor* e, int64_t nsteps, void* stream);
int rma_executor_parity(const rma_executor* e);
/* After the caller synchronised: nonzero (with rma_last_error) if a
 * frame-first fused pass's bounded wait for its frame flag timed out (the
 * halos of that pass are wrong); also reported by the next rma_executor_run.
 * out_fused (may be NULL): passes run as fused launches so far. */
int rma_executor_check(const rma_executor* e, int64_t* out_fused);
int rma_executor_destroy(rma_executor* e);

#ifdef __cplusplus
}
#endif
#endif
