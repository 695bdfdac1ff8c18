// Standalone native driver of the perf_hide diffusion (no Python): the
// reference scripts/diffusion_2D_perf_hide.jl's intended overlap variant,
// written against the C ABI of librma_core.so (rma/capi.h).
//
//   ./build/examples/diffusion_2D_perf_hide [nx] [nt] [mode] [K] [fast]    # 1 GPU
//   (mode 0 perf, 1 perf_hide; K = time steps per kernel pass, 1/2/3/4/6/8)
//   python -m rocm_mpi_amd.launch -n 8 ./build/examples/diffusion_2D_perf_hide 16384 1000
//
// Ranks come from RANK / WORLD_SIZE / LOCAL_RANK (torchrun or our launcher);
// rank 0 writes the RCCL unique id to $RMA_UID_FILE (default
// /tmp/rma_uid_<MASTER_PORT>) and the others read it: an MPI-free bootstrap.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <thread>

#include "rma/capi.h"

#define CK(x)                                                                     \
  do {                                                                            \
    if ((x) != 0) {                                                               \
      std::fprintf(stderr, "%s failed: %s\n", #x, rma_last_error());              \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)
#define HK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));         \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

static int env_int(const char* n, int d) {
  const char* v = std::getenv(n);
  return v ? std::atoi(v) : d;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 16384;
  const int nt = argc > 2 ? std::atoi(argv[2]) : 1000;
  const int mode = argc > 3 ? std::atoi(argv[3]) : 1;  // 0 perf, 1 perf_hide
  const int K = argc > 4 ? std::atoi(argv[4]) : 1;     // steps per kernel pass
  const int fast = argc > 5 ? std::atoi(argv[5]) : 0;  // 1: fast-math K-step passes
  const int rank = env_int("RANK", 0), size = env_int("WORLD_SIZE", 1);
  const int local = env_int("LOCAL_RANK", rank);
  int ndev = 0;
  HK(hipGetDeviceCount(&ndev));
  const int dev = local % std::max(ndev, 1);
  HK(hipSetDevice(dev));

  char uid[128] = {0};
  if (size > 1) {
    std::string path = std::getenv("RMA_UID_FILE") ? std::getenv("RMA_UID_FILE")
                                                   : "/tmp/rma_uid_" +
                                                         std::string(std::getenv("MASTER_PORT")
                                                                         ? std::getenv("MASTER_PORT")
                                                                         : "0");
    if (rank == 0) {
      CK(rma_unique_id(uid));
      std::ofstream(path + ".tmp", std::ios::binary).write(uid, 128);
      std::rename((path + ".tmp").c_str(), path.c_str());
    } else {
      for (int i = 0;; ++i) {
        std::ifstream f(path, std::ios::binary);
        if (f && f.read(uid, 128)) break;
        if (i > 6000) {
          std::fprintf(stderr, "rank %d: no unique id at %s\n", rank, path.c_str());
          return 1;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
      }
    }
  }
  rma_grid* g = nullptr;
  int me = 0, dims[3], coords[3];
  const int dims_in[3] = {0, 0, 1};
  // temporal blocking: at most K steps per kernel pass (the executor plans the
  // passes) need overlap 2K and halo width K
  const int ol[3] = {2 * std::max(1, K), 2 * std::max(1, K), 2};
  const int hw[3] = {std::max(1, K), std::max(1, K), 1};
  CK(rma_init_global_grid((int)n, (int)n, 1, dims_in, nullptr, ol, hw, size, rank,
                          size > 1 ? uid : nullptr, dev, &g, &me, dims, coords));
  const double lx = 10, ly = 10, lam = 1, Cp0 = 1;
  const double dx = lx / rma_nx_g(g), dy = ly / rma_ny_g(g);
  const double dt = std::min(dx * dx, dy * dy) * Cp0 / lam / 4.1;
  const double coef[4] = {-lam, 1 / dx, 1 / dy, dt};
  double *T, *T2, *iCp;
  const size_t bytes = (size_t)n * n * sizeof(double);
  HK(hipMalloc(&T, bytes));
  HK(hipMalloc(&T2, bytes));
  HK(hipMalloc(&iCp, bytes));
  hipStream_t s;
  HK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(rma_fill(iCp, n * n, 1.0 / Cp0, s));
  CK(rma_init_gaussian(g, T, n, n, dx, dy, lx, ly, s));
  HK(hipMemcpyAsync(T2, T, bytes, hipMemcpyDeviceToDevice, s));
  rma_executor* ex = nullptr;
  CK(rma_executor_create_kf(g, mode, T, T2, iCp, n, n, coef, 1, 1, K, fast, nullptr, nullptr,
                            nullptr, &ex));
  if (me == 0)
    std::printf("Global grid: %ldx%ldx1 (nprocs: %d, dims: %dx%dx%d)\n", (long)rma_nx_g(g),
                (long)rma_ny_g(g), size, dims[0], dims[1], dims[2]);
  CK(rma_executor_run(ex, 10, s));  // the reference's 10 untimed iterations
  CK(rma_tic(g, s));
  CK(rma_executor_run(ex, nt - 10, s));
  double wtime = 0;
  CK(rma_toc(g, s, &wtime));
  const double A_eff = 3.0 / 1e9 * n * n * sizeof(double);
  const double T_eff = A_eff / (wtime / (nt - 10));
  // peak of the field on this rank (host copy of one column through the centre suffices)
  if (me == 0)
    std::printf("Executed %d steps in = %1.3e sec (@ T_eff = %1.2f GB/s) \n", nt, wtime, T_eff);
  CK(rma_executor_destroy(ex));
  HK(hipFree(T));
  HK(hipFree(T2));
  HK(hipFree(iCp));
  HK(hipStreamDestroy(s));
  CK(rma_finalize_global_grid(g));
  return 0;
}
