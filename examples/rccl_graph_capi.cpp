// The framework's RCCL halo path under hipGraph capture WITHOUT torch: the C
// ABI of librma_core.so on /opt/rocm's HIP runtime and RCCL. A periodic
// single-rank perf_hide tile whose halo planes go through RCCL send/recv to
// itself (rma_grid_self_via_rccl), run eagerly and from hipGraph replays
// (rma_executor_create_g); the two fields must be bitwise equal. In a torch
// process (torch's bundled HIP 7.0 runtime, RCCL 2.26 or the system 2.27) the
// same capture segfaults (bench/rccl_graph_probe.py); this separates the
// framework's capture sequence from that runtime combination.
//
//   RMA_DIAG=rccl_graph RMA_RCCL_BLOCKING=1 ./build/examples/rccl_graph_capi [n] [steps] [K]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

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

static std::vector<double> run(int64_t n, int steps, int K, int graph, double* ms) {
  const int dims[3] = {1, 1, 1}, periods[3] = {1, 1, 0};
  const int ol[3] = {2 * K, 2 * K, 2}, hw[3] = {K, K, 1};
  rma_grid* g = nullptr;
  int me = 0, od[3], oc[3];
  CK(rma_init_global_grid((int)n, (int)n, 1, dims, periods, ol, hw, 1, 0, nullptr, 0, &g, &me,
                          od, oc));
  CK(rma_grid_self_via_rccl(g));
  const double dx = 10.0 / (double)rma_nx_g(g), dy = 10.0 / (double)rma_ny_g(g);
  const double coef[4] = {-1.0, 1 / dx, 1 / dy, (dx < dy ? dx * dx : dy * dy) / 4.1};
  const size_t bytes = (size_t)n * n * sizeof(double);
  double *T, *T2, *iCp;
  HK(hipMalloc(&T, bytes));
  HK(hipMalloc(&T2, bytes));
  HK(hipMalloc(&iCp, bytes));
  hipStream_t s;
  HK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(rma_fill(iCp, n * n, 1.0, s));
  CK(rma_init_random(g, T, n, n, dx, dy, 1234, s));
  HK(hipMemcpyAsync(T2, T, bytes, hipMemcpyDeviceToDevice, s));
  rma_executor* ex = nullptr;
  CK(rma_executor_create_g(g, 1, T, T2, iCp, n, n, coef, 1, 1, K, K > 1, graph ? 20 : 0,
                           nullptr, nullptr, nullptr, &ex));
  std::printf("stage: run graph=%d\n", graph);
  std::fflush(stdout);
  CK(rma_executor_run(ex, 40, s));  // warm-up (captures the graph when graph=1)
  HK(hipStreamSynchronize(s));
  const auto t0 = std::chrono::steady_clock::now();
  CK(rma_executor_run(ex, steps, s));
  HK(hipStreamSynchronize(s));
  *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() /
        steps;
  std::vector<double> out((size_t)n * n);
  HK(hipMemcpy(out.data(), rma_executor_parity(ex) ? T2 : T, bytes, hipMemcpyDeviceToHost));
  CK(rma_executor_destroy(ex));
  HK(hipFree(T));
  HK(hipFree(T2));
  HK(hipFree(iCp));
  HK(hipStreamDestroy(s));
  CK(rma_finalize_global_grid(g));
  return out;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 4096;
  const int steps = argc > 2 ? std::atoi(argv[2]) : 400;
  const int K = argc > 3 ? std::atoi(argv[3]) : 1;
  double ms_eager = 0, ms_graph = 0;
  const std::vector<double> a = run(n, steps, K, 0, &ms_eager);
  std::printf("eager: %.5f ms/step\n", ms_eager);
  std::fflush(stdout);
  const std::vector<double> b = run(n, steps, K, 1, &ms_graph);
  size_t bad = 0;
  for (size_t i = 0; i < a.size(); ++i) bad += a[i] != b[i];
  std::printf("graph: %.5f ms/step, %zu cells differ from eager\n", ms_graph, bad);
  std::printf(bad == 0 ? "OK\n" : "MISMATCH\n");
  return bad == 0 ? 0 : 4;
}
