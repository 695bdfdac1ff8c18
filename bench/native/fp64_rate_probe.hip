// fp64 issue-rate probe: v_mfma_f64_16x16x4f64 vs VALU v_fma_f64 on MI355X.
//
// Why the stencil passes do not use MFMA (docs/ARCHITECTURE.md §3.2): a
// 5-point update is a banded linear map; on the 16x16x4 fp64 MFMA a 16-row
// y-stencil tile needs 5 MFMAs (K = 18 input rows) = 5120 multiply-adds for
// 256 outputs of 3 useful ones (6.7x waste). That only pays if the fp64 MFMA
// rate is well above the VALU's. This probe measures both rates with every CU
// busy (independent accumulators, back-to-back issue), so the claim rests on
// a number from this machine. Prints one JSON line.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 4096;

// 8 independent 16x16 accumulators per wave; each MFMA = 16*16*4 = 1024 FMA
__global__ __launch_bounds__(256) void mfma_loop(double* out, double a0, double b0) {
  d4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
  double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;  // vector store, keeps the loop alive
}

// 16 independent fp64 FMA chains per lane
__global__ __launch_bounds__(256) void valu_loop(double* out, double a0, double b0) {
  double acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = threadIdx.x * 1e-3 + i;
  const double a = a0 + threadIdx.x * 1e-12, b = b0;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = __builtin_fma(acc[i], a, b);
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class F>
double time_ms(F launch, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms / reps;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int blocks = p.multiProcessorCount * 8;  // 8 blocks of 4 waves per CU
  const int threads = 256;
  double* out = nullptr;
  CK(hipMalloc(&out, sizeof(double) * blocks * threads));
  const double waves = blocks * threads / 64.0;
  const double t_mfma = time_ms([&] { mfma_loop<<<blocks, threads>>>(out, 1.0, 0.5); }, 5);
  const double t_valu = time_ms([&] { valu_loop<<<blocks, threads>>>(out, 0.999, 1e-3); }, 5);
  CK(hipGetLastError());
  // FLOP = 2 per multiply-add
  const double f_mfma = waves * kIters * 8 * 1024.0 * 2;
  const double f_valu = waves * 64.0 * kIters * 16 * 2;
  std::printf(
      "{\"cus\": %d, \"mfma_f64_16x16x4_tflops\": %.2f, \"valu_fma_f64_tflops\": %.2f, "
      "\"mfma_ms\": %.3f, \"valu_ms\": %.3f}\n",
      p.multiProcessorCount, f_mfma / t_mfma / 1e9, f_valu / t_valu / 1e9, t_mfma, t_valu);
  CK(hipFree(out));
  return 0;
}
