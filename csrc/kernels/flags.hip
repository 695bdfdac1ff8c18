// Stream-ordered cross-process flags for the HIP IPC transport
// (csrc/runtime/ipc.cpp, stream mode): one tiny kernel that waits until a
// 64-bit word in host-registered shared memory equals a value, one that
// writes it.
//
// Why kernels and not hipStreamWaitValue64 / hipStreamWriteValue64: on the
// HIP runtime torch bundles, those stream operations work eagerly but replay
// to a wrong field once captured in a hipGraph
// (profiles/r5/ipc_graph_replay_failure.log), their command-processor form
// refuses host-registered memory, and a wait never returns if the peer died.
// Kernel nodes capture like any other launch, and the wait is BOUNDED: it
// gives up after a timeout on the constant-rate wall clock, records the
// failure in an error word the host checks, and exits -- every wave of the
// grid always finishes.
//
// Memory model: the flag lives in shared host memory that both processes
// registered for their GPU. Loads and stores are system-scope atomics
// (vector memory instructions that bypass the non-coherent caches); the
// writer's release follows the copies it publishes in stream order, the
// waiter's acquire precedes the copies that read the mailbox.
#include <hip/hip_runtime.h>

#include "rma/hip_check.h"
#include "rma/kernels.h"

namespace rma {
namespace {

__global__ __launch_bounds__(64) void flag_wait_kernel(const uint64_t* flag, uint64_t want,
                                                       uint64_t max_ticks, uint32_t* err,
                                                       uint32_t code) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  for (;;) {
    const uint64_t v = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v == want) return;
    if (wall_clock64() - t0 > max_ticks) {
      // the host sees the failure at its next check; the grid exits
      __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(4);
  }
}

__global__ __launch_bounds__(64) void flag_write_kernel(uint64_t* flag, uint64_t value) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// direct-store halos: lane i < 8 waits for its flag (monotonic pass counters,
// so >=: a neighbour may already be one pass ahead); every lane exits
__global__ __launch_bounds__(64) void flags_wait_ge_kernel(const uint64_t* flags, uint32_t mask,
                                                           uint64_t want, uint64_t max_ticks,
                                                           uint32_t* err, uint32_t code) {
  const int i = threadIdx.x;
  if (i >= 8 || !((mask >> i) & 1u)) return;
  const uint64_t t0 = wall_clock64();
  for (;;) {
    const uint64_t v = __hip_atomic_load(flags + i, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v >= want) return;
    if (wall_clock64() - t0 > max_ticks) {
      __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(4);
  }
}

__global__ __launch_bounds__(64) void flags_write_kernel(FlagTargets t, uint64_t value) {
  const int i = threadIdx.x;
  if (i < 8 && t.dst[i]) __hip_atomic_store(t.dst[i], value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

uint64_t wall_ticks_per_s() {
  static const uint64_t rate = [] {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
      khz = 100000;  // gfx9 constant-rate clock: 100 MHz
    return (uint64_t)khz * 1000ull;
  }();
  return rate;
}

}  // namespace

void flag_wait_gpu(const uint64_t* flag, uint64_t want, double timeout_s, uint32_t* err,
                   uint32_t code, stream_t stream) {
  RMA_CHECK_ARG(flag != nullptr && err != nullptr, "null flag or error word");
  RMA_CHECK_ARG(timeout_s > 0 && timeout_s < 1e6, "flag wait timeout " << timeout_s << " s");
  const uint64_t ticks = (uint64_t)(timeout_s * (double)wall_ticks_per_s());
  hipLaunchKernelGGL(flag_wait_kernel, dim3(1), dim3(64), 0, as_stream(stream), flag, want,
                     ticks, err, code);
  RMA_HIP_LAUNCH_CHECK();
}

void flags_wait_ge_gpu(const uint64_t* flags, uint32_t mask, uint64_t want, double timeout_s,
                       uint32_t* err, uint32_t code, stream_t stream) {
  RMA_CHECK_ARG(flags != nullptr && err != nullptr, "null flags or error word");
  RMA_CHECK_ARG(timeout_s > 0 && timeout_s < 1e6, "flag wait timeout " << timeout_s << " s");
  if (mask == 0) return;
  const uint64_t ticks = (uint64_t)(timeout_s * (double)wall_ticks_per_s());
  hipLaunchKernelGGL(flags_wait_ge_kernel, dim3(1), dim3(64), 0, as_stream(stream), flags, mask,
                     want, ticks, err, code);
  RMA_HIP_LAUNCH_CHECK();
}

void flags_write_gpu(const FlagTargets& t, uint64_t value, stream_t stream) {
  hipLaunchKernelGGL(flags_write_kernel, dim3(1), dim3(64), 0, as_stream(stream), t, value);
  RMA_HIP_LAUNCH_CHECK();
}

void flag_write_gpu(uint64_t* flag, uint64_t value, stream_t stream) {
  RMA_CHECK_ARG(flag != nullptr, "null flag");
  hipLaunchKernelGGL(flag_write_kernel, dim3(1), dim3(64), 0, as_stream(stream), flag, value);
  RMA_HIP_LAUNCH_CHECK();
}

}  // namespace rma
