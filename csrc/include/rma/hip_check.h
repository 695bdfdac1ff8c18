// HIP error checking for the native core (HIP translation units only).
#pragma once

#include <hip/hip_runtime.h>

#include "rma/common.h"

#define RMA_HIP_CHECK(expr)                                                              \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) {                                                              \
      ::rma::throw_error("HIP call failed: " #expr, __FILE__, __LINE__,                  \
                         std::string(hipGetErrorName(_e)) + ": " + hipGetErrorString(_e)); \
    }                                                                                    \
  } while (0)

// Check the launch status of the kernel just enqueued (configuration errors
// are reported synchronously by hipGetLastError / hipPeekAtLastError).
#define RMA_HIP_LAUNCH_CHECK() RMA_HIP_CHECK(hipGetLastError())

namespace rma {
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
}  // namespace rma
