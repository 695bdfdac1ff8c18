// Host stand-in for the few HIP runtime calls of csrc/runtime/loopback.cpp and
// csrc/runtime/halo.cpp, so both compile with g++ under ThreadSanitizer and
// AddressSanitizer (tests/native/threaded_selftest.cpp).
//
// Model: every stream operation runs synchronously on the calling thread
// (a copy happens at enqueue time, after everything enqueued before it), so
// stream ordering degenerates to program order. Events are heap objects:
// recording or waiting on an event another thread already destroyed is a
// heap-use-after-free for ASan, a race with the free for TSan, and a
// "dead event" abort without any sanitizer. Allocation counters let the test
// check that nothing leaks.
#pragma once

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef enum hipError_t {
  hipSuccess = 0,
  hipErrorInvalidValue = 1,
  hipErrorInvalidResourceHandle = 400,
} hipError_t;

typedef enum hipMemcpyKind {
  hipMemcpyHostToHost = 0,
  hipMemcpyHostToDevice = 1,
  hipMemcpyDeviceToHost = 2,
  hipMemcpyDeviceToDevice = 3,
  hipMemcpyDefault = 4,
} hipMemcpyKind;

#define hipEventDefault 0x0
#define hipEventDisableTiming 0x2

struct rma_stub_event {
  uint64_t magic;                  // kAlive until destroyed (plain: the free races with it)
  std::atomic<uint64_t> records;   // real events are internally synchronised
};
typedef rma_stub_event* hipEvent_t;
struct ihipStream_t;
typedef ihipStream_t* hipStream_t;

namespace rma_stub {
constexpr uint64_t kAlive = 0xA11FE5EEDULL;
inline std::atomic<long>& live_events() {
  static std::atomic<long> n{0};
  return n;
}
inline std::atomic<long>& live_allocs() {
  static std::atomic<long> n{0};
  return n;
}
inline std::atomic<long>& waits() {
  static std::atomic<long> n{0};
  return n;
}
[[noreturn]] inline void dead_event(const char* op) {
  std::fprintf(stderr, "hip stub: %s on a destroyed event\n", op);
  std::abort();
}
}  // namespace rma_stub

inline const char* hipGetErrorName(hipError_t e) { return e == hipSuccess ? "hipSuccess" : "hipError"; }
inline const char* hipGetErrorString(hipError_t e) { return e == hipSuccess ? "no error" : "stub error"; }
inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipDeviceSynchronize() { return hipSuccess; }

inline hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
  if (!e) return hipErrorInvalidValue;
  *e = new rma_stub_event{rma_stub::kAlive, {0}};
  ++rma_stub::live_events();
  return hipSuccess;
}
inline hipError_t hipEventDestroy(hipEvent_t e) {
  if (!e) return hipErrorInvalidResourceHandle;
  if (e->magic != rma_stub::kAlive) rma_stub::dead_event("hipEventDestroy");
  e->magic = 0;
  delete e;
  --rma_stub::live_events();
  return hipSuccess;
}
inline hipError_t hipEventRecord(hipEvent_t e, hipStream_t) {
  if (!e) return hipErrorInvalidResourceHandle;
  if (e->magic != rma_stub::kAlive) rma_stub::dead_event("hipEventRecord");
  e->records.fetch_add(1, std::memory_order_release);
  return hipSuccess;
}
inline hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t e, unsigned) {
  if (!e) return hipErrorInvalidResourceHandle;
  if (e->magic != rma_stub::kAlive) rma_stub::dead_event("hipStreamWaitEvent");
  (void)e->records.load(std::memory_order_acquire);
  ++rma_stub::waits();
  return hipSuccess;
}
inline hipError_t hipMemcpyAsync(void* dst, const void* src, size_t n, hipMemcpyKind, hipStream_t) {
  if (n) std::memcpy(dst, src, n);
  return hipSuccess;
}
inline hipError_t hipMalloc(void** p, size_t n) {
  if (!p) return hipErrorInvalidValue;
  *p = std::malloc(n ? n : 1);
  if (!*p) return hipErrorInvalidValue;
  std::memset(*p, 0xCD, n);
  ++rma_stub::live_allocs();
  return hipSuccess;
}
inline hipError_t hipFree(void* p) {
  if (p) {
    std::free(p);
    --rma_stub::live_allocs();
  }
  return hipSuccess;
}
