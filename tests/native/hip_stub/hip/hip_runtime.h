// Host stand-in for the few HIP runtime calls of csrc/runtime/loopback.cpp,
// csrc/runtime/halo.cpp and csrc/runtime/ipc.cpp, so they compile with a host
// compiler under ThreadSanitizer and AddressSanitizer
// (tests/native/threaded_selftest.cpp). IPC "processes" are
// threads of one process: a memory handle carries the pointer itself.
//
// Model: every stream operation runs synchronously on the calling thread
// (a copy happens at enqueue time, after everything enqueued before it), so
// stream ordering degenerates to program order. Events are heap objects:
// recording or waiting on an event another thread already destroyed is a
// heap-use-after-free for ASan, a race with the free for TSan, and a
// "dead event" abort without any sanitizer. Allocation counters let the test
// check that nothing leaks.
//
// Shared memory: rank threads that open the same POSIX shm object get ONE
// mapping of it (refcounted), as processes would get one physical page.
// ThreadSanitizer tracks synchronisation per virtual address, so a release
// store through one alias and an acquire load through another would look
// unsynchronised -- a false report about the stub, not about ipc.cpp.
#pragma once

#include <sys/mman.h>
#include <sys/stat.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <utility>

namespace rma_stub {
struct Mapping {
  void* addr;
  size_t len;
  int refs;
};
inline std::mutex& map_mu() {
  static std::mutex m;
  return m;
}
inline std::map<std::pair<dev_t, ino_t>, Mapping>& mappings() {
  static std::map<std::pair<dev_t, ino_t>, Mapping> m;
  return m;
}
inline void* mmap_shared(void* a, size_t len, int prot, int flags, int fd, off_t off) {
  struct stat st;
  if (!(flags & MAP_SHARED) || fstat(fd, &st) != 0) return ::mmap(a, len, prot, flags, fd, off);
  std::lock_guard<std::mutex> lk(map_mu());
  const auto key = std::make_pair(st.st_dev, st.st_ino);
  auto it = mappings().find(key);
  if (it != mappings().end()) {
    ++it->second.refs;
    return it->second.addr;
  }
  void* m = ::mmap(a, len, prot, flags, fd, off);
  if (m != MAP_FAILED) mappings()[key] = {m, len, 1};
  return m;
}
inline int munmap_shared(void* a, size_t len) {
  std::lock_guard<std::mutex> lk(map_mu());
  for (auto it = mappings().begin(); it != mappings().end(); ++it)
    if (it->second.addr == a) {
      if (--it->second.refs > 0) return 0;
      mappings().erase(it);
      break;
    }
  return ::munmap(a, len);
}
}  // namespace rma_stub
#define mmap rma_stub::mmap_shared
#define munmap rma_stub::munmap_shared

typedef enum hipError_t {
  hipSuccess = 0,
  hipErrorInvalidValue = 1,
  hipErrorInvalidResourceHandle = 400,
  hipErrorNotSupported = 801,
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
#define hipHostMallocMapped 0x2
#define hipHostRegisterMapped 0x2
#define hipIpcMemLazyEnablePeerAccess 0x1
#define hipStreamNonBlocking 0x1

typedef enum hipDeviceAttribute_t {
  hipDeviceAttributeMultiprocessorCount = 63,
  hipDeviceAttributeWallClockRate = 200,
} hipDeviceAttribute_t;
typedef enum hipStreamCaptureMode {
  hipStreamCaptureModeGlobal = 0,
  hipStreamCaptureModeThreadLocal = 1,
  hipStreamCaptureModeRelaxed = 2,
} hipStreamCaptureMode;
struct ihipGraph;
struct hipGraphExec;
typedef ihipGraph* hipGraph_t;
typedef hipGraphExec* hipGraphExec_t;
struct hipGraphNode;
typedef hipGraphNode* hipGraphNode_t;

typedef struct hipIpcMemHandle_st {
  char reserved[64];
} hipIpcMemHandle_t;

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

// streams: distinct non-null handles (work runs at enqueue time anyway)
namespace rma_stub {
inline std::atomic<long>& live_streams() {
  static std::atomic<long> n{0};
  return n;
}
// the executor's fused-pass policy counts tasks per CU: a small "device"
// (RMA_STUB_CUS, default 2) makes test-sized tiles take that path too
inline int stub_cus() {
  const char* e = std::getenv("RMA_STUB_CUS");
  return e && *e ? std::atoi(e) : 2;
}
}  // namespace rma_stub
inline hipError_t hipStreamCreateWithPriority(hipStream_t* s, unsigned, int) {
  *s = reinterpret_cast<hipStream_t>(new char);
  ++rma_stub::live_streams();
  return hipSuccess;
}
inline hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned f) {
  return hipStreamCreateWithPriority(s, f, 0);
}
inline hipError_t hipStreamDestroy(hipStream_t s) {
  delete reinterpret_cast<char*>(s);
  --rma_stub::live_streams();
  return hipSuccess;
}
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
inline hipError_t hipDeviceGetStreamPriorityRange(int* least, int* greatest) {
  *least = 0;
  *greatest = -1;
  return hipSuccess;
}
inline hipError_t hipGetDevice(int* d) {
  *d = 0;
  return hipSuccess;
}
inline hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t a, int) {
  *v = a == hipDeviceAttributeMultiprocessorCount ? rma_stub::stub_cus() : 100000;
  return hipSuccess;
}
inline hipError_t hipEventCreate(hipEvent_t* e);
inline hipError_t hipEventElapsedTime(float* ms, hipEvent_t, hipEvent_t) {
  *ms = 0.0f;
  return hipSuccess;
}
// graphs: not modelled (the executor only captures with a capturable transport)
inline hipError_t hipStreamBeginCapture(hipStream_t, hipStreamCaptureMode) {
  return hipErrorNotSupported;
}
inline hipError_t hipStreamEndCapture(hipStream_t, hipGraph_t* g) {
  *g = nullptr;
  return hipErrorNotSupported;
}
inline hipError_t hipGraphInstantiate(hipGraphExec_t*, hipGraph_t, hipGraphNode_t*, char*, size_t) {
  return hipErrorNotSupported;
}
inline hipError_t hipGraphLaunch(hipGraphExec_t, hipStream_t) { return hipErrorNotSupported; }
inline hipError_t hipGraphDestroy(hipGraph_t) { return hipSuccess; }
inline hipError_t hipGraphExecDestroy(hipGraphExec_t) { return hipSuccess; }

inline const char* hipGetErrorName(hipError_t e) { return e == hipSuccess ? "hipSuccess" : "hipError"; }
inline const char* hipGetErrorString(hipError_t e) { return e == hipSuccess ? "no error" : "stub error"; }
inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipDeviceSynchronize() { return hipSuccess; }
inline hipError_t hipSetDevice(int) { return hipSuccess; }
inline hipError_t hipEventSynchronize(hipEvent_t e) {
  if (!e) return hipErrorInvalidResourceHandle;
  if (e->magic != rma_stub::kAlive) rma_stub::dead_event("hipEventSynchronize");
  return hipSuccess;
}

inline hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
  if (!e) return hipErrorInvalidValue;
  *e = new rma_stub_event{rma_stub::kAlive, {0}};
  ++rma_stub::live_events();
  return hipSuccess;
}
inline hipError_t hipEventCreate(hipEvent_t* e) { return hipEventCreateWithFlags(e, 0); }
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
template <typename T>
inline hipError_t hipMalloc(T** p, size_t n) {  // HIP's typed overload
  return hipMalloc(reinterpret_cast<void**>(p), n);
}
inline hipError_t hipMemset(void* p, int v, size_t n) {
  std::memset(p, v, n);
  return hipSuccess;
}
inline hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t) { return hipMemset(p, v, n); }
inline hipError_t hipFree(void* p) {
  if (p) {
    std::free(p);
    --rma_stub::live_allocs();
  }
  return hipSuccess;
}
inline hipError_t hipHostMalloc(void** p, size_t n, unsigned) { return hipMalloc(p, n); }
inline hipError_t hipHostFree(void* p) { return hipFree(p); }
inline hipError_t hipHostRegister(void*, size_t, unsigned) { return hipSuccess; }
inline hipError_t hipHostUnregister(void*) { return hipSuccess; }
inline hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned) {
  *d = h;  // one address space
  return hipSuccess;
}
inline hipError_t hipIpcGetMemHandle(hipIpcMemHandle_t* h, void* p) {
  std::memset(h, 0, sizeof *h);
  std::memcpy(h->reserved, &p, sizeof p);
  return hipSuccess;
}
inline hipError_t hipIpcOpenMemHandle(void** p, hipIpcMemHandle_t h, unsigned) {
  std::memcpy(p, h.reserved, sizeof *p);
  return hipSuccess;
}
inline hipError_t hipIpcCloseMemHandle(void*) { return hipSuccess; }
inline hipError_t hipMemGetAddressRange(void** base, size_t* bytes, void* p) {
  *base = p;  // the stub does not track allocation extents: p is its own base
  *bytes = size_t(1) << 40;
  return hipSuccess;
}
