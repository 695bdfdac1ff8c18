#include "rma/config.h"
#include "rma/comm.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <type_traits>

#include <dlfcn.h>

#include "rma/hip_check.h"

namespace rma {

namespace {
// ---------------------------------------------------------------------------
// RCCL entry points. By default the library this core is linked against,
// which in a torch process resolves to torch's bundled RCCL (it is loaded
// first, into the global scope). RMA_RCCL_LIB=system (or a path) loads
// /opt/rocm/lib/librccl.so.1 privately instead (RTLD_LOCAL | RTLD_DEEPBIND:
// its internal calls bind to itself; it shares the process's HIP runtime) for
// the native communicators only -- torch's own process groups keep theirs.
// Used to test RCCL P2P under hipGraph capture with the system RCCL
// (bench/rccl_graph_probe.py).
struct RcclApi {
  decltype(&ncclGetErrorString) GetErrorString = &ncclGetErrorString;
  decltype(&ncclGetLastError) GetLastError = &ncclGetLastError;
  decltype(&ncclGetVersion) GetVersion = &ncclGetVersion;
  decltype(&ncclGetUniqueId) GetUniqueId = &ncclGetUniqueId;
  decltype(&ncclCommInitRankConfig) CommInitRankConfig = &ncclCommInitRankConfig;
  decltype(&ncclCommInitRank) CommInitRank = &ncclCommInitRank;
  decltype(&ncclCommAbort) CommAbort = &ncclCommAbort;
  decltype(&ncclCommGetAsyncError) CommGetAsyncError = &ncclCommGetAsyncError;
  decltype(&ncclCommDestroy) CommDestroy = &ncclCommDestroy;
  decltype(&ncclCommSplit) CommSplit = &ncclCommSplit;
  decltype(&ncclCommCount) CommCount = &ncclCommCount;
  decltype(&ncclGroupStart) GroupStart = &ncclGroupStart;
  decltype(&ncclGroupEnd) GroupEnd = &ncclGroupEnd;
  decltype(&ncclSend) Send = &ncclSend;
  decltype(&ncclRecv) Recv = &ncclRecv;
  decltype(&ncclAllReduce) AllReduce = &ncclAllReduce;
  decltype(&ncclBroadcast) Broadcast = &ncclBroadcast;
  std::string source = "linked";
};

RcclApi load_rccl_api() {
  RcclApi a;
  const char* e = std::getenv("RMA_RCCL_LIB");
  if (!e || !*e || std::string(e) == "linked") return a;
  const std::string path = std::string(e) == "system" ? "/opt/rocm/lib/librccl.so.1" : e;
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
  if (!h) throw_error("RMA_RCCL_LIB: dlopen failed", __FILE__, __LINE__, dlerror());
  auto sym = [&](auto& fp, const char* name) {
    void* p = dlsym(h, name);
    if (!p) throw_error("RMA_RCCL_LIB: missing symbol", __FILE__, __LINE__, name);
    fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(p);
  };
  sym(a.GetErrorString, "ncclGetErrorString");
  sym(a.GetLastError, "ncclGetLastError");
  sym(a.GetVersion, "ncclGetVersion");
  sym(a.GetUniqueId, "ncclGetUniqueId");
  sym(a.CommInitRankConfig, "ncclCommInitRankConfig");
  sym(a.CommInitRank, "ncclCommInitRank");
  sym(a.CommAbort, "ncclCommAbort");
  sym(a.CommGetAsyncError, "ncclCommGetAsyncError");
  sym(a.CommDestroy, "ncclCommDestroy");
  sym(a.CommSplit, "ncclCommSplit");
  sym(a.CommCount, "ncclCommCount");
  sym(a.GroupStart, "ncclGroupStart");
  sym(a.GroupEnd, "ncclGroupEnd");
  sym(a.Send, "ncclSend");
  sym(a.Recv, "ncclRecv");
  sym(a.AllReduce, "ncclAllReduce");
  sym(a.Broadcast, "ncclBroadcast");
  a.source = path;
  return a;
}

const RcclApi& rccl() {
  static const RcclApi a = load_rccl_api();
  return a;
}
}  // namespace

#define RMA_NCCL_CHECK(expr)                                                              \
  do {                                                                                    \
    ncclResult_t _r = (expr);                                                             \
    if (_r != ncclSuccess && _r != ncclInProgress) {                                      \
      ::rma::throw_error("RCCL call failed: " #expr, __FILE__, __LINE__,                  \
                         std::string(rccl().GetErrorString(_r)) + " / " +                    \
                             (rccl().GetLastError(nullptr) ? rccl().GetLastError(nullptr) : "")); \
    }                                                                                     \
  } while (0)

namespace {
ncclComm_t C(void* p) { return reinterpret_cast<ncclComm_t>(p); }

ncclDataType_t to_nccl(DType d) {
  switch (d) {
    case DType::kFloat64: return ncclFloat64;
    case DType::kFloat32: return ncclFloat32;
    case DType::kInt64: return ncclInt64;
    case DType::kInt32: return ncclInt32;
    case DType::kUInt8: return ncclUint8;
  }
  return ncclFloat64;
}

ncclRedOp_t to_nccl(RedOp o) {
  switch (o) {
    case RedOp::kSum: return ncclSum;
    case RedOp::kMax: return ncclMax;
    case RedOp::kMin: return ncclMin;
    case RedOp::kProd: return ncclProd;
  }
  return ncclSum;
}
}  // namespace

int rccl_version() {
  int v = 0;
  rccl().GetVersion(&v);
  return v;
}

std::string rccl_library() { return rccl().source; }

std::string device_pci_bus_id(int device) {
  char buf[64] = {0};
  RMA_HIP_CHECK(hipDeviceGetPCIBusId(buf, (int)sizeof(buf) - 1, device));
  return std::string(buf);
}

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  RMA_NCCL_CHECK(rccl().GetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

RcclComm::RcclComm(int nranks, int rank, const std::string& uid, int device,
                   double init_timeout_s)
    : nranks_(nranks), rank_(rank), device_(device) {
  RMA_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "rank " << rank << "/" << nranks);
  RMA_CHECK_ARG(uid.size() == sizeof(ncclUniqueId),
                "unique id has " << uid.size() << " bytes, expected " << sizeof(ncclUniqueId));
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  RMA_HIP_CHECK(hipSetDevice(device));
  ncclComm_t c = nullptr;
  if (init_timeout_s > 0) {
    nonblocking_ = true;
    timeout_s_ = init_timeout_s;
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    RMA_NCCL_CHECK(rccl().CommInitRankConfig(&c, nranks, id, rank, &cfg));
    comm_ = c;
    poll_ready(comm_, "ncclCommInitRankConfig (did every rank join?)");
    // opt-in: a blocking data communicator split from this one. Measured
    // with RCCL send/recv to self at 16384^2 one-step: 0.831 vs 0.832 ms of
    // host time per step (two groups) with polled group ends, i.e. the cost
    // is RCCL's own enqueue, not the polling (profiles/rccl_self_16k_k1_r2*.json)
    if (diag_flag("rccl_data_blocking")) split_blocking(rank);  // RMA_DIAG rccl_data_blocking
  } else {
    RMA_NCCL_CHECK(rccl().CommInitRank(&c, nranks, id, rank));
    comm_ = c;
  }
  RMA_HIP_CHECK(hipMalloc(&scratch_, 2 * sizeof(double)));
}

// Every rank joined: run the data path on a BLOCKING communicator split from
// the non-blocking one (group ends return once enqueued instead of being
// polled; dead peers are still caught by wait()'s timeout). Best effort: if
// the split fails or stalls, the non-blocking communicator stays the data
// path (same transport, polled group ends) and the parent is NOT aborted.
void RcclComm::split_blocking(int rank) {
  ncclConfig_t bc = NCCL_CONFIG_INITIALIZER;
  bc.blocking = 1;
  ncclComm_t child = nullptr;
  const ncclResult_t r = rccl().CommSplit(C(comm_), 0, rank, &child, &bc);
  auto give_up = [&](const std::string& why) {
    if (child) (void)rccl().CommAbort(child);
    fprintf(stderr, "[rocm_mpi_amd rank %d] RCCL: no blocking data communicator (%s); "
            "group ends are polled\n", rank, why.c_str());
  };
  if (r != ncclSuccess && r != ncclInProgress) {
    give_up(rccl().GetErrorString(r));
    return;
  }
  // a non-blocking parent completes the split asynchronously
  const auto t0 = std::chrono::steady_clock::now();
  const double limit = std::min(timeout_s_, 120.0);
  for (int spins = 0;; ++spins) {
    ncclResult_t st = ncclSuccess;
    (void)rccl().CommGetAsyncError(C(comm_), &st);
    if (st == ncclSuccess && child) {
      ncclResult_t cs = ncclSuccess;
      (void)rccl().CommGetAsyncError(child, &cs);
      if (cs == ncclSuccess) break;
      if (cs != ncclInProgress) {
        give_up(rccl().GetErrorString(cs));
        return;
      }
    } else if (st != ncclSuccess && st != ncclInProgress) {
      give_up(rccl().GetErrorString(st));
      return;
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
      give_up("split did not complete");
      return;
    }
    if (spins < 4096)
      std::this_thread::yield();
    else
      std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  parent_ = comm_;
  comm_ = child;
}

void RcclComm::poll_ready(void* comm, const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  int spins = 0;
  for (;;) {
    ncclResult_t st = ncclSuccess;
    const ncclResult_t r = rccl().CommGetAsyncError(C(comm), &st);
    if (r != ncclSuccess) st = r;
    if (st == ncclSuccess) return;
    if (st != ncclInProgress) {
      abort();
      throw_error("RCCL asynchronous error", __FILE__, __LINE__,
                  std::string(what) + ": " + rccl().GetErrorString(st));
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > timeout_s_) {
      abort();
      throw_error("RCCL timeout", __FILE__, __LINE__,
                  std::string(what) + " still in progress after " + std::to_string(timeout_s_) +
                      " s; communicator aborted");
    }
    // yield first (a group end completes in tens of us), then back off
    if (++spins < 4096)
      std::this_thread::yield();
    else
      std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

void RcclComm::settle(const char* what) {
  if (!nonblocking_ || parent_) return;  // blocking data communicator
  poll_ready(comm_, what);
}

RcclComm::~RcclComm() {
  if (scratch_) (void)hipFree(scratch_);
  if (aborted_) return;  // already torn down by abort()
  if (comm_) (void)rccl().CommDestroy(C(comm_));
  if (parent_) (void)rccl().CommDestroy(C(parent_));
}

int RcclComm::count() const {
  RMA_CHECK_ARG(comm_ != nullptr && !aborted_, "communicator is gone");
  int n = -1;
  RMA_NCCL_CHECK(rccl().CommCount(C(comm_), &n));
  return n;
}

bool RcclComm::capturable() const { return diag_flag("rccl_graph"); }  // RMA_DIAG rccl_graph

void RcclComm::group_start() {
  RMA_NCCL_CHECK(rccl().GroupStart());
  ++group_depth_;
}
void RcclComm::group_end() {
  --group_depth_;
  RMA_NCCL_CHECK(rccl().GroupEnd());
  if (group_depth_ == 0) settle("ncclGroupEnd");
}

void RcclComm::send(const void* buf, size_t bytes, int peer, stream_t stream) {
  RMA_CHECK_ARG(peer >= 0 && peer < nranks_, "peer " << peer);
  RMA_NCCL_CHECK(rccl().Send(buf, bytes, ncclUint8, peer, C(comm_), as_stream(stream)));
  if (group_depth_ == 0) settle("ncclSend");
}

void RcclComm::recv(void* buf, size_t bytes, int peer, stream_t stream) {
  RMA_CHECK_ARG(peer >= 0 && peer < nranks_, "peer " << peer);
  RMA_NCCL_CHECK(rccl().Recv(buf, bytes, ncclUint8, peer, C(comm_), as_stream(stream)));
  if (group_depth_ == 0) settle("ncclRecv");
}

void RcclComm::allreduce(const void* sendbuf, void* recvbuf, size_t count, DType dt, RedOp op,
                         stream_t stream) {
  RMA_NCCL_CHECK(
      rccl().AllReduce(sendbuf, recvbuf, count, to_nccl(dt), to_nccl(op), C(comm_), as_stream(stream)));
  settle("ncclAllReduce");
}

void RcclComm::broadcast(const void* sendbuf, void* recvbuf, size_t count, DType dt, int root,
                         stream_t stream) {
  RMA_NCCL_CHECK(
      rccl().Broadcast(sendbuf, recvbuf, count, to_nccl(dt), root, C(comm_), as_stream(stream)));
  settle("ncclBroadcast");
}

void RcclComm::gather(const void* sendbuf, void* recvbuf, size_t bytes, int root,
                      stream_t stream) {
  hipStream_t s = as_stream(stream);
  RMA_NCCL_CHECK(rccl().GroupStart());
  if (rank_ == root) {
    for (int r = 0; r < nranks_; ++r) {
      char* dst = static_cast<char*>(recvbuf) + (size_t)r * bytes;
      if (r == root) {
        RMA_HIP_CHECK(hipMemcpyAsync(dst, sendbuf, bytes, hipMemcpyDeviceToDevice, s));
      } else {
        RMA_NCCL_CHECK(rccl().Recv(dst, bytes, ncclUint8, r, C(comm_), s));
      }
    }
  } else {
    RMA_NCCL_CHECK(rccl().Send(sendbuf, bytes, ncclUint8, root, C(comm_), s));
  }
  RMA_NCCL_CHECK(rccl().GroupEnd());
  settle("gather");
}

void RcclComm::barrier(stream_t stream, double timeout_s) {
  hipStream_t s = as_stream(stream);
  RMA_HIP_CHECK(hipMemsetAsync(scratch_, 0, sizeof(double), s));
  RMA_NCCL_CHECK(rccl().AllReduce(scratch_, scratch_ + 1, 1, ncclFloat64, ncclSum, C(comm_), s));
  settle("barrier");
  wait(stream, timeout_s);
}

void RcclComm::check_async() {
  if (aborted_) throw_error("communicator was aborted", __FILE__, __LINE__, "");
  ncclResult_t ar = ncclSuccess;
  RMA_NCCL_CHECK(rccl().CommGetAsyncError(C(comm_), &ar));
  if (ar != ncclSuccess && ar != ncclInProgress) {
    abort();
    throw_error("RCCL asynchronous error", __FILE__, __LINE__, rccl().GetErrorString(ar));
  }
}

void RcclComm::wait(stream_t stream, double timeout_s) {
  hipStream_t s = as_stream(stream);
  const auto t0 = std::chrono::steady_clock::now();
  int spins = 0;
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) RMA_HIP_CHECK(q);
    check_async();
    if (timeout_s > 0) {
      const double el =
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_s) {
        abort();
        throw_error("communication timeout", __FILE__, __LINE__,
                    "stream did not drain within " + std::to_string(timeout_s) +
                        " s (dead or stalled peer?); communicator aborted");
      }
    }
    if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

void RcclComm::abort() {
  if (aborted_ || !comm_) return;
  aborted_ = true;
  (void)rccl().CommAbort(C(comm_));
  if (parent_) (void)rccl().CommAbort(C(parent_));
}

}  // namespace rma
