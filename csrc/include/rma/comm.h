// GPU-direct communicator: RCCL point-to-point and tiny collectives over xGMI.
//
// Replaces the reference's MPI.jl + ROCm-aware OpenMPI/UCX transport
// (scripts/setenv.sh:11-18, scripts/rocmaware_test_selectdevice.jl:3-24) and
// the MPI calls hidden inside ImplicitGlobalGrid. Bootstrap is
// MPI-free: rank 0 calls unique_id(), the bytes travel through the
// torch.distributed store, every rank constructs RcclComm(nranks, rank, id).
//
// Failure detection: every RCCL/HIP return code is checked and
// turned into rma::Error carrying the rank; wait() polls the stream together
// with ncclCommGetAsyncError and aborts the communicator after a timeout, so a
// dead peer produces an exception instead of a hang. With init_timeout_s > 0
// the communicator is created non-blocking (ncclConfig_t::blocking = 0): the
// constructor polls ncclCommGetAsyncError and aborts after the timeout, so a
// rank that never joins cannot hang the others inside ncclCommInitRank; every
// later RCCL call is settled (polled until it left ncclInProgress) before
// anything else is enqueued on its stream.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>

#include "rma/kernels.h"
#include "rma/p2p.h"

namespace rma {

enum class DType : int { kFloat64 = 0, kFloat32 = 1, kInt64 = 2, kInt32 = 3, kUInt8 = 4 };
enum class RedOp : int { kSum = 0, kMax = 1, kMin = 2, kProd = 3 };

class RcclComm : public P2PTransport {
 public:
  static std::string unique_id();  // 128 opaque bytes, generate on ONE rank
  RcclComm(int nranks, int rank, const std::string& uid, int device,
           double init_timeout_s = 0.0);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  int rank() const override { return rank_; }
  int size() const override { return nranks_; }
  int device() const { return device_; }
  // ranks of the communicator as RCCL itself reports them (ncclCommCount)
  int count() const;

  void group_start() override;
  void group_end() override;
  void send(const void* buf, size_t bytes, int peer, stream_t stream) override;
  void recv(void* buf, size_t bytes, int peer, stream_t stream) override;
  // RCCL P2P inside hipStreamBeginCapture crashed (SIGSEGV) with the RCCL
  // 2.26 bundled by torch on MI355X (scripts/rccl_probe.py, 2026-10-15):
  // graph replay is refused unless RMA_DIAG=rccl_graph.
  bool capturable() const override;
  void allreduce(const void* sendbuf, void* recvbuf, size_t count, DType dt, RedOp op,
                 stream_t stream);
  void broadcast(const void* sendbuf, void* recvbuf, size_t count, DType dt, int root,
                 stream_t stream);
  // Root gathers `bytes` from every rank into recvbuf (rank-major); P2P-based.
  void gather(const void* sendbuf, void* recvbuf, size_t bytes, int root, stream_t stream);
  // Device-side barrier: 1-element all-reduce on `stream`, then wait().
  void barrier(stream_t stream, double timeout_s);
  // Block until `stream` drains; throw (after ncclCommAbort) on async error or
  // timeout (timeout_s <= 0: no timeout).
  void wait(stream_t stream, double timeout_s);
  // Raises if RCCL reported an asynchronous error.
  void check_async();
  void abort();
  bool aborted() const { return aborted_; }
  // nonblocking(): the communicator was created non-blocking (init with a
  // timeout; group ends are then polled until RCCL has enqueued them);
  // data_blocking(): the data path runs on a blocking communicator
  // (RMA_RCCL_BLOCKING=1 init, or RMA_DIAG rccl_data_blocking: split from the
  // non-blocking one after init; no host-time gain measured, see comm.cpp).
  bool nonblocking() const { return nonblocking_; }
  bool data_blocking() const { return parent_ != nullptr || !nonblocking_; }

 private:
  // Non-blocking data communicator: wait until the last call left ncclInProgress.
  void settle(const char* what);
  void poll_ready(void* comm, const char* what);
  void split_blocking(int rank);
  int nranks_, rank_, device_;
  void* comm_ = nullptr;  // ncclComm_t of the data path
  void* parent_ = nullptr;  // the non-blocking communicator comm_ was split from
  double* scratch_ = nullptr;  // 2 doubles of device memory for barrier()
  bool aborted_ = false;
  bool nonblocking_ = false;
  double timeout_s_ = 0.0;
  int group_depth_ = 0;  // settle only outside ncclGroupStart/End
};

int rccl_version();
// "linked" or the path RMA_RCCL_LIB loaded the native communicators' RCCL from
std::string rccl_library();
// PCI bus id ("0000:05:00.0") of a HIP device: tells whether two ranks drive
// the same physical GPU (bench.py refuses that for a scaling point).
std::string device_pci_bus_id(int device);

}  // namespace rma
