// Device-direct transport between PROCESSES of one node without RCCL: HIP IPC.
//
// The reference moves halos between ranks with ROCm-aware MPI, i.e. device
// buffers handed to MPI_Send/Recv (scripts/rocmaware_test_selectdevice.jl:16-22,
// ImplicitGlobalGrid's update_halo! with IGG_ROCMAWARE_MPI=1); inside a node
// the MPI library moves those bytes through CUDA/HIP IPC. This transport does
// the same natively: every receiver owns, per sender, a double-buffered device
// MAILBOX that the sender maps with hipIpcOpenMemHandle and fills with one
// device-to-device copy per message on its own stream (over xGMI when the
// ranks drive different GPUs, on-device when they share one). Ordering is
// stream-ordered on the GPU and handshaked on the host:
//   * sender, generation g of a (sender, receiver) pair: waits (host) until the
//     receiver has published "done with g-2", copies into slot g%2, records
//     its "sent" event, waits for it on the host, publishes g in the
//     receiver's shared-memory flag block;
//   * receiver: waits (host) until the sender published g, copies the slot
//     out, records its "done" event, waits for it, publishes g.
// (RMA_IPC_GPU_EVENTS=1: the flags mean "record enqueued" and the streams wait
// on the peer's interprocess events instead of the host; RMA_IPC_STREAM_FLAGS=1:
// the GPU writes the flags after the copies; see ipc.cpp.) The
// executor enqueues the interior before the frame and the exchange for such a
// host-synchronising transport, so the blocking costs no overlap.
// Host waits are bounded (timeout -> rma::Error naming the peer); the GPU only
// ever waits on event records the host has seen enqueued, so a dead peer ends
// in an exception, not a hang. Flags live in one POSIX shared-memory block per
// receiver (/dev/shm). Not stream-capturable (host handshake), like loopback.
//
// Bootstrap (rocm_mpi_amd/parallel/comm.py IpcComm): construct on every rank
// with the peer list (neighbours and diagonals), publish export_for(p) through
// the torch.distributed store, connect(p, blob) with what p exported for me.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "rma/p2p.h"

namespace rma {

class IpcTransport : public P2PTransport {
 public:
  // token: job-unique name part of the shared-memory blocks; mailbox_bytes:
  // capacity of ONE slot per sender (the bytes of one group to one peer)
  IpcTransport(int rank, int size, int device, const std::vector<int>& peers,
               size_t mailbox_bytes, const std::string& token, double timeout_s);
  ~IpcTransport() override;
  IpcTransport(const IpcTransport&) = delete;
  IpcTransport& operator=(const IpcTransport&) = delete;

  // what peer p needs from me: my mailbox for p's messages, my "done" event
  // for p's messages, my "sent" event for my messages to p (opaque bytes)
  std::string export_for(int peer) const;
  // open what peer p exported for me (and p's shared-memory flag block)
  void connect(int peer, const std::string& blob);
  bool connected() const;

  int rank() const override { return rank_; }
  int size() const override { return size_; }
  void group_start() override;
  void group_end() override;
  void send(const void* buf, size_t bytes, int peer, stream_t stream) override;
  void recv(void* buf, size_t bytes, int peer, stream_t stream) override;
  bool capturable() const override { return false; }
  size_t mailbox_bytes() const { return cap_; }

 private:
  struct Op {
    void* buf;
    size_t bytes;
    int peer;
    stream_t stream;
  };
  struct Peer {
    int rank = -1;
    // mine (receiver side): mailbox for this peer's messages + done event
    void* mailbox = nullptr;
    void* done_ev = nullptr;
    // mine (sender side): sent event for my messages to this peer
    void* sent_ev = nullptr;
    // host-synchronised mode: plain events (a host wait on an interprocess
    // event costs ~1 ms on this runtime)
    void* sent_local = nullptr;
    void* done_local = nullptr;
    // the peer's, opened: its mailbox for my messages, its done / sent events
    void* r_mailbox = nullptr;
    void* r_done_ev = nullptr;
    void* r_sent_ev = nullptr;
    void* r_flags = nullptr;  // the peer's shared-memory flag block (mapped)
    void* r_flags_dev = nullptr;  // ... registered for GPU writes (stream flags)
    uint64_t send_gen = 0, recv_gen = 0;
    bool connected = false;
  };
  Peer& peer(int p);
  void wait_flag(const void* addr, uint64_t want, int p, const char* what) const;

  int rank_, size_, device_;
  size_t cap_;
  double timeout_s_;
  std::string token_;
  std::vector<Peer> peers_;
  void* flags_ = nullptr;  // my flag block: [sender][2] = {sent, done}
  void* flags_dev_ = nullptr;  // its device address (RMA_IPC_STREAM_FLAGS=1)
  size_t flags_bytes_ = 0;
  std::string shm_name_;
  int depth_ = 0;
  std::vector<Op> sends_, recvs_;
};

std::string ipc_shm_name(const std::string& token, int rank);

}  // namespace rma
