// Device-direct transport between PROCESSES of one node without RCCL: HIP IPC.
//
// The reference moves halos between ranks with ROCm-aware MPI, i.e. device
// buffers handed to MPI_Send/Recv (scripts/rocmaware_test_selectdevice.jl:16-22,
// ImplicitGlobalGrid's update_halo! with IGG_ROCMAWARE_MPI=1); inside a node
// the MPI library moves those bytes through CUDA/HIP IPC. This transport does
// the same natively: every receiver owns, per sender, a double-buffered device
// MAILBOX that the sender maps with hipIpcOpenMemHandle and fills with one
// device-to-device copy per message on its own stream (over xGMI when the
// ranks drive different GPUs, on-device when they share one). The handshake
// flags of a (sender, receiver) pair live in the receiver's POSIX
// shared-memory block, mapped by both. Two modes (RMA_IPC_MODE):
//
//   * stream (default): nothing waits on the host. Per mailbox slot a
//     full/empty flag; the sender's stream waits for "empty" (a one-wave
//     kernel polling the flag, host-registered and mapped for the GPU,
//     csrc/kernels/flags.hip), copies, and writes "full" (a one-wave kernel,
//     system-scope release) behind its copies; the receiver's stream waits
//     for "full", copies the slot out and writes "empty". group_end() only
//     enqueues. The protocol carries no generation number and the waits are
//     kernels, so a captured exchange replays like any other kernel node
//     (HIP's own hipStreamWaitValue64 / WriteValue64 replayed to a wrong
//     field once captured, profiles/r5/ipc_graph_replay_failure.log). A wait
//     is bounded: after timeout_s it records which peer it waited for in an
//     error word (pinned host memory) and exits; the next group or
//     check_error() raises.
//   * host: the round-4 validation mode. Per pair a generation counter; the
//     sender waits (host, bounded) until the receiver published "done with
//     g-2", copies into slot g%2, waits for its own copies (a local event),
//     publishes g; the receiver waits for g, copies out, waits for its own
//     copies, publishes g. Timeouts name the peer.
//
// A group is validated as a whole before any flag or generation changes (a
// mailbox overflow leaves the transport consistent); an error in the middle
// of enqueueing poisons the transport (every later call throws), since the
// peers' view of the protocol may then be out of step. Flags live in one
// shared-memory block per receiver; unlink_shm() removes its name once every
// peer has connected (comm.py IpcComm does it after a barrier), so a crashed
// job leaves nothing in /dev/shm. Not stream-capturable in host mode.
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
  enum class Mode : int { kHost = 0, kStream = 1 };
  // token: job-unique name part of the shared-memory blocks; mailbox_bytes:
  // capacity of ONE slot per sender (the bytes of one group to one peer);
  // mode -1: RMA_IPC_MODE (stream | host), default stream
  IpcTransport(int rank, int size, int device, const std::vector<int>& peers,
               size_t mailbox_bytes, const std::string& token, double timeout_s, int mode = -1);
  ~IpcTransport() override;
  IpcTransport(const IpcTransport&) = delete;
  IpcTransport& operator=(const IpcTransport&) = delete;

  // what peer p needs from me: my mailbox for p's messages (opaque bytes)
  std::string export_for(int peer) const;
  // open what peer p exported for me (and p's shared-memory flag block)
  void connect(int peer, const std::string& blob);
  bool connected() const;
  // remove the name of my flag block (mappings stay valid): call once every
  // peer has connected
  void unlink_shm();
  // stream mode, teardown after a peer died: satisfy every GPU-side wait of
  // this rank from the host (its receives see "full", its sends "empty"), so
  // its streams drain instead of waiting forever for a dead peer's flags. The
  // data then received is garbage; the transport is poisoned.
  void abort_waits();

  int rank() const override { return rank_; }
  int size() const override { return size_; }
  void group_start() override;
  void group_end() override;
  void send(const void* buf, size_t bytes, int peer, stream_t stream) override;
  void recv(void* buf, size_t bytes, int peer, stream_t stream) override;
  // stream mode: kernels and copies only (RMA_DIAG=no_ipc_graph refuses capture)
  bool capturable() const override;
  // raise if a stream-mode wait timed out (peer gone or protocol out of step)
  void check_error();
  size_t mailbox_bytes() const { return cap_; }
  Mode mode() const { return mode_; }
  bool poisoned() const { return poisoned_; }
  // host waits inside group_end() so far (host mode: two per peer and group;
  // stream mode: 0)
  uint64_t host_waits() const { return host_waits_; }

 private:
  struct Op {
    void* buf;
    size_t bytes;
    int peer;
    stream_t stream;
  };
  struct Peer {
    int rank = -1;
    void* mailbox = nullptr;     // mine: 2 slots for this peer's messages
    void* sent_local = nullptr;  // host mode: my copies to this peer done
    void* done_local = nullptr;  // host mode: my copies out of its slot done
    void* r_mailbox = nullptr;   // the peer's, opened: its mailbox for my messages
    void* r_flags = nullptr;     // the peer's shared-memory flag block (mapped)
    void* r_flags_dev = nullptr;  // ... registered for the GPU (stream mode)
    uint64_t send_gen = 0, recv_gen = 0;
    bool connected = false;
  };
  Peer& peer(int p);
  void wait_flag(const void* addr, uint64_t want, int p, const char* what);
  void release() noexcept;
  void enqueue_group();

  int rank_, size_, device_;
  size_t cap_;
  double timeout_s_;
  std::string token_;
  Mode mode_;
  std::vector<Peer> peers_;
  void* flags_ = nullptr;      // my flag block: [sender][4] = {sent, done, full0, full1}
  void* flags_dev_ = nullptr;  // its device address (stream mode)
  uint32_t* err_host_ = nullptr;  // stream mode: wait-timeout word (pinned, mapped)
  uint32_t* err_dev_ = nullptr;
  size_t flags_bytes_ = 0;
  std::string shm_name_;
  bool shm_linked_ = false;
  int depth_ = 0;
  bool poisoned_ = false;
  uint64_t host_waits_ = 0;
  std::vector<Op> sends_, recvs_;
};

std::string ipc_shm_name(const std::string& token, int rank);

// Device memory of other processes of this node, mapped into this one
// (direct-store halos, DiffusionExecutor::set_direct: a neighbour's T / T2
// and its pass-count words, so this rank's kernels store straight into them
// -- on-device when the ranks share a GPU, over xGMI between GPUs).
// export_ptr(p): the IPC handle of p's allocation (hipMemGetAddressRange:
// torch's caching allocator hands out pieces of larger hipMalloc segments)
// plus p's offset in it and the creating process id; open(blob): p in this
// process. A handle is opened once however many pointers into its
// allocation are asked for (a peer that is two of my neighbours); the
// destructor closes every mapping, so it must outlive every kernel that
// stores through them.
class IpcMap {
 public:
  IpcMap() = default;
  ~IpcMap();
  IpcMap(const IpcMap&) = delete;
  IpcMap& operator=(const IpcMap&) = delete;
  static std::string export_ptr(const void* p);
  void* open(const std::string& blob);
  size_t mappings() const { return maps_.size(); }
  void close_all() noexcept;

 private:
  struct Mapping {
    std::string key;  // exporter pid : allocation base
    void* base;
    size_t bytes;
  };
  std::vector<Mapping> maps_;
};

}  // namespace rma
