// HIP IPC transport between processes of one node (rma/ipc.h).
#include "rma/ipc.h"

#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <thread>

#include "rma/hip_check.h"

namespace rma {

namespace {
hipEvent_t E(void* p) { return reinterpret_cast<hipEvent_t>(p); }
std::atomic<uint64_t>* slot_flag(void* block, int sender, int which) {
  return reinterpret_cast<std::atomic<uint64_t>*>(block) + 2 * sender + which;
}
constexpr int kSent = 0, kDone = 1;
// Default: the sender waits on the host for its own copies (its own event)
// before it publishes a generation, the receiver for its own copies before it
// frees the slot, so no process ever waits on an event it opened from another
// one. RMA_IPC_GPU_EVENTS=1 instead makes the streams wait on the peers'
// interprocess events (no host blocking); on the HIP 7.0 runtime in torch that
// hipStreamWaitEvent on an opened event fails intermittently with "invalid
// argument" (bench/ipc_transport_probe.py, profiles/SUMMARY_r4.md §9).
bool host_sync() {
  static const bool v = [] {
    const char* e = std::getenv("RMA_IPC_GPU_EVENTS");
    return !(e && e[0] == '1');
  }();
  return v;
}
// RMA_IPC_STREAM_FLAGS=1: the flags are written by the GPU, in stream order
// after the copies (hipStreamWriteValue64 into the shared-memory block,
// registered with hipHostRegister in every process that writes it), so the
// sender's host never waits for its copies; the receiver's host still polls
// for the sender's flag before it enqueues its copies
bool stream_flags() {
  static const bool v = [] {
    const char* e = std::getenv("RMA_IPC_STREAM_FLAGS");
    return e && e[0] == '1';
  }();
  return v;
}
size_t page_round(size_t b) { return (b + 4095) / 4096 * 4096; }
void* register_block(void* host, size_t bytes) {
  RMA_HIP_CHECK(hipHostRegister(host, bytes, hipHostRegisterMapped));
  void* d = nullptr;
  RMA_HIP_CHECK(hipHostGetDevicePointer(&d, host, 0));
  return d;
}
}  // namespace

std::string ipc_shm_name(const std::string& token, int rank) {
  return "/rma_ipc_" + token + "_" + std::to_string(rank);
}

IpcTransport::IpcTransport(int rank, int size, int device, const std::vector<int>& peers,
                           size_t mailbox_bytes, const std::string& token, double timeout_s)
    : rank_(rank), size_(size), device_(device), cap_(mailbox_bytes), timeout_s_(timeout_s),
      token_(token) {
  RMA_CHECK_ARG(size >= 1 && rank >= 0 && rank < size, "rank " << rank << " of " << size);
  RMA_CHECK_ARG(mailbox_bytes >= 8, "mailbox of " << mailbox_bytes << " bytes");
  RMA_CHECK_ARG(!token.empty() && token.size() < 64 &&
                    token.find('/') == std::string::npos,
                "shared-memory token '" << token << "'");
  RMA_HIP_CHECK(hipSetDevice(device));
  // my flag block: per sender {sent generation, done generation}
  shm_name_ = ipc_shm_name(token, rank);
  flags_bytes_ = page_round(sizeof(uint64_t) * 2 * (size_t)size);
  const int fd = shm_open(shm_name_.c_str(), O_CREAT | O_RDWR | O_TRUNC, 0600);
  if (fd < 0) throw_error("shm_open failed", __FILE__, __LINE__, shm_name_);
  if (ftruncate(fd, (off_t)flags_bytes_) != 0) {
    close(fd);
    throw_error("ftruncate of the IPC flag block failed", __FILE__, __LINE__, shm_name_);
  }
  flags_ = mmap(nullptr, flags_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (flags_ == MAP_FAILED) {
    flags_ = nullptr;
    throw_error("mmap of the IPC flag block failed", __FILE__, __LINE__, shm_name_);
  }
  for (int s = 0; s < size; ++s) {
    slot_flag(flags_, s, kSent)->store(0);
    slot_flag(flags_, s, kDone)->store(0);
  }
  if (stream_flags()) flags_dev_ = register_block(flags_, flags_bytes_);
  peers_.resize(size);
  std::vector<int> ps(peers);
  std::sort(ps.begin(), ps.end());
  ps.erase(std::unique(ps.begin(), ps.end()), ps.end());
  for (int p : ps) {
    if (p < 0) continue;
    RMA_CHECK_ARG(p < size, "peer " << p << " of " << size);
    Peer& P = peers_[p];
    P.rank = p;
    RMA_HIP_CHECK(hipMalloc(&P.mailbox, 2 * cap_));
    hipEvent_t e;
    RMA_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventInterprocess | hipEventDisableTiming));
    P.done_ev = e;
    RMA_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventInterprocess | hipEventDisableTiming));
    P.sent_ev = e;
    RMA_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    P.sent_local = e;
    RMA_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    P.done_local = e;
    if (p == rank) {  // periodic self neighbour through the transport: no IPC
      P.r_mailbox = P.mailbox;
      P.r_done_ev = P.done_ev;
      P.r_sent_ev = P.sent_ev;
      P.r_flags = flags_;
      P.r_flags_dev = flags_dev_;
      P.connected = true;
    }
  }
}

IpcTransport::~IpcTransport() {
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  for (Peer& P : peers_) {
    if (P.rank < 0) continue;
    if (P.rank != rank_) {
      if (P.r_mailbox) (void)hipIpcCloseMemHandle(P.r_mailbox);
      if (P.r_done_ev) (void)hipEventDestroy(E(P.r_done_ev));
      if (P.r_sent_ev) (void)hipEventDestroy(E(P.r_sent_ev));
      if (P.r_flags_dev) (void)hipHostUnregister(P.r_flags);
      if (P.r_flags) munmap(P.r_flags, flags_bytes_);
    }
    if (P.mailbox) (void)hipFree(P.mailbox);
    if (P.done_ev) (void)hipEventDestroy(E(P.done_ev));
    if (P.sent_ev) (void)hipEventDestroy(E(P.sent_ev));
    if (P.sent_local) (void)hipEventDestroy(E(P.sent_local));
    if (P.done_local) (void)hipEventDestroy(E(P.done_local));
  }
  if (flags_) {
    if (flags_dev_) (void)hipHostUnregister(flags_);
    munmap(flags_, flags_bytes_);
    shm_unlink(shm_name_.c_str());
  }
}

IpcTransport::Peer& IpcTransport::peer(int p) {
  RMA_CHECK_ARG(p >= 0 && p < size_ && peers_[p].rank == p,
                "rank " << p << " is not a peer of the IPC transport of rank " << rank_);
  Peer& P = peers_[p];
  RMA_CHECK_ARG(P.connected, "IPC transport: peer " << p << " not connected");
  return P;
}

std::string IpcTransport::export_for(int p) const {
  RMA_CHECK_ARG(p >= 0 && p < size_ && peers_[p].rank == p, "rank " << p << " is not a peer");
  const Peer& P = peers_[p];
  hipIpcMemHandle_t mh;
  hipIpcEventHandle_t dh, sh;
  RMA_HIP_CHECK(hipIpcGetMemHandle(&mh, P.mailbox));
  RMA_HIP_CHECK(hipIpcGetEventHandle(&dh, E(P.done_ev)));
  RMA_HIP_CHECK(hipIpcGetEventHandle(&sh, E(P.sent_ev)));
  std::string blob(sizeof mh + sizeof dh + sizeof sh + sizeof(uint64_t), '\0');
  char* b = &blob[0];
  std::memcpy(b, &mh, sizeof mh);
  std::memcpy(b + sizeof mh, &dh, sizeof dh);
  std::memcpy(b + sizeof mh + sizeof dh, &sh, sizeof sh);
  const uint64_t cap = cap_;
  std::memcpy(b + sizeof mh + sizeof dh + sizeof sh, &cap, sizeof cap);
  return blob;
}

void IpcTransport::connect(int p, const std::string& blob) {
  RMA_CHECK_ARG(p >= 0 && p < size_ && peers_[p].rank == p, "rank " << p << " is not a peer");
  Peer& P = peers_[p];
  if (P.connected) return;
  hipIpcMemHandle_t mh;
  hipIpcEventHandle_t dh, sh;
  uint64_t cap = 0;
  RMA_CHECK_ARG(blob.size() == sizeof mh + sizeof dh + sizeof sh + sizeof cap,
                "IPC export blob of " << blob.size() << " bytes from rank " << p);
  const char* b = blob.data();
  std::memcpy(&mh, b, sizeof mh);
  std::memcpy(&dh, b + sizeof mh, sizeof dh);
  std::memcpy(&sh, b + sizeof mh + sizeof dh, sizeof sh);
  std::memcpy(&cap, b + sizeof mh + sizeof dh + sizeof sh, sizeof cap);
  RMA_CHECK_ARG(cap == cap_, "IPC mailbox sizes differ: rank " << p << " " << cap << ", rank "
                                                               << rank_ << " " << cap_);
  RMA_HIP_CHECK(hipIpcOpenMemHandle(&P.r_mailbox, mh, hipIpcMemLazyEnablePeerAccess));
  hipEvent_t e;
  RMA_HIP_CHECK(hipIpcOpenEventHandle(&e, dh));
  P.r_done_ev = e;
  RMA_HIP_CHECK(hipIpcOpenEventHandle(&e, sh));
  P.r_sent_ev = e;
  const std::string name = ipc_shm_name(token_, p);
  const int fd = shm_open(name.c_str(), O_RDWR, 0600);
  if (fd < 0) throw_error("shm_open of a peer's IPC flag block failed", __FILE__, __LINE__, name);
  void* m = mmap(nullptr, flags_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) throw_error("mmap of a peer's IPC flag block failed", __FILE__, __LINE__, name);
  P.r_flags = m;
  if (stream_flags()) P.r_flags_dev = register_block(m, flags_bytes_);
  P.connected = true;
}

bool IpcTransport::connected() const {
  for (const Peer& P : peers_)
    if (P.rank >= 0 && !P.connected) return false;
  return true;
}

void IpcTransport::wait_flag(const void* addr, uint64_t want, int p, const char* what) const {
  auto* f = reinterpret_cast<const std::atomic<uint64_t>*>(addr);
  if (f->load(std::memory_order_acquire) >= want) return;
  const auto t0 = std::chrono::steady_clock::now();
  int spins = 0;
  while (f->load(std::memory_order_acquire) < want) {
    if (++spins < 1000) continue;
    std::this_thread::sleep_for(std::chrono::microseconds(spins < 20000 ? 1 : 50));
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() >
        timeout_s_)
      throw_error("IPC transport timed out", __FILE__, __LINE__,
                  "rank " + std::to_string(rank_) + " waiting for rank " + std::to_string(p) +
                      " (" + what + " of generation " + std::to_string(want) + ")");
  }
}

void IpcTransport::group_start() {
  if (depth_++ == 0) {
    sends_.clear();
    recvs_.clear();
  }
}

void IpcTransport::send(const void* buf, size_t bytes, int peer_rank, stream_t stream) {
  (void)peer(peer_rank);
  const bool solo = depth_ == 0;
  if (solo) group_start();
  sends_.push_back({const_cast<void*>(buf), bytes, peer_rank, stream});
  if (solo) group_end();
}

void IpcTransport::recv(void* buf, size_t bytes, int peer_rank, stream_t stream) {
  (void)peer(peer_rank);
  const bool solo = depth_ == 0;
  if (solo) group_start();
  recvs_.push_back({buf, bytes, peer_rank, stream});
  if (solo) group_end();
}

void IpcTransport::group_end() {
  RMA_CHECK_ARG(depth_ > 0, "group_end without group_start");
  if (--depth_ > 0) return;
  // per peer, in issue order (the n-th send to p matches p's n-th recv from me)
  std::map<int, std::vector<const Op*>> out, in;
  for (const Op& o : sends_) out[o.peer].push_back(&o);
  for (const Op& o : recvs_) in[o.peer].push_back(&o);
  const bool hs = host_sync();
  // sends first: a rank's sends of generation g wait only for its peers'
  // receives of g - 2 (completed group calls), its receives for the peers'
  // sends of g, which they publish before waiting for anything of this group
  for (auto& [p, ops] : out) {
    Peer& P = peer(p);
    hipStream_t s = as_stream(ops.front()->stream);
    size_t total = 0;
    for (const Op* o : ops) {
      RMA_CHECK_ARG(as_stream(o->stream) == s, "IPC transport: one stream per peer and group");
      total += o->bytes;
    }
    RMA_CHECK_ARG(total <= cap_, "IPC transport: " << total << " bytes to rank " << p
                                                   << " in one group exceed the mailbox of "
                                                   << cap_ << " (RMA_IPC_MAILBOX_MB)");
    const uint64_t g = ++P.send_gen;
    if (g > 2) {  // slot g % 2 was last read by the peer's receive of g - 2
      wait_flag(slot_flag(P.r_flags, rank_, kDone), g - 2, p, "receive done");
      if (!hs && !P.r_flags_dev) RMA_HIP_CHECK(hipStreamWaitEvent(s, E(P.r_done_ev), 0));
    }
    char* dst = static_cast<char*>(P.r_mailbox) + (g & 1) * cap_;
    size_t off = 0;
    for (const Op* o : ops) {
      if (o->bytes)
        RMA_HIP_CHECK(hipMemcpyAsync(dst + off, o->buf, o->bytes, hipMemcpyDeviceToDevice, s));
      off += o->bytes;
    }
    if (P.r_flags_dev) {  // the GPU publishes g once the copies are done
      RMA_HIP_CHECK(hipStreamWriteValue64(
          s, slot_flag(P.r_flags_dev, rank_, kSent), g, 0));
      continue;
    }
    if (hs) {
      RMA_HIP_CHECK(hipEventRecord(E(P.sent_local), s));
      RMA_HIP_CHECK(hipEventSynchronize(E(P.sent_local)));
    } else {
      RMA_HIP_CHECK(hipEventRecord(E(P.sent_ev), s));
    }
    slot_flag(P.r_flags, rank_, kSent)->store(g, std::memory_order_release);
  }
  for (auto& [p, ops] : in) {
    Peer& P = peer(p);
    hipStream_t s = as_stream(ops.front()->stream);
    size_t total = 0;
    for (const Op* o : ops) {
      RMA_CHECK_ARG(as_stream(o->stream) == s, "IPC transport: one stream per peer and group");
      total += o->bytes;
    }
    RMA_CHECK_ARG(total <= cap_, "IPC transport: " << total << " bytes from rank " << p
                                                   << " in one group exceed the mailbox of "
                                                   << cap_ << " (RMA_IPC_MAILBOX_MB)");
    const uint64_t g = ++P.recv_gen;
    wait_flag(slot_flag(flags_, p, kSent), g, p, "send");
    if (!hs && !flags_dev_) RMA_HIP_CHECK(hipStreamWaitEvent(s, E(P.r_sent_ev), 0));
    const char* src = static_cast<const char*>(P.mailbox) + (g & 1) * cap_;
    size_t off = 0;
    for (const Op* o : ops) {
      if (o->bytes)
        RMA_HIP_CHECK(hipMemcpyAsync(o->buf, src + off, o->bytes, hipMemcpyDeviceToDevice, s));
      off += o->bytes;
    }
    if (flags_dev_) {  // the GPU frees the slot once the copies are done
      RMA_HIP_CHECK(hipStreamWriteValue64(s, slot_flag(flags_dev_, p, kDone), g, 0));
      continue;
    }
    if (hs) {
      RMA_HIP_CHECK(hipEventRecord(E(P.done_local), s));
      RMA_HIP_CHECK(hipEventSynchronize(E(P.done_local)));
    } else {
      RMA_HIP_CHECK(hipEventRecord(E(P.done_ev), s));
    }
    slot_flag(flags_, p, kDone)->store(g, std::memory_order_release);
  }
  sends_.clear();
  recvs_.clear();
}

}  // namespace rma
