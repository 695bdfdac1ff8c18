// HIP IPC transport between processes of one node (rma/ipc.h).
#include "rma/config.h"
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
#include "rma/kernels.h"

namespace rma {

namespace {
hipEvent_t E(void* p) { return reinterpret_cast<hipEvent_t>(p); }
// flag words of sender s in a receiver's block
constexpr int kWords = 4, kSent = 0, kDone = 1, kFull0 = 2;
std::atomic<uint64_t>* flag(void* block, int sender, int which) {
  return reinterpret_cast<std::atomic<uint64_t>*>(block) + kWords * sender + which;
}
uint64_t* dflag(void* dev_block, int sender, int which) {
  return reinterpret_cast<uint64_t*>(dev_block) + kWords * sender + which;
}
size_t page_round(size_t b) { return (b + 4095) / 4096 * 4096; }
void* register_block(void* host, size_t bytes) {
  RMA_HIP_CHECK(hipHostRegister(host, bytes, hipHostRegisterMapped));
  void* d = nullptr;
  RMA_HIP_CHECK(hipHostGetDevicePointer(&d, host, 0));
  return d;
}
IpcTransport::Mode mode_from(int m) {
  if (m == 0) return IpcTransport::Mode::kHost;
  if (m == 1) return IpcTransport::Mode::kStream;
  const char* e = std::getenv("RMA_IPC_MODE");
  if (e && std::strcmp(e, "host") == 0) return IpcTransport::Mode::kHost;
  if (e && *e && std::strcmp(e, "stream") != 0)
    throw_error("RMA_IPC_MODE must be stream or host", __FILE__, __LINE__, e);
  return IpcTransport::Mode::kStream;
}
}  // namespace

std::string ipc_shm_name(const std::string& token, int rank) {
  return "/rma_ipc_" + token + "_" + std::to_string(rank);
}

IpcTransport::IpcTransport(int rank, int size, int device, const std::vector<int>& peers,
                           size_t mailbox_bytes, const std::string& token, double timeout_s,
                           int mode)
    : rank_(rank), size_(size), device_(device), cap_(mailbox_bytes), timeout_s_(timeout_s),
      token_(token), mode_(mode_from(mode)) {
  RMA_CHECK_ARG(size >= 1 && rank >= 0 && rank < size, "rank " << rank << " of " << size);
  RMA_CHECK_ARG(mailbox_bytes >= 8, "mailbox of " << mailbox_bytes << " bytes");
  RMA_CHECK_ARG(!token.empty() && token.size() < 64 &&
                    token.find('/') == std::string::npos,
                "shared-memory token '" << token << "'");
  for (int p : peers) RMA_CHECK_ARG(p < size, "peer " << p << " of " << size);
  // every resource below is released by release() if a later step throws
  // (the destructor does not run for a constructor that throws)
  try {
    RMA_HIP_CHECK(hipSetDevice(device));
    if (mode_ == Mode::kStream) {
      void* e = nullptr;
      RMA_HIP_CHECK(hipHostMalloc(&e, sizeof(uint32_t), hipHostMallocMapped));
      err_host_ = static_cast<uint32_t*>(e);
      *err_host_ = 0;
      void* d = nullptr;
      RMA_HIP_CHECK(hipHostGetDevicePointer(&d, e, 0));
      err_dev_ = static_cast<uint32_t*>(d);
    }
    shm_name_ = ipc_shm_name(token, rank);
    flags_bytes_ = page_round(sizeof(uint64_t) * kWords * (size_t)size);
    const int fd = shm_open(shm_name_.c_str(), O_CREAT | O_RDWR | O_TRUNC, 0600);
    if (fd < 0) throw_error("shm_open failed", __FILE__, __LINE__, shm_name_);
    shm_linked_ = true;
    if (ftruncate(fd, (off_t)flags_bytes_) != 0) {
      close(fd);
      throw_error("ftruncate of the IPC flag block failed", __FILE__, __LINE__, shm_name_);
    }
    void* m = mmap(nullptr, flags_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) throw_error("mmap of the IPC flag block failed", __FILE__, __LINE__, shm_name_);
    flags_ = m;
    for (int s = 0; s < size; ++s)
      for (int w = 0; w < kWords; ++w) flag(flags_, s, w)->store(0);
    if (mode_ == Mode::kStream) flags_dev_ = register_block(flags_, flags_bytes_);
    peers_.resize(size);
    std::vector<int> ps(peers);
    std::sort(ps.begin(), ps.end());
    ps.erase(std::unique(ps.begin(), ps.end()), ps.end());
    for (int p : ps) {
      if (p < 0) continue;
      Peer& P = peers_[p];
      P.rank = p;
      RMA_HIP_CHECK(hipMalloc(&P.mailbox, 2 * cap_));
      if (mode_ == Mode::kHost) {
        hipEvent_t e;
        RMA_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        P.sent_local = e;
        RMA_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        P.done_local = e;
      }
      if (p == rank) {  // periodic self neighbour through the transport: no IPC
        P.r_mailbox = P.mailbox;
        P.r_flags = flags_;
        P.r_flags_dev = flags_dev_;
        P.connected = true;
      }
    }
  } catch (...) {
    release();
    throw;
  }
}

void IpcTransport::release() noexcept {
  (void)hipSetDevice(device_);
  if (!peers_.empty()) (void)hipDeviceSynchronize();
  for (Peer& P : peers_) {
    if (P.rank < 0) continue;
    if (P.rank != rank_) {
      if (P.r_mailbox) (void)hipIpcCloseMemHandle(P.r_mailbox);
      if (P.r_flags_dev) (void)hipHostUnregister(P.r_flags);
      if (P.r_flags) munmap(P.r_flags, flags_bytes_);
    }
    if (P.mailbox) (void)hipFree(P.mailbox);
    if (P.sent_local) (void)hipEventDestroy(E(P.sent_local));
    if (P.done_local) (void)hipEventDestroy(E(P.done_local));
    P = Peer();
  }
  peers_.clear();
  if (flags_) {
    if (flags_dev_) (void)hipHostUnregister(flags_);
    munmap(flags_, flags_bytes_);
    flags_ = flags_dev_ = nullptr;
  }
  if (shm_linked_) {
    shm_unlink(shm_name_.c_str());
    shm_linked_ = false;
  }
  if (err_host_) {
    (void)hipHostFree(err_host_);
    err_host_ = nullptr;
    err_dev_ = nullptr;
  }
}

IpcTransport::~IpcTransport() { release(); }

void IpcTransport::check_error() {
  if (!err_host_) return;
  const uint32_t e = __atomic_load_n(err_host_, __ATOMIC_ACQUIRE);
  if (e == 0) return;
  poisoned_ = true;
  const int p = (int)(e & 0xFFFF) - 1;
  throw_error("IPC transport: a stream wait timed out", __FILE__, __LINE__,
              "rank " + std::to_string(rank_) + " waited " + std::to_string(timeout_s_) +
                  " s for rank " + std::to_string(p) + " (" +
                  ((e >> 16) == 1 ? "empty mailbox slot" : "sent message") +
                  "): peer gone or protocol out of step");
}

void IpcTransport::unlink_shm() {
  if (shm_linked_) {
    shm_unlink(shm_name_.c_str());
    shm_linked_ = false;
  }
}

void IpcTransport::abort_waits() {
  poisoned_ = true;
  if (mode_ != Mode::kStream) return;
  for (const Peer& P : peers_) {
    if (P.rank < 0 || !P.connected) continue;
    for (int k = 0; k < 2; ++k) {
      flag(flags_, P.rank, kFull0 + k)->store(1, std::memory_order_release);
      flag(P.r_flags, rank_, kFull0 + k)->store(0, std::memory_order_release);
    }
  }
}

bool IpcTransport::capturable() const {
  if (mode_ != Mode::kStream) return false;
  static const bool allow = !diag_flag("no_ipc_graph");  // RMA_DIAG no_ipc_graph
  return allow;
}

IpcTransport::Peer& IpcTransport::peer(int p) {
  RMA_CHECK_ARG(p >= 0 && p < size_ && (size_t)p < peers_.size() && peers_[p].rank == p,
                "rank " << p << " is not a peer of the IPC transport of rank " << rank_);
  Peer& P = peers_[p];
  RMA_CHECK_ARG(P.connected, "IPC transport: peer " << p << " not connected");
  return P;
}

std::string IpcTransport::export_for(int p) const {
  RMA_CHECK_ARG(p >= 0 && p < size_ && peers_[p].rank == p, "rank " << p << " is not a peer");
  const Peer& P = peers_[p];
  hipIpcMemHandle_t mh;
  RMA_HIP_CHECK(hipIpcGetMemHandle(&mh, P.mailbox));
  std::string blob(sizeof mh + 2 * sizeof(uint64_t), '\0');
  char* b = &blob[0];
  std::memcpy(b, &mh, sizeof mh);
  const uint64_t meta[2] = {cap_, (uint64_t)mode_};
  std::memcpy(b + sizeof mh, meta, sizeof meta);
  return blob;
}

void IpcTransport::connect(int p, const std::string& blob) {
  RMA_CHECK_ARG(p >= 0 && p < size_ && peers_[p].rank == p, "rank " << p << " is not a peer");
  Peer& P = peers_[p];
  if (P.connected) return;
  hipIpcMemHandle_t mh;
  uint64_t meta[2] = {0, 0};
  RMA_CHECK_ARG(blob.size() == sizeof mh + sizeof meta,
                "IPC export blob of " << blob.size() << " bytes from rank " << p);
  std::memcpy(&mh, blob.data(), sizeof mh);
  std::memcpy(meta, blob.data() + sizeof mh, sizeof meta);
  RMA_CHECK_ARG(meta[0] == cap_, "IPC mailbox sizes differ: rank " << p << " " << meta[0]
                                                                  << ", rank " << rank_ << " "
                                                                  << cap_);
  RMA_CHECK_ARG(meta[1] == (uint64_t)mode_, "IPC modes differ between rank " << p << " and rank "
                                                                         << rank_
                                                                         << " (RMA_IPC_MODE)");
  // the peer's shared-memory block first: it exists only on this node, so a
  // peer on another node fails here, before any IPC handle is opened
  const std::string name = ipc_shm_name(token_, p);
  const int fd = shm_open(name.c_str(), O_RDWR, 0600);
  if (fd < 0)
    throw_error("shm_open of a peer's IPC flag block failed (is the peer on this node?)",
                __FILE__, __LINE__, name);
  void* m = mmap(nullptr, flags_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) throw_error("mmap of a peer's IPC flag block failed", __FILE__, __LINE__, name);
  P.r_flags = m;
  if (mode_ == Mode::kStream) P.r_flags_dev = register_block(m, flags_bytes_);
  RMA_HIP_CHECK(hipIpcOpenMemHandle(&P.r_mailbox, mh, hipIpcMemLazyEnablePeerAccess));
  P.connected = true;
}

bool IpcTransport::connected() const {
  for (const Peer& P : peers_)
    if (P.rank >= 0 && !P.connected) return false;
  return true;
}

void IpcTransport::wait_flag(const void* addr, uint64_t want, int p, const char* what) {
  ++host_waits_;
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
  RMA_CHECK_ARG(!poisoned_, "IPC transport unusable after an earlier error in group_end");
  check_error();
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
  RMA_CHECK_ARG(!poisoned_, "IPC transport unusable after an earlier error in group_end");
  // validate the whole group before any flag, generation or copy: one stream
  // per peer and direction, and every peer's bytes within the mailbox slot
  std::map<int, size_t> out_b, in_b;
  std::map<int, stream_t> out_s, in_s;
  for (const Op& o : sends_) {
    (void)peer(o.peer);
    auto it = out_s.emplace(o.peer, o.stream).first;
    RMA_CHECK_ARG(it->second == o.stream, "IPC transport: one stream per peer and group");
    out_b[o.peer] += o.bytes;
  }
  for (const Op& o : recvs_) {
    (void)peer(o.peer);
    auto it = in_s.emplace(o.peer, o.stream).first;
    RMA_CHECK_ARG(it->second == o.stream, "IPC transport: one stream per peer and group");
    in_b[o.peer] += o.bytes;
  }
  for (const auto& [p, b] : out_b)
    RMA_CHECK_ARG(b <= cap_, "IPC transport: " << b << " bytes to rank " << p
                                               << " in one group exceed the mailbox of " << cap_
                                               << " (RMA_IPC_MAILBOX_MB)");
  for (const auto& [p, b] : in_b)
    RMA_CHECK_ARG(b <= cap_, "IPC transport: " << b << " bytes from rank " << p
                                               << " in one group exceed the mailbox of " << cap_
                                               << " (RMA_IPC_MAILBOX_MB)");
  try {
    enqueue_group();
  } catch (...) {
    // a peer may already have seen part of this group: the protocol is out of step
    poisoned_ = true;
    sends_.clear();
    recvs_.clear();
    throw;
  }
  sends_.clear();
  recvs_.clear();
}

void IpcTransport::enqueue_group() {
  // per peer, in issue order (the n-th send to p matches p's n-th recv from me)
  std::map<int, std::vector<const Op*>> out, in;
  for (const Op& o : sends_) out[o.peer].push_back(&o);
  for (const Op& o : recvs_) in[o.peer].push_back(&o);
  // sends first: a rank's sends of generation g wait only for its peers'
  // receives of g - 2 (completed group calls), its receives for the peers'
  // sends of g, which they publish before waiting for anything of this group
  for (auto& [p, ops] : out) {
    Peer& P = peer(p);
    hipStream_t s = as_stream(ops.front()->stream);
    const uint64_t g = ++P.send_gen;
    const int slot = (int)(g & 1);
    if (mode_ == Mode::kStream) {  // slot empty -> copies -> slot full, all on the GPU
      flag_wait_gpu(dflag(P.r_flags_dev, rank_, kFull0 + slot), 0, timeout_s_, err_dev_,
                    (1u << 16) | (uint32_t)(p + 1), s);
    } else if (g > 2) {  // slot g % 2 was last read by the peer's receive of g - 2
      wait_flag(flag(P.r_flags, rank_, kDone), g - 2, p, "receive done");
    }
    char* dst = static_cast<char*>(P.r_mailbox) + slot * cap_;
    size_t off = 0;
    for (const Op* o : ops) {
      if (o->bytes)
        RMA_HIP_CHECK(hipMemcpyAsync(dst + off, o->buf, o->bytes, hipMemcpyDeviceToDevice, s));
      off += o->bytes;
    }
    if (mode_ == Mode::kStream) {
      flag_write_gpu(dflag(P.r_flags_dev, rank_, kFull0 + slot), 1, s);
      continue;
    }
    RMA_HIP_CHECK(hipEventRecord(E(P.sent_local), s));
    ++host_waits_;
    RMA_HIP_CHECK(hipEventSynchronize(E(P.sent_local)));
    flag(P.r_flags, rank_, kSent)->store(g, std::memory_order_release);
  }
  for (auto& [p, ops] : in) {
    Peer& P = peer(p);
    hipStream_t s = as_stream(ops.front()->stream);
    const uint64_t g = ++P.recv_gen;
    const int slot = (int)(g & 1);
    if (mode_ == Mode::kStream)
      flag_wait_gpu(dflag(flags_dev_, p, kFull0 + slot), 1, timeout_s_, err_dev_,
                    (2u << 16) | (uint32_t)(p + 1), s);
    else
      wait_flag(flag(flags_, p, kSent), g, p, "send");
    const char* src = static_cast<const char*>(P.mailbox) + slot * cap_;
    size_t off = 0;
    for (const Op* o : ops) {
      if (o->bytes)
        RMA_HIP_CHECK(hipMemcpyAsync(o->buf, src + off, o->bytes, hipMemcpyDeviceToDevice, s));
      off += o->bytes;
    }
    if (mode_ == Mode::kStream) {
      flag_write_gpu(dflag(flags_dev_, p, kFull0 + slot), 0, s);
      continue;
    }
    RMA_HIP_CHECK(hipEventRecord(E(P.done_local), s));
    ++host_waits_;
    RMA_HIP_CHECK(hipEventSynchronize(E(P.done_local)));
    flag(flags_, p, kDone)->store(g, std::memory_order_release);
  }
}

namespace {
struct IpcExport {
  hipIpcMemHandle_t h;
  uint64_t offset, bytes, pid, base, magic;  // base: the allocation in the exporter
};
constexpr uint64_t kIpcExportMagic = 0x524d41495043ULL;  // "RMAIPC"
}  // namespace

std::string IpcMap::export_ptr(const void* p) {
  RMA_CHECK_ARG(p != nullptr, "IPC export of a null pointer");
  void* base = nullptr;
  size_t bytes = 0;
  RMA_HIP_CHECK(hipMemGetAddressRange(&base, &bytes, const_cast<void*>(p)));
  IpcExport e{};
  RMA_HIP_CHECK(hipIpcGetMemHandle(&e.h, base));
  e.offset = (uint64_t)((const char*)p - (const char*)base);
  e.bytes = bytes;
  e.pid = (uint64_t)getpid();
  e.base = (uint64_t)(uintptr_t)base;
  e.magic = kIpcExportMagic;
  return std::string(reinterpret_cast<const char*>(&e), sizeof e);
}

void* IpcMap::open(const std::string& blob) {
  IpcExport e{};
  RMA_CHECK_ARG(blob.size() == sizeof e, "IPC pointer export of " << blob.size() << " bytes");
  std::memcpy(&e, blob.data(), sizeof e);
  RMA_CHECK_ARG(e.magic == kIpcExportMagic && e.offset < e.bytes, "not an IpcMap export");
  RMA_CHECK_ARG(e.pid != (uint64_t)getpid(),
                "IPC pointer export of this process: use the pointer itself");
  // one mapping per exporter allocation (two exports of one allocation need
  // not carry identical handle bytes)
  const std::string key = std::to_string(e.pid) + ":" + std::to_string(e.base);
  for (const Mapping& m : maps_)
    if (m.key == key) return static_cast<char*>(m.base) + e.offset;
  void* base = nullptr;
  RMA_HIP_CHECK(hipIpcOpenMemHandle(&base, e.h, hipIpcMemLazyEnablePeerAccess));
  maps_.push_back({key, base, (size_t)e.bytes});
  return static_cast<char*>(base) + e.offset;
}

void IpcMap::close_all() noexcept {
  for (const Mapping& m : maps_) (void)hipIpcCloseMemHandle(m.base);
  maps_.clear();
}

IpcMap::~IpcMap() { close_all(); }

}  // namespace rma
