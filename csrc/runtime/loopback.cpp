#include "rma/loopback.h"

#include <hip/hip_runtime.h>

#include <chrono>

#include "rma/hip_check.h"

namespace rma {

namespace {
constexpr size_t kPool = 4096;
hipEvent_t E(void* p) { return reinterpret_cast<hipEvent_t>(p); }
}  // namespace

LoopbackHub::LoopbackHub(int nranks, double timeout_s)
    : pools_(nranks > 0 ? (size_t)nranks : 0), n_(nranks), timeout_s_(timeout_s) {
  RMA_CHECK_ARG(nranks >= 1, "nranks=" << nranks);
}

LoopbackHub::~LoopbackHub() {
  for (Pool& p : pools_)
    for (void* e : p.ev) (void)hipEventDestroy(E(e));
}

void* LoopbackHub::event(int rank) {
  Pool& p = pools_[(size_t)rank];
  if (p.ev.size() < kPool) {
    hipEvent_t e;
    RMA_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    p.ev.push_back(e);
    return e;
  }
  void* e = p.ev[p.next];
  p.next = (p.next + 1) % kPool;
  return e;
}

void LoopbackHub::post(int src, int dst, Msg m) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    q_[{src, dst}].push_back(std::move(m));
  }
  cv_.notify_all();
}

LoopbackHub::Msg LoopbackHub::take(int src, int dst) {
  std::unique_lock<std::mutex> lk(mu_);
  auto& q = q_[{src, dst}];
  const auto deadline = std::chrono::steady_clock::now() +
                        std::chrono::duration<double>(timeout_s_);
  while (q.empty()) {
    if (cv_.wait_until(lk, deadline) == std::cv_status::timeout && q.empty())
      throw_error("loopback receive timed out", __FILE__, __LINE__,
                  "rank " + std::to_string(dst) + " waiting for rank " + std::to_string(src));
  }
  Msg m = std::move(q.front());
  q.pop_front();
  return m;
}

void LoopbackHub::wait_consumed(const Msg& m) {
  std::unique_lock<std::mutex> lk(mu_);
  const auto deadline = std::chrono::steady_clock::now() +
                        std::chrono::duration<double>(timeout_s_);
  while (!*m.consumed_set) {
    if (cv_.wait_until(lk, deadline) == std::cv_status::timeout && !*m.consumed_set)
      throw_error("loopback send timed out", __FILE__, __LINE__,
                  "message was never received (peer gone?)");
  }
}

LoopbackEndpoint::LoopbackEndpoint(std::shared_ptr<LoopbackHub> hub, int rank)
    : hub_(std::move(hub)), rank_(rank) {
  RMA_CHECK_ARG(rank >= 0 && rank < hub_->size(), "rank " << rank);
}

// The events this endpoint recorded stay alive in the hub (see loopback.h):
// a peer may still wait on the last "consumed" event after we are gone.
LoopbackEndpoint::~LoopbackEndpoint() = default;

void LoopbackEndpoint::group_start() {
  if (depth_++ == 0) {
    sends_.clear();
    recvs_.clear();
  }
}

void LoopbackEndpoint::send(const void* buf, size_t bytes, int peer, stream_t stream) {
  RMA_CHECK_ARG(peer >= 0 && peer < hub_->size(), "peer " << peer);
  sends_.push_back({const_cast<void*>(buf), bytes, peer, stream});
  if (depth_ == 0) group_end();
}

void LoopbackEndpoint::recv(void* buf, size_t bytes, int peer, stream_t stream) {
  RMA_CHECK_ARG(peer >= 0 && peer < hub_->size(), "peer " << peer);
  recvs_.push_back({buf, bytes, peer, stream});
  if (depth_ == 0) group_end();
}

void LoopbackEndpoint::group_end() {
  if (depth_ > 0 && --depth_ > 0) return;
  std::vector<LoopbackHub::Msg> posted;
  // 1. post every send (ready event behind the producer work on its stream)
  for (const auto& s : sends_) {
    void* ev = hub_->event(rank_);
    RMA_HIP_CHECK(hipEventRecord(E(ev), as_stream(s.stream)));
    LoopbackHub::Msg m{s.buf, s.bytes, ev, std::make_shared<void*>(nullptr),
                       std::make_shared<bool>(false)};
    posted.push_back(m);
    hub_->post(rank_, s.peer, m);
  }
  // 2. receive: wait for the sender's event, copy, publish "consumed"
  for (const auto& r : recvs_) {
    LoopbackHub::Msg m = hub_->take(r.peer, rank_);
    RMA_CHECK_ARG(m.bytes == r.bytes, "loopback size mismatch: sent " << m.bytes << " B, expected "
                                                                      << r.bytes << " B");
    hipStream_t s = as_stream(r.stream);
    RMA_HIP_CHECK(hipStreamWaitEvent(s, E(m.ready), 0));
    RMA_HIP_CHECK(hipMemcpyAsync(r.buf, m.ptr, r.bytes, hipMemcpyDefault, s));
    void* done = hub_->event(rank_);
    RMA_HIP_CHECK(hipEventRecord(E(done), s));
    {
      std::lock_guard<std::mutex> lk(hub_->mu_ref());
      *m.consumed = done;
      *m.consumed_set = true;
    }
    hub_->notify();
  }
  // 3. a send completes when its receiver's copy has run (RCCL semantics)
  for (size_t i = 0; i < sends_.size(); ++i) {
    hub_->wait_consumed(posted[i]);
    RMA_HIP_CHECK(hipStreamWaitEvent(as_stream(sends_[i].stream), E(*posted[i].consumed), 0));
  }
  sends_.clear();
  recvs_.clear();
}

}  // namespace rma
