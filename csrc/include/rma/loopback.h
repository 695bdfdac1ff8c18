// In-process device transport: N logical ranks = N host threads of one process.
//
// A message is a device-to-device hipMemcpyAsync enqueued on the RECEIVER's
// stream after it waits for an event the sender recorded behind its producer
// kernels; the sender's stream in turn waits for a "consumed" event so the
// send buffer is not overwritten early — the same completion semantics as an
// RCCL send/recv pair inside ncclGroupStart/End. group_end() posts all sends
// before blocking (host side, bounded by a timeout) for its receives, so ring
// and neighbour patterns cannot deadlock. Works on one GPU (several logical
// ranks sharing it) and across GPUs of one process (peer copies over xGMI).
#pragma once

#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <vector>

#include "rma/p2p.h"

namespace rma {

class LoopbackHub {
 public:
  LoopbackHub(int nranks, double timeout_s);
  int size() const { return n_; }
  double timeout() const { return timeout_s_; }

  struct Msg {
    const void* ptr;
    size_t bytes;
    void* ready;     // hipEvent_t recorded on the sender's stream
    std::shared_ptr<void*> consumed;  // hipEvent_t set by the receiver
    std::shared_ptr<bool> consumed_set;
  };
  void post(int src, int dst, Msg m);
  Msg take(int src, int dst);                     // blocks until available
  void wait_consumed(const Msg& m);               // blocks until receiver enqueued the copy
  std::mutex& mu_ref() { return mu_; }
  void notify() { cv_.notify_all(); }
  // next event of `rank`'s pool (created on first use, recycled round-robin
  // after kEventPool; owned by the hub). Only rank's own thread calls this.
  void* event(int rank);
  ~LoopbackHub();
  LoopbackHub(const LoopbackHub&) = delete;
  LoopbackHub& operator=(const LoopbackHub&) = delete;

 private:
  struct Pool {
    std::vector<void*> ev;
    size_t next = 0;
  };
  std::vector<Pool> pools_;  // per rank
  int n_;
  double timeout_s_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::pair<int, int>, std::deque<Msg>> q_;
};

class LoopbackEndpoint : public P2PTransport {
 public:
  LoopbackEndpoint(std::shared_ptr<LoopbackHub> hub, int rank);
  ~LoopbackEndpoint() override;
  int rank() const override { return rank_; }
  int size() const override { return hub_->size(); }
  void group_start() override;
  void group_end() override;
  void send(const void* buf, size_t bytes, int peer, stream_t stream) override;
  void recv(void* buf, size_t bytes, int peer, stream_t stream) override;
  bool capturable() const override { return false; }

 private:
  struct Op {
    void* buf;
    size_t bytes;
    int peer;
    stream_t stream;
  };
  std::shared_ptr<LoopbackHub> hub_;
  int rank_;
  int depth_ = 0;
  std::vector<Op> sends_, recvs_;
};

}  // namespace rma
