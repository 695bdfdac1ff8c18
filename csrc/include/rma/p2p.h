// Point-to-point transport interface used by the halo engine.
//
// Implementations:
//   * RcclComm         — GPU-direct RCCL over xGMI (production, one process per GPU);
//   * LoopbackEndpoint — N logical ranks as threads of ONE process, messages are
//                        device-to-device hipMemcpyAsync ordered by events. On one
//                        GPU it lets the full multi-rank native path (halo engine +
//                        overlapped executor) be tested on a single MI355X; across
//                        GPUs of one process the copies go peer-to-peer over xGMI.
// Semantics follow ncclGroupStart/End: sends and receives issued between
// group_start() and group_end() form one group; messages between a pair of
// ranks match in issue order.
#pragma once

#include <cstddef>

#include "rma/kernels.h"

namespace rma {

class P2PTransport {
 public:
  virtual ~P2PTransport() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual void group_start() = 0;
  virtual void group_end() = 0;
  virtual void send(const void* buf, size_t bytes, int peer, stream_t stream) = 0;
  virtual void recv(void* buf, size_t bytes, int peer, stream_t stream) = 0;
  // Can a group be recorded by hipStreamBeginCapture and replayed later?
  // (RCCL: yes; the loopback transport synchronises on the host: no.)
  virtual bool capturable() const { return true; }
};

}  // namespace rma
