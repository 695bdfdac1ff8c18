#include "rma/config.h"
#include "rma/halo.h"

#include <hip/hip_runtime.h>

#include <cstdlib>

#include "rma/hip_check.h"
#include "rma/kernels.h"
#include "rma/topology.h"

namespace rma {

HaloExchanger::HaloExchanger(P2PTransport* comm, int self_rank,
                             std::array<std::array<int, 2>, 3> neighbors)
    : comm_(comm), self_(self_rank), nbr_(neighbors) {
  for (int d = 0; d < 3; ++d)
    for (int s = 0; s < 2; ++s) {
      const int p = nbr_[d][s];
      RMA_CHECK_ARG(p == kProcNull || p >= 0, "bad neighbour " << p);
      RMA_CHECK_ARG(p < 0 || p == self_ || comm_ != nullptr,
                    "remote neighbour " << p << " but no communicator");
    }
}

HaloExchanger::~HaloExchanger() {
  for (void* p : bufs_)
    if (p) (void)hipFree(p);
  for (void* p : retired_) (void)hipFree(p);
}

bool HaloExchanger::active(int dim) const { return nbr_[dim][0] >= 0 || nbr_[dim][1] >= 0; }

void* HaloExchanger::buffer(size_t slot, size_t bytes) {
  if (slot >= bufs_.size()) {
    bufs_.resize(slot + 1, nullptr);
    buf_bytes_.resize(slot + 1, 0);
  }
  if (buf_bytes_[slot] < bytes) {
    // a peer's copy out of the old buffer may still be queued on the peer's
    // stream (a send completes when the receiver ENQUEUED its copy): retire
    // it until this exchanger goes away instead of freeing it under the copy
    if (bufs_[slot]) retired_.push_back(bufs_[slot]);
    bufs_[slot] = nullptr;
    RMA_HIP_CHECK(hipMalloc(&bufs_[slot], bytes));
    buf_bytes_[slot] = bytes;
    cache_.clear();  // cached batches point at the old buffer
  }
  return bufs_[slot];
}

namespace {
bool same_fields(const std::vector<HaloField>& a, const std::vector<HaloField>& b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (a[i].ptr != b[i].ptr || a[i].size != b[i].size || a[i].elem_bytes != b[i].elem_bytes ||
        a[i].ol != b[i].ol || a[i].hw != b[i].hw)
      return false;
  return true;
}
}  // namespace

const HaloExchanger::Planned& HaloExchanger::planned(const std::vector<HaloField>& fields,
                                                     int dims_mask) {
  ++tick_;
  for (Planned& c : cache_)
    if (c.dims_mask == dims_mask && same_fields(c.fields, fields)) {
      c.used = tick_;
      ++hits_;
      return c;
    }
  ++misses_;
  Planned c;
  c.fields = fields;
  c.dims_mask = dims_mask;
  // the order of operations is the host-only plan (halo_plan.cpp), which the
  // sanitizer self test also executes on host memory
  c.plan = (dims_mask & kMerged)
               ? plan_exchange_merged(fields, nbr_, diag_, self_, self_via_comm_)
               : plan_exchange(fields, nbr_, self_, self_via_comm_, dims_mask);
  for (size_t s = 0; s < c.plan.slot_bytes.size(); ++s) buffer(s, c.plan.slot_bytes[s]);
  auto ptr = [&](const HaloMsg& m) -> void* {
    return m.slot >= 0 ? bufs_[m.slot]
                       : static_cast<char*>(fields[m.field].ptr) + m.view.offset * fields[m.field].elem_bytes;
  };
  for (const HaloDimPlan& dp : c.plan.dims) {
    c.batches.push_back({batch_copies(dim_copies(dp, fields, bufs_, 0)),
                         batch_copies(dim_copies(dp, fields, bufs_, 1))});
    c.send_ptr.emplace_back();
    c.recv_ptr.emplace_back();
    for (const HaloMsg& m : dp.sends) c.send_ptr.back().push_back(ptr(m));
    for (const HaloMsg& m : dp.recvs) c.recv_ptr.back().push_back(ptr(m));
  }
  c.used = tick_;
  if (cache_.size() >= kPlanCache) {
    size_t lru = 0;
    for (size_t i = 1; i < cache_.size(); ++i)
      if (cache_[i].used < cache_[lru].used) lru = i;
    cache_.erase(cache_.begin() + (std::ptrdiff_t)lru);
  }
  cache_.push_back(std::move(c));
  return cache_.back();
}

void HaloExchanger::prepare(const std::vector<HaloField>& fields, int dims_mask) {
  (void)planned(fields, dims_mask);
}

namespace {
// RMA_DIAG no_halo_batch: one launch per plane copy (A/B and diagnosis)
void launch_batches(const std::vector<CopyBatch>& bs, stream_t stream) {
  static const bool single = diag_flag("no_halo_batch");
  for (const CopyBatch& b : bs) {
    if (single) {
      for (const Copy2d& c : b.copies) copy2d_batch_gpu(&c, 1, b.elem_bytes, stream);
    } else {
      copy2d_batch_gpu(b.copies.data(), (int)b.copies.size(), b.elem_bytes, stream);
    }
  }
}

}  // namespace

void HaloExchanger::exchange(const std::vector<HaloField>& fields, stream_t stream,
                             int dims_mask) {
  const Planned& c = planned(fields, dims_mask);
  for (size_t d = 0; d < c.plan.dims.size(); ++d) {
    const HaloDimPlan& dp = c.plan.dims[d];
    // self copies + packs in one batched launch, the group, unpacks in one
    launch_batches(c.batches[d][0], stream);
    if (!dp.sends.empty() || !dp.recvs.empty()) {
      RMA_CHECK_ARG(comm_ != nullptr, "remote neighbour without communicator");
      comm_->group_start();
      for (size_t i = 0; i < dp.sends.size(); ++i)
        comm_->send(c.send_ptr[d][i], dp.sends[i].bytes, dp.sends[i].peer, stream);
      for (size_t i = 0; i < dp.recvs.size(); ++i)
        comm_->recv(c.recv_ptr[d][i], dp.recvs[i].bytes, dp.recvs[i].peer, stream);
      comm_->group_end();
    }
    launch_batches(c.batches[d][1], stream);
  }
  bytes_last_ = c.plan.bytes_sent;
}

void HaloExchanger::exchange_merged(const std::vector<HaloField>& fields, stream_t stream) {
  RMA_CHECK_ARG(has_diag_, "merged halo exchange needs the diagonal neighbours (set_diagonals)");
  exchange(fields, stream, kMerged | 3);
}

void HaloExchanger::exchange_cross(const std::vector<HaloField>& fields, stream_t stream,
                                   int dims_mask) {
  const Planned& c = planned(fields, dims_mask);
  // packs and self copies dimension by dimension (stream-ordered launches:
  // deterministic where two dimensions' self copies meet at a corner)
  for (size_t d = 0; d < c.plan.dims.size(); ++d) launch_batches(c.batches[d][0], stream);
  bool any = false;
  for (const HaloDimPlan& dp : c.plan.dims) any = any || !dp.sends.empty() || !dp.recvs.empty();
  if (any) {
    RMA_CHECK_ARG(comm_ != nullptr, "remote neighbour without communicator");
    comm_->group_start();
    for (size_t d = 0; d < c.plan.dims.size(); ++d) {
      const HaloDimPlan& dp = c.plan.dims[d];
      for (size_t i = 0; i < dp.sends.size(); ++i)
        comm_->send(c.send_ptr[d][i], dp.sends[i].bytes, dp.sends[i].peer, stream);
      for (size_t i = 0; i < dp.recvs.size(); ++i)
        comm_->recv(c.recv_ptr[d][i], dp.recvs[i].bytes, dp.recvs[i].peer, stream);
    }
    comm_->group_end();
  }
  for (size_t d = 0; d < c.plan.dims.size(); ++d) launch_batches(c.batches[d][1], stream);
  bytes_last_ = c.plan.bytes_sent;
}

}  // namespace rma
