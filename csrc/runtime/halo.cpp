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
}

bool HaloExchanger::active(int dim) const { return nbr_[dim][0] >= 0 || nbr_[dim][1] >= 0; }

void* HaloExchanger::buffer(size_t slot, size_t bytes) {
  if (slot >= bufs_.size()) {
    bufs_.resize(slot + 1, nullptr);
    buf_bytes_.resize(slot + 1, 0);
  }
  if (buf_bytes_[slot] < bytes) {
    if (bufs_[slot]) RMA_HIP_CHECK(hipFree(bufs_[slot]));
    bufs_[slot] = nullptr;
    RMA_HIP_CHECK(hipMalloc(&bufs_[slot], bytes));
    buf_bytes_[slot] = bytes;
  }
  return bufs_[slot];
}

void HaloExchanger::prepare(const std::vector<HaloField>& fields, int dims_mask) {
  const HaloPlan plan = plan_exchange(fields, nbr_, self_, self_via_comm_, dims_mask);
  for (size_t s = 0; s < plan.slot_bytes.size(); ++s) buffer(s, plan.slot_bytes[s]);
}

namespace {
char* at(const HaloField& f, const PlaneView& v) {
  return static_cast<char*>(f.ptr) + v.offset * f.elem_bytes;
}

// RMA_HALO_BATCH=0: one launch per plane copy (A/B and diagnosis)
void launch_batches(const std::vector<CopyBatch>& bs, stream_t stream) {
  static const char* e = std::getenv("RMA_HALO_BATCH");
  const bool single = e && e[0] == '0';
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
  // the order of operations is the host-only plan (halo_plan.cpp), which the
  // sanitizer self test also executes on host memory
  const HaloPlan plan = plan_exchange(fields, nbr_, self_, self_via_comm_, dims_mask);
  for (size_t s = 0; s < plan.slot_bytes.size(); ++s) buffer(s, plan.slot_bytes[s]);
  for (const HaloDimPlan& dp : plan.dims) {
    // self copies + packs in one batched launch, the group, unpacks in one
    launch_batches(batch_copies(dim_copies(dp, fields, bufs_, 0)), stream);
    if (!dp.sends.empty() || !dp.recvs.empty()) {
      RMA_CHECK_ARG(comm_ != nullptr, "remote neighbour without communicator");
      comm_->group_start();
      for (const HaloMsg& m : dp.sends)
        comm_->send(m.slot >= 0 ? bufs_[m.slot] : at(fields[m.field], m.view), m.bytes, m.peer,
                    stream);
      for (const HaloMsg& m : dp.recvs)
        comm_->recv(m.slot >= 0 ? bufs_[m.slot] : at(fields[m.field], m.view), m.bytes, m.peer,
                    stream);
      comm_->group_end();
    }
    launch_batches(batch_copies(dim_copies(dp, fields, bufs_, 1)), stream);
  }
  bytes_last_ = plan.bytes_sent;
}

}  // namespace rma
