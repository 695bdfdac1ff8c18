// Halo exchange engine: ImplicitGlobalGrid's update_halo! for
// device arrays, GPU-direct over RCCL.
//
// Semantics kept from IGG (call sites scripts/diffusion_2D_ap.jl:42,
// diffusion_2D_kp.jl:91, diffusion_2D_perf.jl:51):
//   * dimensions are exchanged one after the other (x, then y, then z), so the
//     later planes carry the corner values received earlier;
//   * per side with a real neighbour: the send plane(s) [ol-hw, ol) (low side)
//     and [n-ol, n-ol+hw) (high side) go to the neighbour, whose halo planes
//     [0,hw) / [n-hw,n) receive them (0-based; ol = overlap of THIS array, which
//     differs from the grid overlap by size(A)-n for staggered arrays);
//   * periodic dimensions with a single process copy locally.
// MI355X-first changes: contiguous planes (y-planes of 2D fields, z-planes)
// are sent/received in place (zero-copy); only strided planes go through
// persistent pack/unpack buffers (allocated once, reused — no allocation in
// the steady state, so a step can be captured in a hipGraph); all sends and
// receives of one dimension form ONE RCCL group on the caller's stream.
#pragma once

#include <array>
#include <cstdint>
#include <vector>

#include "rma/comm.h"
#include "rma/halo_plan.h"
#include "rma/kernels.h"

namespace rma {

class HaloExchanger {
 public:
  // neighbors[d] = {low, high} ranks (kProcNull = -1 at open edges);
  // comm may be null when every neighbour is either absent or this rank.
  HaloExchanger(P2PTransport* comm, int self_rank, std::array<std::array<int, 2>, 3> neighbors);
  ~HaloExchanger();
  HaloExchanger(const HaloExchanger&) = delete;
  HaloExchanger& operator=(const HaloExchanger&) = delete;

  // Enqueue the full exchange of all fields on `stream` (asynchronous).
  // dims_mask bit d enables dimension d.
  void exchange(const std::vector<HaloField>& fields, stream_t stream, int dims_mask = 7);
  // The same messages with ONE RCCL group for all dimensions (packs of every
  // dimension first, unpacks after the group). Only the halo cells that lie in
  // one dimension's halo are exact; corner cells (in two dimensions' halos)
  // may hold a stale value. For cross-shaped (5-point) stencils whose next
  // update reads no corner halo cell (one-step passes): one group instead of
  // one per dimension, i.e. one RCCL enqueue and one RCCL kernel per exchange.
  void exchange_cross(const std::vector<HaloField>& fields, stream_t stream, int dims_mask = 7);
  // x and y in ONE group with the corner blocks sent straight to the diagonal
  // neighbours (halo_plan.h plan_exchange_merged): exact corners like
  // exchange(), half the groups. Needs set_diagonals(); 2D fields.
  void exchange_merged(const std::vector<HaloField>& fields, stream_t stream);
  // Pre-allocate the pack buffers for this field set (call before capture).
  void prepare(const std::vector<HaloField>& fields, int dims_mask = 7);
  // ranks at (x-1,y-1), (x+1,y-1), (x-1,y+1), (x+1,y+1) (CartTopology::diagonals)
  void set_diagonals(const std::array<int, 4>& d) {
    diag_ = d;
    has_diag_ = true;
    cache_.clear();
  }
  bool has_diagonals() const { return has_diag_; }
  // bit of dims_mask that selects the merged plan (planned() cache key)
  static constexpr int kMerged = 8;

  bool active(int dim) const;  // any neighbour in this dim?
  // Graph capture is possible when no message goes through a non-capturable
  // transport (local self copies and the pack kernels always capture).
  bool capturable() const {
    if (comm_ == nullptr || comm_->capturable()) return true;
    for (int d = 0; d < 3; ++d)
      for (int s = 0; s < 2; ++s)
        if (nbr_[d][s] >= 0 && (nbr_[d][s] != self_ || self_via_comm_)) return false;
    return true;
  }
  // Route self-neighbours (periodic, one process along a dim) through the
  // transport instead of a local copy (tests the P2P path on one GPU).
  void set_self_via_transport(bool on) {
    self_via_comm_ = on && comm_ != nullptr;
    cache_.clear();
  }
  const std::array<std::array<int, 2>, 3>& neighbors() const { return nbr_; }
  int64_t bytes_sent_last() const { return bytes_last_; }
  // exchanges served from the plan cache / planned afresh (tests, diagnosis)
  int64_t plan_hits() const { return hits_; }
  int64_t plan_misses() const { return misses_; }
  const std::array<int, 4>& diagonals() const { return diag_; }

 private:
  // One planned exchange: the host plan plus its copy batches with every
  // pointer resolved (fields and pack buffers). The executor alternates
  // between two fields (T, T2), so a few entries serve the steady state and
  // an exchange costs only its launches and the RCCL group.
  struct Planned {
    std::vector<HaloField> fields;
    int dims_mask = 0;
    HaloPlan plan;
    std::vector<std::array<std::vector<CopyBatch>, 2>> batches;  // per plan dim, phase 0 / 1
    std::vector<std::vector<void*>> send_ptr, recv_ptr;          // per plan dim, message order
    uint64_t used = 0;
  };
  static constexpr size_t kPlanCache = 4;
  const Planned& planned(const std::vector<HaloField>& fields, int dims_mask);
  void* buffer(size_t slot, size_t bytes);
  P2PTransport* comm_;
  int self_;
  bool self_via_comm_ = false;
  std::array<int, 4> diag_{-1, -1, -1, -1};
  bool has_diag_ = false;
  std::array<std::array<int, 2>, 3> nbr_;
  std::vector<void*> bufs_;
  std::vector<size_t> buf_bytes_;
  std::vector<void*> retired_;  // outgrown pack buffers, freed in the destructor
  int64_t bytes_last_ = 0;
  std::vector<Planned> cache_;
  uint64_t tick_ = 0;
  int64_t hits_ = 0, misses_ = 0;
};

}  // namespace rma
