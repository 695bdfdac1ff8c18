// Host-only plan of one halo exchange (no HIP): which planes of which fields
// are copied locally, packed, sent, received and unpacked, per dimension and
// in which order. HaloExchanger (halo.cpp) executes a plan on the GPU; the
// sanitizer self test (tests/native/host_selftest.cpp) executes the same plan
// on host memory for several fake ranks in one process under ASan/UBSan.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

#include "rma/common.h"
#include "rma/kernels.h"  // Copy2d (HIP-free)

namespace rma {

struct HaloField {
  void* ptr = nullptr;
  std::array<int64_t, 3> size{1, 1, 1};  // extent along x, y, z (x fastest)
  int elem_bytes = 8;
  std::array<int64_t, 3> ol{2, 2, 2};    // overlap of this array per dim
  std::array<int64_t, 3> hw{1, 1, 1};    // halo width per dim
};

// A strided view of one plane block of a field: n_o rows of n_k contiguous
// elements, rows `ld` elements apart, starting at element `offset`.
struct PlaneView {
  int64_t offset, n_o, n_k, ld;
  bool contiguous() const { return n_o == 1 || ld == n_k; }
  int64_t elems() const { return n_o * n_k; }
};
PlaneView plane_view(const HaloField& f, int dim, int64_t index0);
// A field has a halo along d when it is not flat there and its overlap holds
// two halo planes (ImplicitGlobalGrid skips such dimensions for that field,
// e.g. an array of size n-1 with overlap 2).
bool has_halo(const HaloField& f, int dim);
void validate_field(const HaloField& f);

// One exchange, dimension by dimension (x, then y, then z: the later planes
// carry the corner values received earlier). Within a dimension the executor
// runs: self copies and packs, ONE group of sends + receives, unpacks.
struct HaloCopy {          // local periodic copy (self neighbour)
  int field;
  PlaneView dst, src;
};
struct HaloPack {          // strided plane <-> contiguous buffer slot
  int field;
  PlaneView view;
  int slot;
};
struct HaloMsg {           // one send or receive of the group
  int peer;
  int field;               // in-place plane of this field (slot < 0) ...
  PlaneView view;
  int slot;                // ... or buffer slot (>= 0)
  size_t bytes;
};
struct HaloDimPlan {
  int dim = 0;
  std::vector<HaloCopy> copies;
  std::vector<HaloPack> packs;     // before the group
  std::vector<HaloMsg> sends;      // (lo, hi) order per field
  std::vector<HaloMsg> recvs;      // (hi, lo) order per field
  std::vector<HaloPack> unpacks;   // after the group
};
struct HaloPlan {
  std::vector<HaloDimPlan> dims;
  std::vector<size_t> slot_bytes;  // size of every buffer slot
  int64_t bytes_sent = 0;
};

// nbr[d] = {low, high} rank (-1: none). self_via_comm routes self neighbours
// through the transport (one send + one receive to oneself) instead of a copy.
HaloPlan plan_exchange(const std::vector<HaloField>& fields,
                       const std::array<std::array<int, 2>, 3>& nbr, int self,
                       bool self_via_comm, int dims_mask);

// x and y in ONE group (2D fields, z flat): x planes restricted to the rows
// outside the y halo, y planes as full contiguous rows (zero-copy; their
// corner cells are rewritten after the group), plus the hw_x x hw_y corner
// blocks sent straight to the diagonal neighbours and unpacked after the
// group, so the corners need no second, dimension-ordered group (local
// periodic copies: disjoint blocks, y planes restricted too). Every halo cell receives the value the
// dimension-ordered exchange gives it (host self test: bitwise equal). diag:
// the ranks at (x-1,y-1), (x+1,y-1), (x-1,y+1), (x+1,y+1) (-1: none). One
// HaloDimPlan (dim = -1) whose sends are ordered by (field, direction) and
// receives by (field, the sender's direction), so every pair of ranks matches
// its messages in issue order.
HaloPlan plan_exchange_merged(const std::vector<HaloField>& fields,
                              const std::array<std::array<int, 2>, 3>& nbr,
                              const std::array<int, 4>& diag, int self, bool self_via_comm);

// The plane copies of one phase of a dimension, as (element bytes, copy) in
// plan order: phase 0 = self copies + packs (before the group; independent:
// halo planes [0,hw), [n-hw,n) vs send planes [ol-hw,ol), [n-ol,n-ol+hw) with
// ol >= 2hw), phase 1 = unpacks (after it). slots[i] is buffer slot i.
std::vector<std::pair<int, Copy2d>> dim_copies(const HaloDimPlan& dp,
                                               const std::vector<HaloField>& fields,
                                               const std::vector<void*>& slots, int phase);
// Batches of <= kCopy2dBatch copies of one element size (one launch each):
// a single batch for the usual all-fp64 phase.
struct CopyBatch {
  int elem_bytes;
  std::vector<Copy2d> copies;
};
std::vector<CopyBatch> batch_copies(const std::vector<std::pair<int, Copy2d>>& q);

}  // namespace rma
