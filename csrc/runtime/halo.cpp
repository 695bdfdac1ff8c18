#include "rma/halo.h"

#include <hip/hip_runtime.h>

#include "rma/hip_check.h"
#include "rma/topology.h"

namespace rma {

PlaneView plane_view(const HaloField& f, int dim, int64_t i0) {
  const int64_t nx = f.size[0], ny = f.size[1], nz = f.size[2];
  const int64_t hw = f.hw[dim];
  switch (dim) {
    case 0: return {i0, nz * ny, hw, nx};
    case 1: return {i0 * nx, nz, hw * nx, ny * nx};
    default: return {i0 * nx * ny, 1, hw * nx * ny, nx * ny * nz};
  }
}

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

namespace {
void validate(const HaloField& f) {
  RMA_CHECK_ARG(f.ptr != nullptr, "null field");
  RMA_CHECK_ARG(f.elem_bytes == 2 || f.elem_bytes == 4 || f.elem_bytes == 8 || f.elem_bytes == 16,
                "elem_bytes=" << f.elem_bytes);
  for (int d = 0; d < 3; ++d) RMA_CHECK_ARG(f.hw[d] >= 1 && f.size[d] >= 1, "bad field dims");
}
}  // namespace

// A field has a halo along d when it is not flat there and its overlap holds
// two halo planes (ImplicitGlobalGrid skips such dimensions for that field,
// e.g. an array of size n-1 with overlap 2).
bool has_halo(const HaloField& f, int d) {
  return f.size[d] > 1 && f.ol[d] >= 2 * f.hw[d] && f.size[d] >= f.ol[d] + f.hw[d];
}

namespace {

char* at(const HaloField& f, const PlaneView& v) {
  return static_cast<char*>(f.ptr) + v.offset * f.elem_bytes;
}
}  // namespace

void HaloExchanger::prepare(const std::vector<HaloField>& fields, int dims_mask) {
  size_t slot = 0;
  for (int d = 0; d < 3; ++d) {
    if (!(dims_mask >> d & 1) || !active(d)) continue;
    for (const auto& f : fields) {
      if (!has_halo(f, d)) continue;
      const PlaneView v = plane_view(f, d, 0);
      const size_t bytes = (size_t)v.elems() * f.elem_bytes;
      for (int s = 0; s < 2; ++s) {
        const int p = nbr_[d][s];
        if (p < 0 || (p == self_ && !self_via_comm_) || v.contiguous()) continue;
        buffer(slot++, bytes);  // send
        buffer(slot++, bytes);  // recv
      }
    }
  }
}

void HaloExchanger::exchange(const std::vector<HaloField>& fields, stream_t stream,
                             int dims_mask) {
  bytes_last_ = 0;
  size_t slot = 0;
  struct Pending {
    const HaloField* f;
    PlaneView dst;
    void* buf;
  };
  for (int d = 0; d < 3; ++d) {
    if (!(dims_mask >> d & 1) || !active(d)) continue;
    struct Op {
      int peer;
      void* ptr;
      size_t bytes;
    };
    std::vector<Op> sends, recvs;  // sends in (lo, hi) order, recvs in (hi, lo) order per field
    std::vector<Pending> unpack;
    for (const auto& f : fields) {
      validate(f);
      if (!has_halo(f, d)) continue;
      const int64_t n = f.size[d], ol = f.ol[d], hw = f.hw[d];
      // send planes: lo [ol-hw, ol), hi [n-ol, n-ol+hw); recv planes: lo [0,hw), hi [n-hw, n)
      const PlaneView send_v[2] = {plane_view(f, d, ol - hw), plane_view(f, d, n - ol)};
      const PlaneView recv_v[2] = {plane_view(f, d, 0), plane_view(f, d, n - hw)};
      const size_t bytes = (size_t)send_v[0].elems() * f.elem_bytes;
      Op s_ops[2] = {{-1, nullptr, 0}, {-1, nullptr, 0}};
      Op r_ops[2] = {{-1, nullptr, 0}, {-1, nullptr, 0}};
      for (int s = 0; s < 2; ++s) {
        const int p = nbr_[d][s];
        if (p < 0) continue;
        if (p == self_ && !self_via_comm_) {
          // periodic, single process along d: my side-s halo <- my opposite send plane
          const PlaneView& src = send_v[1 - s];
          const PlaneView& dst = recv_v[s];
          copy2d_gpu(at(f, dst), dst.ld, at(f, src), src.ld, src.n_o, src.n_k, f.elem_bytes,
                     stream);
          continue;
        }
        RMA_CHECK_ARG(comm_ != nullptr, "remote neighbour without communicator");
        if (send_v[s].contiguous()) {
          s_ops[s] = {p, at(f, send_v[s]), bytes};
          r_ops[s] = {p, at(f, recv_v[s]), bytes};
        } else {
          void* sb = buffer(slot++, bytes);
          void* rb = buffer(slot++, bytes);
          copy2d_gpu(sb, send_v[s].n_k, at(f, send_v[s]), send_v[s].ld, send_v[s].n_o,
                     send_v[s].n_k, f.elem_bytes, stream);
          s_ops[s] = {p, sb, bytes};
          r_ops[s] = {p, rb, bytes};
          unpack.push_back({&f, recv_v[s], rb});
        }
        bytes_last_ += (int64_t)bytes;
      }
      for (int s = 0; s < 2; ++s)
        if (s_ops[s].peer >= 0) sends.push_back(s_ops[s]);
      for (int s = 1; s >= 0; --s)
        if (r_ops[s].peer >= 0) recvs.push_back(r_ops[s]);
    }
    if (!sends.empty() || !recvs.empty()) {
      comm_->group_start();
      for (const auto& o : sends) comm_->send(o.ptr, o.bytes, o.peer, stream);
      for (const auto& o : recvs) comm_->recv(o.ptr, o.bytes, o.peer, stream);
      comm_->group_end();
    }
    for (const auto& u : unpack)
      copy2d_gpu(at(*u.f, u.dst), u.dst.ld, u.buf, u.dst.n_k, u.dst.n_o, u.dst.n_k,
                 u.f->elem_bytes, stream);
  }
}

}  // namespace rma
