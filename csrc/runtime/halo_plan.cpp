#include "rma/halo_plan.h"

#include <algorithm>

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

bool has_halo(const HaloField& f, int d) {
  return f.size[d] > 1 && f.ol[d] >= 2 * f.hw[d] && f.size[d] >= f.ol[d] + f.hw[d];
}

void validate_field(const HaloField& f) {
  RMA_CHECK_ARG(f.ptr != nullptr, "null field");
  RMA_CHECK_ARG(f.elem_bytes == 2 || f.elem_bytes == 4 || f.elem_bytes == 8 || f.elem_bytes == 16,
                "elem_bytes=" << f.elem_bytes);
  for (int d = 0; d < 3; ++d) RMA_CHECK_ARG(f.hw[d] >= 1 && f.size[d] >= 1, "bad field dims");
}

HaloPlan plan_exchange(const std::vector<HaloField>& fields,
                       const std::array<std::array<int, 2>, 3>& nbr, int self,
                       bool self_via_comm, int dims_mask) {
  HaloPlan plan;
  for (const auto& f : fields) validate_field(f);
  for (int d = 0; d < 3; ++d) {
    if (!(dims_mask >> d & 1) || (nbr[d][0] < 0 && nbr[d][1] < 0)) continue;
    HaloDimPlan dp;
    dp.dim = d;
    for (int fi = 0; fi < (int)fields.size(); ++fi) {
      const HaloField& f = fields[fi];
      if (!has_halo(f, d)) continue;
      const int64_t n = f.size[d], ol = f.ol[d], hw = f.hw[d];
      // send planes: lo [ol-hw, ol), hi [n-ol, n-ol+hw); recv planes: lo [0,hw), hi [n-hw, n)
      const PlaneView send_v[2] = {plane_view(f, d, ol - hw), plane_view(f, d, n - ol)};
      const PlaneView recv_v[2] = {plane_view(f, d, 0), plane_view(f, d, n - hw)};
      const size_t bytes = (size_t)send_v[0].elems() * f.elem_bytes;
      HaloMsg s_ops[2], r_ops[2];
      bool on[2] = {false, false};
      for (int s = 0; s < 2; ++s) {
        const int p = nbr[d][s];
        if (p < 0) continue;
        if (p == self && !self_via_comm) {
          // periodic, single process along d: my side-s halo <- my opposite send plane
          dp.copies.push_back({fi, recv_v[s], send_v[1 - s]});
          continue;
        }
        on[s] = true;
        if (send_v[s].contiguous()) {  // zero-copy: straight from / into the field
          s_ops[s] = {p, fi, send_v[s], -1, bytes};
          r_ops[s] = {p, fi, recv_v[s], -1, bytes};
        } else {
          const int sb = (int)plan.slot_bytes.size();
          plan.slot_bytes.push_back(bytes);
          plan.slot_bytes.push_back(bytes);
          dp.packs.push_back({fi, send_v[s], sb});
          s_ops[s] = {p, fi, send_v[s], sb, bytes};
          r_ops[s] = {p, fi, recv_v[s], sb + 1, bytes};
          dp.unpacks.push_back({fi, recv_v[s], sb + 1});
        }
        plan.bytes_sent += (int64_t)bytes;
      }
      for (int s = 0; s < 2; ++s)
        if (on[s]) dp.sends.push_back(s_ops[s]);
      for (int s = 1; s >= 0; --s)
        if (on[s]) dp.recvs.push_back(r_ops[s]);
    }
    plan.dims.push_back(std::move(dp));
  }
  return plan;
}

HaloPlan plan_exchange_merged(const std::vector<HaloField>& fields,
                              const std::array<std::array<int, 2>, 3>& nbr,
                              const std::array<int, 4>& diag, int self, bool self_via_comm) {
  HaloPlan plan;
  HaloDimPlan dp;
  dp.dim = -1;
  for (const auto& f : fields) {
    validate_field(f);
    RMA_CHECK_ARG(f.size[2] == 1, "merged x+y halo exchange: 2D fields only (nz = " << f.size[2]
                                                                               << ")");
  }
  // direction k = (sy+1)*3 + (sx+1), k != 4; the message received from the
  // neighbour at k was sent by it in direction 8 - k
  auto peer_of = [&](int sx, int sy) {
    if (sy == 0) return nbr[0][sx > 0];
    if (sx == 0) return nbr[1][sy > 0];
    return diag[(sy > 0 ? 2 : 0) + (sx > 0 ? 1 : 0)];
  };
  struct Msg {
    int key;
    HaloMsg m;
  };
  std::vector<Msg> sends, recvs;
  for (int fi = 0; fi < (int)fields.size(); ++fi) {
    const HaloField& f = fields[fi];
    const int64_t nx = f.size[0], ny = f.size[1];
    const int64_t olx = f.ol[0], oly = f.ol[1], hwx = f.hw[0], hwy = f.hw[1];
    // sides with a halo exchange: a neighbour there and room for the planes
    const bool hx = has_halo(f, 0), hy = has_halo(f, 1);
    const bool on_x[2] = {hx && nbr[0][0] >= 0, hx && nbr[0][1] >= 0};
    const bool on_y[2] = {hy && nbr[1][0] >= 0, hy && nbr[1][1] >= 0};
    // the other dimension's extent of an edge plane: outside its halo
    const int64_t x0 = on_x[0] ? hwx : 0, x1 = on_x[1] ? nx - hwx : nx;
    const int64_t y0 = on_y[0] ? hwy : 0, y1 = on_y[1] ? ny - hwy : ny;
    auto block = [&](int64_t c0, int64_t c1, int64_t r0, int64_t r1) {
      return PlaneView{r0 * nx + c0, r1 - r0, c1 - c0, nx};
    };
    // the block sent toward direction (sx, sy) / received from it
    auto send_block = [&](int sx, int sy) {
      const int64_t c0 = sx == 0 ? x0 : sx < 0 ? olx - hwx : nx - olx;
      const int64_t c1 = sx == 0 ? x1 : c0 + hwx;
      const int64_t r0 = sy == 0 ? y0 : sy < 0 ? oly - hwy : ny - oly;
      const int64_t r1 = sy == 0 ? y1 : r0 + hwy;
      return block(c0, c1, r0, r1);
    };
    auto recv_block = [&](int sx, int sy) {
      const int64_t c0 = sx == 0 ? x0 : sx < 0 ? 0 : nx - hwx;
      const int64_t c1 = sx == 0 ? x1 : c0 + hwx;
      const int64_t r0 = sy == 0 ? y0 : sy < 0 ? 0 : ny - hwy;
      const int64_t r1 = sy == 0 ? y1 : r0 + hwy;
      return block(c0, c1, r0, r1);
    };
    for (int k = 0; k < 9; ++k) {
      if (k == 4) continue;
      const int sx = k % 3 - 1, sy = k / 3 - 1;
      if ((sx != 0 && !on_x[sx > 0]) || (sy != 0 && !on_y[sy > 0])) continue;
      const int p = peer_of(sx, sy);
      RMA_CHECK_ARG(p >= 0, "merged halo exchange: no rank at diagonal (" << sx << "," << sy
                                                                         << ")");
      PlaneView sv = send_block(sx, sy), rv = recv_block(sx, sy);
      if (sv.elems() == 0) continue;
      if (p == self && !self_via_comm) {
        // periodic self neighbour: my halo toward k <- my own block toward 8 - k
        // (disjoint blocks: the batched copies may run concurrently)
        dp.copies.push_back({fi, rv, send_block(-sx, -sy)});
        continue;
      }
      // a y message (sx = 0) through the transport takes the full rows: one
      // contiguous zero-copy plane; the x-halo cells it carries (the sender's
      // stale ones) are corners, rewritten by the corner unpacks after the group
      const bool corner = sx != 0 && sy != 0;
      if (sx == 0 && (on_x[0] || on_x[1])) {
        sv = block(0, nx, sv.offset / nx, sv.offset / nx + sv.n_o);
        rv = block(0, nx, rv.offset / nx, rv.offset / nx + rv.n_o);
      }
      const size_t bytes = (size_t)sv.elems() * f.elem_bytes;
      RMA_CHECK_ARG(rv.elems() == sv.elems(), "merged halo blocks differ in size");
      HaloMsg sm{p, fi, sv, -1, bytes}, rm{p, fi, rv, -1, bytes};
      if (!sv.contiguous()) {
        sm.slot = (int)plan.slot_bytes.size();
        plan.slot_bytes.push_back(bytes);
        dp.packs.push_back({fi, sv, sm.slot});
      }
      // corners and x planes always land after the group (never during it:
      // a sender's full y rows include those cells)
      if (corner || sx != 0 || !rv.contiguous()) {
        rm.slot = (int)plan.slot_bytes.size();
        plan.slot_bytes.push_back(bytes);
        dp.unpacks.push_back({fi, rv, rm.slot});
      }
      sends.push_back({fi * 9 + k, sm});
      recvs.push_back({fi * 9 + (8 - k), rm});
      plan.bytes_sent += (int64_t)bytes;
    }
  }
  auto by_key = [](const Msg& a, const Msg& b) { return a.key < b.key; };
  std::stable_sort(sends.begin(), sends.end(), by_key);
  std::stable_sort(recvs.begin(), recvs.end(), by_key);
  for (const Msg& m : sends) dp.sends.push_back(m.m);
  for (const Msg& m : recvs) dp.recvs.push_back(m.m);
  if (!dp.copies.empty() || !dp.sends.empty() || !dp.recvs.empty())
    plan.dims.push_back(std::move(dp));
  return plan;
}

namespace {
char* plane_ptr(const HaloField& f, const PlaneView& v) {
  return static_cast<char*>(f.ptr) + v.offset * f.elem_bytes;
}
}  // namespace

std::vector<std::pair<int, Copy2d>> dim_copies(const HaloDimPlan& dp,
                                               const std::vector<HaloField>& fields,
                                               const std::vector<void*>& slots, int phase) {
  std::vector<std::pair<int, Copy2d>> q;
  auto slot = [&](int i) {
    RMA_CHECK_ARG(i >= 0 && i < (int)slots.size() && slots[i], "halo buffer slot " << i);
    return slots[i];
  };
  if (phase == 0) {
    for (const HaloCopy& c : dp.copies) {
      const HaloField& f = fields.at(c.field);
      q.push_back({f.elem_bytes, {plane_ptr(f, c.dst), c.dst.ld, plane_ptr(f, c.src), c.src.ld,
                                  c.src.n_o, c.src.n_k}});
    }
    for (const HaloPack& p : dp.packs) {
      const HaloField& f = fields.at(p.field);
      q.push_back({f.elem_bytes, {slot(p.slot), p.view.n_k, plane_ptr(f, p.view), p.view.ld,
                                  p.view.n_o, p.view.n_k}});
    }
  } else {
    for (const HaloPack& u : dp.unpacks) {
      const HaloField& f = fields.at(u.field);
      q.push_back({f.elem_bytes, {plane_ptr(f, u.view), u.view.ld, slot(u.slot), u.view.n_k,
                                  u.view.n_o, u.view.n_k}});
    }
  }
  return q;
}

std::vector<CopyBatch> batch_copies(const std::vector<std::pair<int, Copy2d>>& q) {
  std::vector<CopyBatch> out;
  std::vector<bool> done(q.size(), false);
  for (size_t i = 0; i < q.size(); ++i) {
    if (done[i]) continue;
    const int eb = q[i].first;
    CopyBatch b{eb, {}};
    for (size_t j = i; j < q.size(); ++j) {
      if (done[j] || q[j].first != eb) continue;
      done[j] = true;
      b.copies.push_back(q[j].second);
      if ((int)b.copies.size() == kCopy2dBatch) {
        out.push_back(std::move(b));
        b = CopyBatch{eb, {}};
      }
    }
    if (!b.copies.empty()) out.push_back(std::move(b));
  }
  return out;
}

}  // namespace rma
