// pybind11 bindings of the native core: rocm_mpi_amd._C
//
// Pure C++ (no HIP headers): pointers travel as integers (torch
// Tensor.data_ptr()), streams as integers (torch.cuda.Stream.cuda_stream).
// Shape/dtype/device validation happens in rocm_mpi_amd/ops before any call.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <string>
#include <tuple>
#include <vector>

#include "rma/config.h"
#include "rma/comm.h"
#include "rma/common.h"
#include "rma/executor.h"
#include "rma/halo.h"
#include "rma/ipc.h"
#include "rma/kernels.h"
#include "rma/loopback.h"
#include "rma/p2p.h"
#include "rma/plan.h"
#include "rma/topology.h"
#include "rma/trace.h"

namespace py = pybind11;
using namespace rma;

namespace {

template <typename T>
T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
stream_t S(uintptr_t s) { return reinterpret_cast<stream_t>(s); }

using Rect4 = std::tuple<int64_t, int64_t, int64_t, int64_t>;
using Coef4 = std::tuple<double, double, double, double>;  // mlam, rdx, rdy, dt
using Geom = std::tuple<int64_t, int64_t, int64_t, int64_t, double, double, double, double, int,
                        int>;  // gx0 gy0 nxg nyg dx dy xoff yoff periodx periody

std::vector<Rect> to_rects(const std::vector<Rect4>& v) {
  std::vector<Rect> r;
  for (auto& t : v) r.push_back({std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t)});
  return r;
}
StencilCoef to_coef(const Coef4& c) {
  return {std::get<0>(c), std::get<1>(c), std::get<2>(c), std::get<3>(c)};
}
TileGeom to_geom(const Geom& g) {
  TileGeom t;
  std::tie(t.gx0, t.gy0, t.nxg, t.nyg, t.dx, t.dy, t.xoff, t.yoff, t.periodx, t.periody) = g;
  return t;
}
Rect4 from_rect(const Rect& r) { return {r.x0, r.x1, r.y0, r.y1}; }

using FieldT = std::tuple<uintptr_t, std::array<int64_t, 3>, int, std::array<int64_t, 3>,
                          std::array<int64_t, 3>>;
std::vector<HaloField> to_fields(const std::vector<FieldT>& v) {
  std::vector<HaloField> out;
  for (auto& t : v) {
    HaloField f;
    f.ptr = reinterpret_cast<void*>(std::get<0>(t));
    f.size = std::get<1>(t);
    f.elem_bytes = std::get<2>(t);
    f.ol = std::get<3>(t);
    f.hw = std::get<4>(t);
    out.push_back(f);
  }
  return out;
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "rocm_mpi_amd native core (HIP kernels for gfx950, RCCL halo exchange, executor)";
  static py::exception<Error> exc(m, "NativeError", PyExc_RuntimeError);
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const Error& e) {
      exc(e.what());
    }
  });

  m.def("set_rank_for_errors", &set_rank_for_errors);
  m.def("rccl_version", &rccl_version);
  m.def("rccl_library", &rccl_library);
  m.def("device_pci_bus_id", &device_pci_bus_id, py::arg("device"));
  m.def(
      "stencil_strip_cells",
      [](int64_t nx, int vec) {
        StencilTuning t;
        t.vec = vec;
        return stencil_strip_cells(nx, t);
      },
      py::arg("nx"), py::arg("vec") = 2);

  // ---------------- kernels ----------------
  m.def(
      "stencil_rects",
      [](uintptr_t T2, uintptr_t T, uintptr_t iCp, int64_t nx, int64_t ny,
         const std::vector<Rect4>& rects, const Coef4& coef, int chunk_rows, int nontemporal,
         int kernel, uintptr_t stream, bool gpu, int unroll, int vec, int xcd_remap) {
        auto r = to_rects(rects);
        StencilTuning tn;
        tn.chunk_rows = chunk_rows;
        tn.nontemporal = nontemporal;
        tn.kernel = kernel;
        tn.unroll = unroll;
        tn.vec = vec;
        tn.xcd_remap = xcd_remap;
        if (gpu)
          stencil_rects_gpu(P<double>(T2), P<const double>(T), P<const double>(iCp), nx, ny,
                            r.data(), (int)r.size(), to_coef(coef), tn, S(stream));
        else {
          py::gil_scoped_release nogil;
          stencil_rects_cpu(P<double>(T2), P<const double>(T), P<const double>(iCp), nx, ny,
                            r.data(), (int)r.size(), to_coef(coef));
        }
      },
      py::arg("T2"), py::arg("T"), py::arg("iCp"), py::arg("nx"), py::arg("ny"), py::arg("rects"),
      py::arg("coef"), py::arg("chunk_rows") = 4, py::arg("nontemporal") = 3,
      py::arg("kernel") = 0, py::arg("stream") = 0, py::arg("gpu") = true,
      py::arg("unroll") = 4, py::arg("vec") = 2, py::arg("xcd_remap") = -1);
  m.def(
      "stencil2_rects",
      [](uintptr_t T2, uintptr_t T, uintptr_t iCp, int64_t nx, int64_t ny,
         const std::vector<Rect4>& rects, const Coef4& coef, int chunk_rows, int nontemporal,
         uintptr_t stream, bool gpu, int unroll, int xcd_remap) {
        auto r = to_rects(rects);
        StencilTuning tn;
        tn.chunk_rows = chunk_rows;
        tn.nontemporal = nontemporal;
        tn.unroll = unroll;
        tn.xcd_remap = xcd_remap;
        if (gpu)
          stencil2_rects_gpu(P<double>(T2), P<const double>(T), P<const double>(iCp), nx, ny,
                             r.data(), (int)r.size(), to_coef(coef), tn, S(stream));
        else {
          py::gil_scoped_release nogil;
          stencil2_rects_cpu(P<double>(T2), P<const double>(T), P<const double>(iCp), nx, ny,
                             r.data(), (int)r.size(), to_coef(coef));
        }
      },
      py::arg("T2"), py::arg("T"), py::arg("iCp"), py::arg("nx"), py::arg("ny"), py::arg("rects"),
      py::arg("coef"), py::arg("chunk_rows") = 8, py::arg("nontemporal") = 3,
      py::arg("stream") = 0, py::arg("gpu") = true, py::arg("unroll") = 2,
      py::arg("xcd_remap") = -1);
  m.def(
      "stencilk_rects",
      [](int K, uintptr_t T2, uintptr_t T, uintptr_t iCp, int64_t nx, int64_t ny,
         const std::vector<Rect4>& rects, const Coef4& coef, int chunk_rows, int nontemporal,
         uintptr_t stream, bool gpu, int xcd_remap, int vec, int kernel, int stages, int cols) {
        auto r = to_rects(rects);
        StencilTuning tn;
        tn.cols = cols;
        tn.chunk_rows = chunk_rows;
        tn.nontemporal = nontemporal;
        tn.xcd_remap = xcd_remap;
        tn.vec = vec;
        tn.kernel = kernel;
        tn.stages = stages;
        if (gpu)
          stencilk_rects_gpu(K, P<double>(T2), P<const double>(T), P<const double>(iCp), nx, ny,
                             r.data(), (int)r.size(), to_coef(coef), tn, S(stream));
        else {
          // the CPU twin of the kernel's arithmetic: fast5 (kernels 5-9, 11, 12), the
          // split fast-math form (14, 15) or canonical
          const bool f5 = (kernel >= 5 && kernel <= 9) || kernel == 11 || kernel == 12 ||
                          kernel == 16 || kernel == 17 || kernel == 19 ||
                          kernel == 20 || kernel == 21 || kernel == 22 || kernel == 23 ||
                          kernel == 25 || kernel == 26 || kernel == 27;
          const bool f6 = kernel == 14 || kernel == 15;
          py::gil_scoped_release nogil;
          if (f6)
            stencilk6_rects_cpu(K, P<double>(T2), P<const double>(T), P<const double>(iCp), nx,
                                ny, r.data(), (int)r.size(), to_coef(coef));
          else if (f5)
            stencilk5_rects_cpu(K, P<double>(T2), P<const double>(T), P<const double>(iCp), nx,
                                ny, r.data(), (int)r.size(), to_coef(coef));
          else
            stencilk_rects_cpu(K, P<double>(T2), P<const double>(T), P<const double>(iCp), nx,
                               ny, r.data(), (int)r.size(), to_coef(coef));
        }
      },
      py::arg("K"), py::arg("T2"), py::arg("T"), py::arg("iCp"), py::arg("nx"), py::arg("ny"),
      py::arg("rects"), py::arg("coef"), py::arg("chunk_rows") = 16, py::arg("nontemporal") = 3,
      py::arg("stream") = 0, py::arg("gpu") = true, py::arg("xcd_remap") = -1,
      py::arg("vec") = 2, py::arg("kernel") = 0, py::arg("stages") = 0, py::arg("cols") = 0);
  m.def(
      "stream_copy",
      [](uintptr_t b, uintptr_t a, int64_t n, uintptr_t s, int nt, int blocks) {
        stream_copy_gpu(P<double>(b), P<const double>(a), n, nt, blocks, S(s));
      },
      py::arg("b"), py::arg("a"), py::arg("n"), py::arg("stream"), py::arg("nt") = 0,
      py::arg("blocks") = 0);
  m.def(
      "stream_triad",
      [](uintptr_t c, uintptr_t a, uintptr_t b, double x, int64_t n, uintptr_t s, int nt,
         int blocks) {
        stream_triad_gpu(P<double>(c), P<const double>(a), P<const double>(b), x, n, nt, blocks,
                         S(s));
      },
      py::arg("c"), py::arg("a"), py::arg("b"), py::arg("x"), py::arg("n"), py::arg("stream"),
      py::arg("nt") = 0, py::arg("blocks") = 0);

  m.def("flux", [](uintptr_t qx, uintptr_t qy, uintptr_t T, int64_t nx, int64_t ny, double mlam,
                   double rdx, double rdy, uintptr_t stream, bool gpu) {
    if (gpu)
      flux_gpu(P<double>(qx), P<double>(qy), P<const double>(T), nx, ny, mlam, rdx, rdy,
               S(stream));
    else
      flux_cpu(P<double>(qx), P<double>(qy), P<const double>(T), nx, ny, mlam, rdx, rdy);
  });
  m.def("residual", [](uintptr_t dTdt, uintptr_t qx, uintptr_t qy, uintptr_t iCp, int64_t nx,
                       int64_t ny, double rdx, double rdy, uintptr_t stream, bool gpu) {
    if (gpu)
      residual_gpu(P<double>(dTdt), P<const double>(qx), P<const double>(qy),
                   P<const double>(iCp), nx, ny, rdx, rdy, S(stream));
    else
      residual_cpu(P<double>(dTdt), P<const double>(qx), P<const double>(qy),
                   P<const double>(iCp), nx, ny, rdx, rdy);
  });
  m.def("update", [](uintptr_t T, uintptr_t dTdt, int64_t nx, int64_t ny, double dt,
                     uintptr_t stream, bool gpu) {
    if (gpu)
      update_gpu(P<double>(T), P<const double>(dTdt), nx, ny, dt, S(stream));
    else
      update_cpu(P<double>(T), P<const double>(dTdt), nx, ny, dt);
  });
  m.def("init_gaussian", [](uintptr_t T, int64_t nx, int64_t ny, const Geom& g, double lx,
                            double ly, uintptr_t stream, bool gpu) {
    if (gpu)
      init_gaussian_gpu(P<double>(T), nx, ny, to_geom(g), lx, ly, S(stream));
    else
      init_gaussian_cpu(P<double>(T), nx, ny, to_geom(g), lx, ly);
  });
  m.def("init_random", [](uintptr_t A, int64_t nx, int64_t ny, const Geom& g, uint64_t seed,
                          double lo, double hi, uintptr_t stream, bool gpu) {
    if (gpu)
      init_random_gpu(P<double>(A), nx, ny, to_geom(g), seed, lo, hi, S(stream));
    else
      init_random_cpu(P<double>(A), nx, ny, to_geom(g), seed, lo, hi);
  });
  m.def("fill", [](uintptr_t A, int64_t n, double v, uintptr_t stream) {
    fill_gpu(P<double>(A), n, v, S(stream));
  });
  m.def("copy2d", [](uintptr_t dst, int64_t dst_ld, uintptr_t src, int64_t src_ld, int64_t n_o,
                     int64_t n_k, int elem_bytes, uintptr_t stream, bool gpu) {
    if (gpu)
      copy2d_gpu(P<void>(dst), dst_ld, P<const void>(src), src_ld, n_o, n_k, elem_bytes,
                 S(stream));
    else
      copy2d_cpu(P<void>(dst), dst_ld, P<const void>(src), src_ld, n_o, n_k, elem_bytes);
  });
  // copies: [(dst, dst_ld, src, src_ld, n_o, n_k)], one element size, one launch
  m.def("copy2d_batch", [](const std::vector<std::tuple<uintptr_t, int64_t, uintptr_t, int64_t,
                                                        int64_t, int64_t>>& copies,
                           int elem_bytes, uintptr_t stream, bool gpu) {
    std::vector<Copy2d> c;
    for (const auto& t : copies)
      c.push_back({P<void>(std::get<0>(t)), std::get<1>(t), P<const void>(std::get<2>(t)),
                   std::get<3>(t), std::get<4>(t), std::get<5>(t)});
    if (gpu)
      copy2d_batch_gpu(c.data(), (int)c.size(), elem_bytes, S(stream));
    else
      copy2d_batch_cpu(c.data(), (int)c.size(), elem_bytes);
  });
  m.def("copy2d_batch_max", [] { return kCopy2dBatch; });
  // the IPC transport's stream-ordered flag kernels (csrc/kernels/flags.hip)
  m.def(
      "flag_wait",
      [](uintptr_t flag, uint64_t want, double timeout_s, uintptr_t err, uint32_t code,
         uintptr_t stream) {
        flag_wait_gpu(P<const uint64_t>(flag), want, timeout_s, P<uint32_t>(err), code, S(stream));
      },
      py::call_guard<py::gil_scoped_release>());
  m.def(
      "flag_write",
      [](uintptr_t flag, uint64_t value, uintptr_t stream) {
        flag_write_gpu(P<uint64_t>(flag), value, S(stream));
      },
      py::call_guard<py::gil_scoped_release>());
  m.def("reduce_workspace_doubles", &reduce_workspace_doubles);
  m.def("reduce_gpu", [](uintptr_t A, int64_t n, int op, uintptr_t out, uintptr_t ws,
                         uintptr_t stream) {
    reduce_gpu(P<const double>(A), n, op, P<double>(out), P<double>(ws), S(stream));
  });
  m.def("reduce_cpu",
        [](uintptr_t A, int64_t n, int op) { return reduce_cpu(P<const double>(A), n, op); });
  m.def("diag_string", &diag_string);  // RMA_DIAG, validated (unknown key: error)
  m.def("diag_value", [](const std::string& k) { return diag_value(k.c_str()); });
  m.def("env_double", &env_double);
  m.def("env_choice", &env_choice);
  m.def("field_stats_workspace_doubles", &field_stats_workspace_doubles);
  m.def("field_stats_gpu", [](uintptr_t A, int64_t n, uintptr_t out3, uintptr_t ws,
                              uintptr_t stream) {
    field_stats_gpu(P<const double>(A), n, P<double>(out3), P<double>(ws), S(stream));
  });
  m.def("field_stats_cpu", [](uintptr_t A, int64_t n) {
    double o[3];
    field_stats_cpu(P<const double>(A), n, o);
    return std::make_tuple(o[0], o[1], o[2]);
  });

  // ---------------- topology ----------------
  m.def("dims_create", &dims_create, py::arg("nprocs"), py::arg("dims"));
  m.attr("PROC_NULL") = kProcNull;
  py::class_<CartTopology>(m, "CartTopology")
      .def(py::init<int, std::array<int, 3>, std::array<int, 3>>(), py::arg("nprocs"),
           py::arg("dims"), py::arg("periods"))
      .def_property_readonly("nprocs", &CartTopology::nprocs)
      .def_property_readonly("dims", &CartTopology::dims)
      .def_property_readonly("periods", &CartTopology::periods)
      .def("coords", &CartTopology::coords)
      .def("rank_of", &CartTopology::rank_of)
      .def("shift", &CartTopology::shift)
      .def("neighbors", &CartTopology::neighbors)
      .def("diagonals", &CartTopology::diagonals);

  // ---------------- communication ----------------
  py::enum_<DType>(m, "DType")
      .value("float64", DType::kFloat64)
      .value("float32", DType::kFloat32)
      .value("int64", DType::kInt64)
      .value("int32", DType::kInt32)
      .value("uint8", DType::kUInt8);
  py::enum_<RedOp>(m, "RedOp")
      .value("sum", RedOp::kSum)
      .value("max", RedOp::kMax)
      .value("min", RedOp::kMin)
      .value("prod", RedOp::kProd);
  py::class_<P2PTransport>(m, "P2PTransport")
      .def_property_readonly("rank", &P2PTransport::rank)
      .def_property_readonly("size", &P2PTransport::size)
      .def("group_start", &P2PTransport::group_start)
      .def("group_end", &P2PTransport::group_end, py::call_guard<py::gil_scoped_release>())
      .def("send", [](P2PTransport& c, uintptr_t buf, size_t bytes, int peer,
                      uintptr_t s) { c.send(P<const void>(buf), bytes, peer, S(s)); },
           py::call_guard<py::gil_scoped_release>())
      .def("recv", [](P2PTransport& c, uintptr_t buf, size_t bytes, int peer,
                      uintptr_t s) { c.recv(P<void>(buf), bytes, peer, S(s)); },
           py::call_guard<py::gil_scoped_release>());
  py::class_<LoopbackHub, std::shared_ptr<LoopbackHub>>(m, "LoopbackHub")
      .def(py::init<int, double>(), py::arg("nranks"), py::arg("timeout_s") = 60.0)
      .def_property_readonly("size", &LoopbackHub::size);
  py::class_<LoopbackEndpoint, P2PTransport>(m, "LoopbackEndpoint")
      .def(py::init<std::shared_ptr<LoopbackHub>, int>(), py::arg("hub"), py::arg("rank"));
  py::class_<IpcTransport, P2PTransport>(m, "IpcTransport")
      .def(py::init<int, int, int, const std::vector<int>&, size_t, const std::string&, double,
                    int>(),
           py::arg("rank"), py::arg("size"), py::arg("device"), py::arg("peers"),
           py::arg("mailbox_bytes"), py::arg("token"), py::arg("timeout_s") = 300.0,
           py::arg("mode") = -1)
      .def("export_for", [](const IpcTransport& t, int p) { return py::bytes(t.export_for(p)); })
      .def("connect", [](IpcTransport& t, int p, py::bytes blob) { t.connect(p, blob); })
      .def("unlink_shm", &IpcTransport::unlink_shm)
      .def("abort_waits", &IpcTransport::abort_waits)
      .def("check_error", &IpcTransport::check_error)
      .def_property_readonly("connected", &IpcTransport::connected)
      .def_property_readonly("mailbox_bytes", &IpcTransport::mailbox_bytes)
      .def_property_readonly("mode",
                             [](const IpcTransport& t) {
                               return t.mode() == IpcTransport::Mode::kStream ? "stream" : "host";
                             })
      .def_property_readonly("poisoned", &IpcTransport::poisoned)
      .def_property_readonly("host_waits", &IpcTransport::host_waits);
  py::class_<IpcMap>(m, "IpcMap")
      .def(py::init<>())
      .def_static("export_ptr",
                  [](uintptr_t p) { return py::bytes(IpcMap::export_ptr((const void*)p)); })
      .def("open", [](IpcMap& m, py::bytes blob) { return (uintptr_t)m.open(blob); })
      .def("close_all", &IpcMap::close_all)
      .def_property_readonly("mappings", &IpcMap::mappings);
  py::class_<RcclComm, P2PTransport>(m, "RcclComm")
      .def_static("unique_id", []() { return py::bytes(RcclComm::unique_id()); })
      .def(py::init([](int nranks, int rank, py::bytes uid, int device, double init_timeout_s) {
             std::string s = uid;
             py::gil_scoped_release nogil;
             return new RcclComm(nranks, rank, s, device, init_timeout_s);
           }),
           py::arg("nranks"), py::arg("rank"), py::arg("uid"), py::arg("device"),
           py::arg("init_timeout_s") = 0.0)
      .def_property_readonly("nonblocking", &RcclComm::nonblocking)
      .def_property_readonly("data_blocking", &RcclComm::data_blocking)
      .def_property_readonly("device", &RcclComm::device)
      .def("count", &RcclComm::count)
      .def("allreduce",
           [](RcclComm& c, uintptr_t sb, uintptr_t rb, size_t count, DType dt, RedOp op,
              uintptr_t s) { c.allreduce(P<const void>(sb), P<void>(rb), count, dt, op, S(s)); })
      .def("broadcast",
           [](RcclComm& c, uintptr_t sb, uintptr_t rb, size_t count, DType dt, int root,
              uintptr_t s) { c.broadcast(P<const void>(sb), P<void>(rb), count, dt, root, S(s)); })
      .def("gather", [](RcclComm& c, uintptr_t sb, uintptr_t rb, size_t bytes, int root,
                        uintptr_t s) { c.gather(P<const void>(sb), P<void>(rb), bytes, root, S(s)); })
      .def(
          "barrier", [](RcclComm& c, uintptr_t s, double t) { c.barrier(S(s), t); },
          py::arg("stream"), py::arg("timeout_s") = 300.0, py::call_guard<py::gil_scoped_release>())
      .def(
          "wait", [](RcclComm& c, uintptr_t s, double t) { c.wait(S(s), t); }, py::arg("stream"),
          py::arg("timeout_s") = 300.0, py::call_guard<py::gil_scoped_release>())
      .def("check_async", &RcclComm::check_async)
      .def("abort", &RcclComm::abort)
      .def_property_readonly("aborted", &RcclComm::aborted);

  py::class_<HaloExchanger>(m, "HaloExchanger")
      .def(py::init([](P2PTransport* comm, int self_rank,
                       std::array<std::array<int, 2>, 3> nbr) {
             return new HaloExchanger(comm, self_rank, nbr);
           }),
           py::arg("comm").none(true), py::arg("self_rank"), py::arg("neighbors"),
           py::keep_alive<1, 2>())
      .def(
          "exchange",
          [](HaloExchanger& h, const std::vector<FieldT>& fields, uintptr_t s, int mask) {
            auto f = to_fields(fields);
            py::gil_scoped_release nogil;  // loopback transports block on peer threads
            h.exchange(f, S(s), mask);
          },
          py::arg("fields"), py::arg("stream"), py::arg("dims_mask") = 7)
      .def(
          "prepare",
          [](HaloExchanger& h, const std::vector<FieldT>& fields, int mask) {
            h.prepare(to_fields(fields), mask);
          },
          py::arg("fields"), py::arg("dims_mask") = 7)
      .def(
          "exchange_merged",
          [](HaloExchanger& h, const std::vector<FieldT>& fields, uintptr_t s) {
            auto f = to_fields(fields);
            py::gil_scoped_release nogil;
            h.exchange_merged(f, S(s));
          },
          py::arg("fields"), py::arg("stream"))
      .def("set_diagonals", &HaloExchanger::set_diagonals)
      .def_property_readonly("has_diagonals", &HaloExchanger::has_diagonals)
      .def_property_readonly("diagonals", &HaloExchanger::diagonals)
      .def("active", &HaloExchanger::active)
      .def("capturable", &HaloExchanger::capturable)
      .def("set_self_via_transport", &HaloExchanger::set_self_via_transport)
      .def_property_readonly("neighbors", &HaloExchanger::neighbors)
      .def_property_readonly("bytes_sent_last", &HaloExchanger::bytes_sent_last)
      .def_property_readonly("plan_hits", &HaloExchanger::plan_hits)
      .def_property_readonly("plan_misses", &HaloExchanger::plan_misses);

  // ---------------- executor ----------------
  m.def("pipe_chunk_rows", &pipe_chunk_rows, py::arg("K"), py::arg("ny"),
        py::arg("canonical") = false);
  m.def("default_chunk_k", [](int K, int64_t ny) { return default_tune_k(K, ny).chunk_rows; },
        py::arg("K"), py::arg("ny"));
  m.def("plan_passes", &plan_passes, py::arg("nsteps"), py::arg("costs"));
  m.def("default_pass_costs", &default_pass_costs, py::arg("kmax"), py::arg("fast5"),
        py::arg("cells") = 0.0);
  m.def("pipe_default_stages", &pipe_default_stages, py::arg("K"));
  m.def("pipe_default_cols", &pipe_default_cols, py::arg("K"), py::arg("stages"),
        py::arg("arith") = 0);
  m.def("pipe_has_cols", &pipe_has_cols, py::arg("K"), py::arg("stages"), py::arg("arith"),
        py::arg("cols"));
  m.def("pipe_vec", &pipe_vec, py::arg("K"), py::arg("stages"), py::arg("arith"), py::arg("nx"),
        py::arg("requested"), py::arg("aligned16") = true);
  m.def("pipe_max_k", []() { return kPipeMaxK; });
  m.def(
      "pass_geometry",
      [](int64_t nx, int64_t ny, int K, std::array<std::array<int, 2>, 3> nbr, bool hide,
         int64_t bwx, int64_t bwy, int64_t olx, int64_t oly) {
        const PassGeom g = pass_geometry(nx, ny, K, nbr, hide, bwx, bwy, olx, oly);
        std::vector<Rect4> fr;
        for (auto& r : g.frame) fr.push_back(from_rect(r));
        return std::make_tuple(from_rect(g.out), fr, from_rect(g.interior));
      },
      py::arg("nx"), py::arg("ny"), py::arg("K"), py::arg("neighbors"), py::arg("hide"),
      py::arg("bwx"), py::arg("bwy"), py::arg("olx"), py::arg("oly"));
  m.def(
      "frame_layout",
      [](int64_t ny, std::array<std::array<int, 2>, 3> nbr) {
        const FrameLayout f = frame_layout(ny, nbr);
        return std::make_tuple(f.chunk_div, f.bands);
      },
      py::arg("ny"), py::arg("neighbors"));
  m.def(
      "canonical_kernel_k",
      [](int K, int64_t ny) {
        const StencilTuning t = canonical_tune_k(K, ny);
        return std::make_tuple(t.kernel, t.vec, t.chunk_rows);
      },
      py::arg("K"), py::arg("ny"));
  m.def(
      "fast_kernel_k",
      [](int K, int64_t ny, const Coef4& coef) {
        const StencilTuning t = fast_tune_k(K, ny, to_coef(coef));
        return std::make_tuple(t.kernel, t.vec, t.chunk_rows);
      },
      py::arg("K"), py::arg("ny"), py::arg("coef"));
  py::class_<DiffusionExecutor>(m, "Executor")
      .def(py::init([](uintptr_t T, uintptr_t T2, uintptr_t iCp, int64_t nx, int64_t ny, int mode,
                       const Coef4& coef, int chunk_rows, int nontemporal, int kernel,
                       int64_t bwx, int64_t bwy, int use_graph, int graph_steps,
                       HaloExchanger* halo, uintptr_t qx, uintptr_t qy, uintptr_t dTdt,
                       int unroll, int vec, int temporal, int64_t olx, int64_t oly,
                       int chunk2, int unroll2, int fast_math) {
             ExecParams p;
             p.fast_math = fast_math;
             p.temporal = temporal;
             p.olx = olx;
             p.oly = oly;
             p.tune2 = default_tune_k(temporal, ny);  // measured defaults
             if (chunk2 > 0) p.tune2.chunk_rows = chunk2;
             p.chunk_rows2 = chunk2;  // 0: per pass depth
             if (temporal == 2) p.tune2.unroll = unroll2;
             p.tune2.nontemporal = nontemporal & 3;
             p.mode = static_cast<Mode>(mode);
             p.coef = to_coef(coef);
             p.tune.chunk_rows = chunk_rows;
             p.tune.nontemporal = nontemporal;
             p.tune.kernel = kernel;
             p.tune.unroll = unroll;
             p.tune.vec = vec;
             p.bwx = bwx;
             p.bwy = bwy;
             p.use_graph = use_graph;
             p.graph_steps = graph_steps;
             return new DiffusionExecutor(P<double>(T), P<double>(T2), P<const double>(iCp), nx,
                                          ny, p, halo, P<double>(qx), P<double>(qy),
                                          P<double>(dTdt));
           }),
           py::arg("T"), py::arg("T2"), py::arg("iCp"), py::arg("nx"), py::arg("ny"),
           py::arg("mode"), py::arg("coef"), py::arg("chunk_rows") = 4,
           py::arg("nontemporal") = 3, py::arg("kernel") = 0, py::arg("bwx") = 1,
           py::arg("bwy") = 1, py::arg("use_graph") = 0, py::arg("graph_steps") = 0,
           py::arg("halo").none(true) = nullptr, py::arg("qx") = 0, py::arg("qy") = 0,
           py::arg("dTdt") = 0, py::arg("unroll") = 4, py::arg("vec") = 2,
           py::arg("temporal") = 1, py::arg("olx") = 2, py::arg("oly") = 2,
           py::arg("chunk2") = 0, py::arg("unroll2") = 2, py::arg("fast_math") = 0,
           py::keep_alive<1, 16>())
      .def(
          "run", [](DiffusionExecutor& e, int64_t n, uintptr_t s) { e.run(n, S(s)); },
          py::arg("nsteps"), py::arg("stream"), py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("parity", &DiffusionExecutor::parity)
      .def_property_readonly("steps_done", &DiffusionExecutor::steps_done)
      .def_property_readonly("passes_done", &DiffusionExecutor::passes_done)
      .def_property_readonly("fused_passes", &DiffusionExecutor::fused_passes)
      .def("check_error", &DiffusionExecutor::check_error)
      .def("plan", &DiffusionExecutor::plan, py::arg("nsteps"))
      .def_property_readonly("pass_costs", &DiffusionExecutor::pass_costs)
      .def("prime", &DiffusionExecutor::prime, py::call_guard<py::gil_scoped_release>())
      .def("set_timing", &DiffusionExecutor::set_timing, py::arg("on"),
           py::call_guard<py::gil_scoped_release>())
      .def("timings",
           [](DiffusionExecutor& e) {
             std::vector<py::dict> out;
             std::vector<PassTiming> ts;
             {
               py::gil_scoped_release nogil;
               ts = e.timings();
             }
             for (const auto& t : ts) {
               py::dict d;
               d["K"] = t.K;
               d["frame_ms"] = t.frame_ms;
               d["halo_ms"] = t.halo_ms;
               d["interior_ms"] = t.interior_ms;
               d["pass_ms"] = t.pass_ms;
               d["exposed_halo_ms"] = t.exposed_halo_ms;
               out.push_back(d);
             }
             return out;
           })
      .def(
          "set_direct",
          // peers: 8 tuples (rank, T ptr, T2 ptr, flag ptr) in DiffusionExecutor::kDirI/J
          // order; in_flags: this rank's 8 device words (0: none)
          [](DiffusionExecutor& e, const std::vector<std::tuple<int, uintptr_t, uintptr_t, uintptr_t>>& peers,
             uintptr_t in_flags, bool host_wait) {
            RMA_CHECK_ARG(peers.size() == 8, "set_direct: 8 directions, got " << peers.size());
            std::array<DiffusionExecutor::DirectPeer, 8> a{};
            for (int d = 0; d < 8; ++d) {
              a[d].rank = std::get<0>(peers[d]);
              a[d].T = P<double>(std::get<1>(peers[d]));
              a[d].T2 = P<double>(std::get<2>(peers[d]));
              a[d].flag = P<uint64_t>(std::get<3>(peers[d]));
            }
            e.set_direct(a, P<uint64_t>(in_flags), host_wait);
          },
          py::arg("peers"), py::arg("in_flags"), py::arg("host_wait") = false,
          py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("direct", &DiffusionExecutor::direct)
      .def_property_readonly("direct_passes", &DiffusionExecutor::direct_passes)
      .def_property_readonly_static("direct_dirs", [](py::object) {
        std::vector<std::pair<int, int>> v;
        for (int d = 0; d < 8; ++d)
          v.emplace_back(DiffusionExecutor::kDirI[d], DiffusionExecutor::kDirJ[d]);
        return v;
      })
      .def("set_solo", &DiffusionExecutor::set_solo, py::arg("on"),
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("solo", &DiffusionExecutor::solo)
      .def_property_readonly("frame_rects",
                             [](const DiffusionExecutor& e) {
                               std::vector<Rect4> v;
                               for (auto& r : e.frame_rects()) v.push_back(from_rect(r));
                               return v;
                             })
      .def_property_readonly("interior_rect",
                             [](const DiffusionExecutor& e) { return from_rect(e.interior_rect()); })
      .def(
          "geometry",
          [](DiffusionExecutor& e, int K) {
            const PassGeom& g = e.geometry(K);
            auto rl = [](const std::vector<Rect>& v) {
              std::vector<Rect4> o;
              for (auto& r : v) o.push_back(from_rect(r));
              return o;
            };
            py::dict d;
            d["aligned"] = g.aligned;
            d["out"] = from_rect(g.out);
            d["frame"] = rl(g.frame);
            d["frame_wide"] = rl(g.frame_wide);
            d["frame_tall"] = rl(g.frame_tall);
            d["interior"] = from_rect(g.interior);
            d["tasks"] = g.tasks();  // the interior grid's tasks (fused / one-launch policy)
            return d;
          },
          py::arg("K"));

  // ---------------- tracing ----------------
  m.def("trace_enable", &trace_enable);
  m.def("trace_enabled", &trace_enabled);
  m.def("trace_push", [](const std::string& s) { trace_push(s.c_str()); });
  m.def("trace_pop", &trace_pop);
  m.def("trace_mark", [](const std::string& s) { trace_mark(s.c_str()); });
}
