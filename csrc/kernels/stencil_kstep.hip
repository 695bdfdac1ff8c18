// K explicit-Euler steps per pass (K = 2, 3, 4, 6, 8), the core's canonical
// overlapped-strip kernel (kernel 3: LDS 1/Cp ring + DPP lane moves; bitwise
// equal to K one-step launches), and the K-step dispatcher: kernels 9/10 go to
// the any-K pipelined kernels (stencil_pipe.hip), the other ids to the lab
// library (lab_hooks.h). The device templates and the scheme notes are in
// stencil_kstep.h.
#include "stencil_kstep.h"

#include <sstream>

#include "lab_hooks.h"

namespace rma {

namespace {
using namespace march;
LabHooks g_lab;
}  // namespace

void set_lab_hooks(const LabHooks& h) { g_lab = h; }
const LabHooks& lab_hooks() { return g_lab; }

void lab_missing(const char* what) {
  std::ostringstream m;
  m << what << " lives in librma_lab.so (csrc/lab: superseded / experimental kernels kept as "
    << "test oracles and for sweeps), which is not loaded: call "
    << "rocm_mpi_amd._native.load_lab() first";
  throw_error("kernel not in the core library", __FILE__, __LINE__, m.str());
}

void stencilk_rects_gpu(int K, double* T2, const double* T, const double* iCp, int64_t nx,
                        int64_t ny, const Rect* rects, int nrects, const StencilCoef& c,
                        const StencilTuning& tune, stream_t stream) {
  RMA_CHECK_ARG(tune.kernel >= 0 && tune.kernel <= 29, "unknown K-step kernel " << tune.kernel);
  RMA_CHECK_ARG(!tune.signal || tune.kernel >= 9,
                "a signalling (frame-first fused) launch needs a pipelined kernel, got " << tune.kernel);
  RMA_CHECK_ARG(!tune.direct || !tune.direct->on || tune.kernel >= 9,
                "direct-store halos need a pipelined kernel, got " << tune.kernel);
  if (tune.kernel >= 9) {  // any-K stage-pipelined kernels (stencil_pipe.h)
    stencil_pipe_rects_gpu(K, tune.stages, tune.kernel - 9, T2, T, iCp, nx, ny, rects, nrects,
                           c, tune, stream);
    return;
  }
  if (tune.kernel != 3) {
    std::ostringstream m;
    m << "K-step kernel " << tune.kernel;
    if (!g_lab.kstep) lab_missing(m.str().c_str());
    RMA_CHECK_ARG(g_lab.kstep(K, T2, T, iCp, nx, ny, rects, nrects, c, tune, stream),
                  "lab K-step kernel " << tune.kernel << " K=" << K << " not instantiated");
    return;
  }
  const kstep::KstepLaunch kl = kstep::check_launch(K, T2, T, iCp, nx, ny, rects, nrects, c, tune);
  const int V = kl.V, remap = kl.remap;
  RectList L;
  const int64_t total = plan_rects(L, rects, nrects, V, tune.chunk_rows, remap, false, K);
  if (L.n == 0) return;
  RMA_CHECK_ARG(total < (int64_t(1) << 31), "grid too large: " << total << " blocks");
  const dim3 grid((unsigned)total), block(kBlock);
  hipStream_t s = as_stream(stream);
  const bool nts = tune.nontemporal & 1;
#define RMA_K3(KK, VV, NTS)                                                                   \
  kstep::stencilk_ovl_kernel<KK, VV, NTS, true, true><<<grid, block, 0, s>>>(                 \
      T2, T, iCp, nx, ny, L, c, tune.chunk_rows, remap);
#define RMA_K3_V(KK)                                                    \
  if (V == 4) {                                                         \
    if (nts) { RMA_K3(KK, 4, true) } else { RMA_K3(KK, 4, false) }      \
  } else if (V == 2) {                                                  \
    if (nts) { RMA_K3(KK, 2, true) } else { RMA_K3(KK, 2, false) }      \
  } else {                                                              \
    if (nts) { RMA_K3(KK, 1, true) } else { RMA_K3(KK, 1, false) }      \
  }
  switch (K) {
    case 2: RMA_K3_V(2) break;
    case 3: RMA_K3_V(3) break;
    case 4: RMA_K3_V(4) break;
    case 6: RMA_K3_V(6) break;
    default: RMA_K3_V(8) break;
  }
#undef RMA_K3_V
#undef RMA_K3
  RMA_HIP_LAUNCH_CHECK();
}

}  // namespace rma
