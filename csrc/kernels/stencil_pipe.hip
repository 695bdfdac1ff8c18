// Host side of the any-K stage-pipelined kernel (stencil_pipe.h): argument
// checks, strip/chunk planning and the (K, S, V, arithmetic) dispatch over the
// instantiation units stencil_pipe_{a,b,c}.hip (default stage split); any
// other (K, S, V, C, arithmetic) goes to the lab library (lab_hooks.h).
#include <hip/hip_runtime.h>

#include <cmath>

#include "rma/hip_check.h"
#include "rma/kernels.h"
#include "lab_hooks.h"
#include "stencil_pipe.h"

namespace rma {

// pipe_default_stages, pipe_has, pipe_has_cols, pipe_default_cols, pipe_vec:
// kernel_select.cpp (host code, shared with the sanitizer builds)

void stencil_pipe_occupancy(int K, int stages, int arith, int V, int occ[2]) {
  const int S = stages > 0 ? stages : pipe_default_stages(K);
  RMA_CHECK_ARG(pipe_has(K, S, arith), "no pipelined kernel for K=" << K << " S=" << S
                                                                   << " arithmetic " << arith);
  pipe::PipeLaunch a{nullptr, nullptr, nullptr, 0, 0, nullptr, 0, StencilCoef{}, 1, 0, nullptr};
  a.occupancy = occ;
  occ[0] = occ[1] = 0;
  // lab variants (other splits, 5 cells per lane, ...) have no direct-store
  // instantiation: {0, 0}, which the executor prices as unavailable
  if (V != 5)
    (void)(pipe::dispatch_r20(K, S, V, arith, a) || pipe::dispatch_r24(K, S, V, arith, a) ||
           pipe::dispatch_r(K, S, V, arith, a) ||
           pipe::dispatch_a(K, S, V, arith, a) ||
           pipe::dispatch_b(K, S, V, arith, a) || pipe::dispatch_c(K, S, V, arith, a));
}

void stencil_pipe_rects_gpu(int K, int stages, int arith, double* T2, const double* T,
                            const double* iCp, int64_t nx, int64_t ny, const Rect* rects,
                            int nrects, const StencilCoef& c, const StencilTuning& tune,
                            stream_t stream) {
  const int S = stages > 0 ? stages : pipe_default_stages(K);
  RMA_CHECK_ARG(K >= 1 && K <= kPipeMaxK,
                "pipelined K-step kernel: 1 <= K <= " << kPipeMaxK << ", got " << K);
  RMA_CHECK_ARG(pipe_has(K, S, arith), "no pipelined kernel instantiated for K=" << K << " S=" << S
                                                                             << " arithmetic " << arith);
  RMA_CHECK_ARG(arith >= 0 && arith <= 20, "pipelined kernel arithmetic " << arith);
  if (arith == pipe::kArFast5RegIso) {
    const double ax = (-c.mlam) * c.rdx * c.rdx, ay = (-c.mlam) * c.rdy * c.rdy;
    RMA_CHECK_ARG(ay / ax == 1.0, "the isotropic fast-math kernel needs ry = (dx/dy)^2 == 1");
  }
  const bool canonical = arith == pipe::kArCanon;
  RMA_CHECK_ARG(canonical || fast5_ok(c),
                "the fast5 arithmetic folds dy^-2/dx^-2 into one factor: needs lam != 0 and "
                "finite coefficients");
  RMA_CHECK_ARG(nrects >= 0 && nrects <= kMaxRects, "nrects=" << nrects);
  RMA_CHECK_ARG(nx >= 3 && ny >= 3, "grid too small: nx=" << nx << " ny=" << ny);
  RMA_CHECK_ARG(ny < (int64_t(1) << 30), "rows are indexed in 32 bits, ny = " << ny);
  RMA_CHECK_ARG(T2 != T, "multi-step kernel cannot run in place");
  RMA_CHECK_ARG(tune.chunk_rows >= 1, "chunk_rows=" << tune.chunk_rows);
  for (int i = 0; i < nrects; ++i) {
    const Rect& r = rects[i];
    if (r.empty()) continue;
    RMA_CHECK_ARG(r.x0 >= 1 && r.x1 <= nx - 1 && r.y0 >= 1 && r.y1 <= ny - 1,
                  "rect " << i << " outside the interior of " << nx << "x" << ny);
  }
  const bool aligned = ((reinterpret_cast<uintptr_t>(T) & 15) == 0) &&
                       ((reinterpret_cast<uintptr_t>(T2) & 15) == 0) &&
                       ((reinterpret_cast<uintptr_t>(iCp) & 15) == 0);
  const int V = pipe_vec(K, S, arith, nx, tune.vec, aligned);
  int C = tune.cols > 0 ? tune.cols : pipe_default_cols(K, S, arith);
  RMA_CHECK_ARG(pipe_has_cols(K, S, arith, C), "no pipelined kernel with " << C
                                                   << " column waves for K=" << K << " S=" << S
                                                   << " arithmetic " << arith);
  if (V != 4) C = 1;  // the 2-column blocks need 16-B pairs at 4 cells per lane
  const int remap = tune.xcd_remap >= 0 ? tune.xcd_remap : (nx > 65536 ? 1 : 0);
  pipe::PipeLaunch a{T2, T, iCp, nx, ny, rects, nrects, c, tune.chunk_rows, remap,
                     as_stream(stream)};
  if (tune.direct && tune.direct->on) {
    const DirectStores& D = *tune.direct;
    // every image lies inside the destination tile (same nx x ny as this one):
    // the x-ranges shifted by -i * sx, the y-ranges by -j * syr
    auto inside = [](int64_t a0, int64_t a1, int64_t shift, int64_t n) {
      return a0 >= a1 || (a0 + shift >= 0 && a1 + shift <= n);
    };
    RMA_CHECK_ARG(inside(D.xm0, D.xm1, D.sx, nx) && inside(D.xp0, D.xp1, -D.sx, nx) &&
                      inside(D.ym0, D.ym1, D.syr, ny) && inside(D.yp0, D.yp1, -D.syr, ny),
                  "direct-store ranges map outside the " << nx << "x" << ny << " tile");
    for (int d = 0; d < 8; ++d) {
      if (!D.dst[d]) continue;
      RMA_CHECK_ARG(V < 2 || (D.sx % 2 == 0 && (D.syr * nx) % 2 == 0 &&
                              (reinterpret_cast<uintptr_t>(D.dst[d]) & 15) == 0),
                    "direct store " << d << ": 16-byte stores need even shifts and an aligned "
                                       "destination");
    }
    a.direct = &D;
  }
  if (tune.signal || tune.signal_rects > 0) {  // lead rects (with or without the signal)
    RMA_CHECK_ARG(tune.signal_rects >= 1 && tune.signal_rects < nrects,
                  "signal rects " << tune.signal_rects << " of " << nrects);
    a.sig = tune.signal;
    a.sig_rects = tune.signal_rects;
    RMA_CHECK_ARG(tune.signal_chunk_rows >= 0, "signal_chunk_rows=" << tune.signal_chunk_rows);
    a.sig_chunk_rows = tune.signal_chunk_rows;
  }
  // V = 5 only in the lab (the core units' cases take any V other than 4 and 2 as 1)
  bool ok = C == 1 && V != 5 &&
            (pipe::dispatch_r20(K, S, V, arith, a) || pipe::dispatch_r24(K, S, V, arith, a) ||
           pipe::dispatch_r(K, S, V, arith, a) ||
             pipe::dispatch_a(K, S, V, arith, a) ||
             pipe::dispatch_b(K, S, V, arith, a) || pipe::dispatch_c(K, S, V, arith, a));
  if (!ok) {  // alternative stage splits, pipeb, two-column blocks, 5 cells: librma_lab.so
    if (!lab_hooks().pipe)
      lab_missing("this pipelined kernel variant (stages / arithmetic / cols / 5 cells per lane)");
    ok = lab_hooks().pipe(K, S, V, C, arith, a);
  }
  RMA_CHECK_ARG(ok, "pipelined kernel K=" << K << " S=" << S << " V=" << V << " C=" << C
                                           << " arithmetic=" << arith << " not instantiated");
  RMA_HIP_LAUNCH_CHECK();
}

}  // namespace rma
