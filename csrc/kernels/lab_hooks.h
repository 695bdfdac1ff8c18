// Registry of the kernels that live outside the core library: librma_lab.so
// (csrc/lab) holds the superseded and experimental kernels (the LDS-tiled
// one-step kernel, K-step kernels) that stay
// useful as test oracles and for sweeps (kernels 0-2, 4-8 of the overlapped-
// strip family, the pipelined kernel's alternative stage splits, its
// ds_bpermute variant and the two-column blocks). The core dispatches to them
// through these hooks, which the lab library installs from a static
// initialiser when it is loaded (rocm_mpi_amd._native.load_lab()); without
// it, asking for one of those kernels is a loud error.
#pragma once

#include "rma/kernels.h"
#include "stencil_pipe.h"

namespace rma {

struct LabHooks {
  // overlapped-strip K-step kernels other than 3; false: not held
  bool (*kstep)(int K, double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                const Rect* rects, int nrects, const StencilCoef& c, const StencilTuning& tune,
                stream_t stream) = nullptr;
  // pipelined (K, S, V, C, arithmetic) outside the default stage split
  bool (*pipe)(int K, int S, int V, int C, int arith, const pipe::PipeLaunch& a) = nullptr;
  // one-step kernels other than the march (tune.kernel 1: LDS-tiled)
  bool (*onestep)(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
                  const Rect* rects, int nrects, const StencilCoef& c, const StencilTuning& tune,
                  stream_t stream) = nullptr;
};

void set_lab_hooks(const LabHooks& h);
const LabHooks& lab_hooks();
[[noreturn]] void lab_missing(const char* what);

namespace lab {
bool kstep(int K, double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
           const Rect* rects, int nrects, const StencilCoef& c, const StencilTuning& tune,
           stream_t stream);
bool pipe(int K, int S, int V, int C, int arith, const pipe::PipeLaunch& a);
bool onestep(double* T2, const double* T, const double* iCp, int64_t nx, int64_t ny,
             const Rect* rects, int nrects, const StencilCoef& c, const StencilTuning& tune,
             stream_t stream);
}  // namespace lab

}  // namespace rma
