// librma_lab.so, 5-cells-per-lane unit: the any-K pipelined kernel
// (stencil_pipe.h) with fast5 arithmetic at 5 cells per lane (320-column
// strips, v-major LDS rows, delayed factor ring), default stage split. An
// experiment kept for sweeps (bench/pass_sweep.py --pipe5, RMA_DIAG=pipe_fast=pipe5):
// 3.5 % less fp64 work and 23 % fewer lane moves per cell update at K = 20,
// but only 0.8-1.6 % faster per pass at 101120^2 (profiles/SUMMARY_r3.md),
// about what the register-factor kernel (piper) gains at K = 20 without the
// nx % 5 == 0 restriction. K = 16..20: at K >= 21 the 6-level stages need
// more than the 256 VGPRs of 2 waves per SIMD and spill (hipcc
// -Rpass-analysis=kernel-resource-usage: K=20 236 VGPRs, K=21..24 256 + 155..217
// spilled), so those depths stay at 4 cells per lane.
#include "../kernels/lab_hooks.h"

namespace rma {
namespace pipe {

#define RMA_PIPE_CASE5(KK)                           \
  if (K == KK) {                                     \
    launch<KK, 4, 5, kArFast5>(a);                   \
    return true;                                     \
  }

bool dispatch_v5(int K, int S, int V, int ar, const PipeLaunch& a) {
  if (V != 5 || !pipe_has_v5(K, S, ar)) return false;
  RMA_PIPE_CASE5(16)
  RMA_PIPE_CASE5(17)
  RMA_PIPE_CASE5(18)
  RMA_PIPE_CASE5(19)
  RMA_PIPE_CASE5(20)
  return false;
}

}  // namespace pipe
}  // namespace rma
