// Instantiations of the any-K pipelined kernel (stencil_pipe.h), unit d:
// fast5 arithmetic at 5 cells per lane (320-column strips, v-major LDS rows,
// delayed factor ring), default stage split, for the deep passes where the
// strip recompute dominates. K = 16..20: at K >= 21 the 6-level stages need
// more than the 256 VGPRs of 2 waves per SIMD and spill (hipcc
// -Rpass-analysis=kernel-resource-usage: K=20 236 VGPRs, K=21..24 256 + 155..217
// spilled), so those depths stay at 4 cells per lane.
#include "stencil_pipe.h"

namespace rma {
namespace pipe {

bool pipe_has_v5(int K, int S, int ar) {
  return ar == kArFast5 && S == 4 && K >= 16 && K <= 20;
}

#define RMA_PIPE_CASE5(KK)                           \
  if (K == KK) {                                     \
    launch<KK, 4, 5, kArFast5>(a);                   \
    return true;                                     \
  }

bool dispatch_d(int K, int S, int V, int ar, const PipeLaunch& a) {
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
