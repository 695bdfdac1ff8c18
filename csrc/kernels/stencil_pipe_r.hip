// Instantiations of the any-K pipelined kernel (stencil_pipe.h), unit r:
// fast5 arithmetic with register-resident factor rows ("piper", arithmetic
// kArFast5Reg): no LDS factor ring, one factor hand-off row per stage
// boundary. Default stage split, K = 12..24.
#include "stencil_pipe.h"

namespace rma {
namespace pipe {

bool dispatch_r(int K, int S, int V, int ar, const PipeLaunch& a) {
  if (ar != kArFast5Reg) return false;
  RMA_PIPE_CASE(12, 4, kArFast5Reg)
  RMA_PIPE_CASE(16, 4, kArFast5Reg)
  RMA_PIPE_CASE(20, 4, kArFast5Reg)
  RMA_PIPE_CASE(24, 4, kArFast5Reg)
  return false;
}

}  // namespace pipe
}  // namespace rma
