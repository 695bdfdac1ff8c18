// Instantiations of the any-K pipelined kernel (stencil_pipe.h), unit r:
// fast5 arithmetic with register-resident factor rows ("piper", arithmetic
// kArFast5Reg): no LDS factor ring, one factor hand-off row per stage
// boundary. Default stage split, K = 17..20 (5-level stages, 233 VGPRs at
// K = 20): the executor's kernel for those depths (K=20 pass at 101120^2:
// 68.07 vs 68.95 and 69.74 vs 71.21 ms, profiles/SUMMARY_r3.md). Where it does
// not pay: K = 12 (equal), K = 16 (198 VGPRs: 2 waves per SIMD instead of 3,
// 61.7 vs 56.4 ms), K = 21..24 (6-level stages need more than 256 VGPRs with
// the two-row T prefetch; 89.3 vs 78.8 ms at K = 24 with 6 spilled).
#include "stencil_pipe.h"

namespace rma {
namespace pipe {

bool dispatch_r(int K, int S, int V, int ar, const PipeLaunch& a) {
  if (ar != kArFast5Reg) return false;
  RMA_PIPE_CASE(10, 4, kArFast5Reg)
  RMA_PIPE_CASE(11, 4, kArFast5Reg)
  RMA_PIPE_CASE(12, 4, kArFast5Reg)
  RMA_PIPE_CASE(13, 4, kArFast5Reg)
  RMA_PIPE_CASE(14, 4, kArFast5Reg)
  RMA_PIPE_CASE(15, 4, kArFast5Reg)
  RMA_PIPE_CASE(16, 4, kArFast5Reg)
  RMA_PIPE_CASE(17, 4, kArFast5Reg)
  RMA_PIPE_CASE(18, 4, kArFast5Reg)
  RMA_PIPE_CASE(19, 4, kArFast5Reg)
  RMA_PIPE_CASE(20, 4, kArFast5Reg)
  RMA_PIPE_CASE(21, 4, kArFast5Reg)
  RMA_PIPE_CASE(22, 4, kArFast5Reg)
  RMA_PIPE_CASE(23, 4, kArFast5Reg)
  RMA_PIPE_CASE(24, 4, kArFast5Reg)
  return false;
}

}  // namespace pipe
}  // namespace rma
