// Instantiations of the any-K pipelined kernel (stencil_pipe.h), unit r:
// fast5 arithmetic with register-resident factor rows ("piper", arithmetic
// kArFast5Reg): no LDS factor ring, one factor hand-off row per stage
// boundary; stage 0 prefetches T and 1/Cp three rows ahead by LDS-DMA, which
// keeps the prefetch out of the registers (K=24 234 VGPRs, K=20 201, K=16 161:
// 3 waves per SIMD, K=12 123: 4). Default stage split, K = 10..24. The
// executor's fast kernel from K = 14 (from K = 10 on tiles of >= 65536 rows):
// per pass at 101120^2 K=10..24 -0.7..-7 % against the ring kernel (K=20
// 68.69 vs 70.20 ms, K=24 79.03 vs 80.22); at 16384^2 K=10 / 12 slower
// (+12 / +7 %). profiles/SUMMARY_r3.md section 8.
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
  // K = 20: stencil_pipe_r20.hip
  RMA_PIPE_CASE(21, 4, kArFast5Reg)
  RMA_PIPE_CASE(22, 4, kArFast5Reg)
  RMA_PIPE_CASE(23, 4, kArFast5Reg)
  RMA_PIPE_CASE(24, 4, kArFast5Reg)
  return false;
}

}  // namespace pipe
}  // namespace rma
