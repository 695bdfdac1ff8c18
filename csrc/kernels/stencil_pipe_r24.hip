// The executor's K = 24 pass: the register-factor pipelined kernel without the
// sched_barriers inside a level (arithmetic kArFast5RegNoSB, bitwise equal to
// piper), compiled with LLVM's iterative-ILP machine scheduler
// (rocm_mpi_amd/_build.py UNIT_FLAGS). With the default scheduler the barriers
// pay off (round 4); under iterative ILP the free schedule is faster: K = 24
// pass at 101376^2 77.75 vs 78.79 ms (-1.3 %, same process, 4 interleaved
// rounds), while at K = 20 it is +0.9 % (profiles/r6/sched_strategy_ab.md).
#include "stencil_pipe.h"

namespace rma {
namespace pipe {

bool dispatch_r24(int K, int S, int V, int ar, const PipeLaunch& a) {
  if (ar != kArFast5RegNoSB) return false;
  RMA_PIPE_CASE(24, 4, kArFast5RegNoSB)
  return false;
}

}  // namespace pipe
}  // namespace rma
