// Instantiation of the register-factor pipelined kernel (stencil_pipe.h,
// "piper", arithmetic kArFast5Reg) at K = 20, the depth of the driver's
// 20-step pass, in a unit of its own: the build compiles it with LLVM's
// iterative-ILP machine scheduler (rocm_mpi_amd/_build.py UNIT_FLAGS). Same
// instructions, another order: -0.7 % per K = 20 pass at 101376^2, same box,
// two alternating rounds (66.40 vs 66.89 ms); at K = 24 the same strategy is
// +0.4 % and max-ILP is worse at both (profiles/r6/sched_strategy_ab.md).
#include "stencil_pipe.h"

namespace rma {
namespace pipe {

bool dispatch_r20(int K, int S, int V, int ar, const PipeLaunch& a) {
  if (ar != kArFast5Reg) return false;
  RMA_PIPE_CASE(20, 4, kArFast5Reg)
  return false;
}

}  // namespace pipe
}  // namespace rma
