// Instantiations of the any-K pipelined kernel (stencil_pipe.h), unit d:
// fast5 arithmetic, alternative stage splits and the ds_bpermute lane-move
// variant for sweeps. Split over several units so the build compiles them in parallel.
#include "stencil_pipe.h"

namespace rma {
namespace pipe {

bool dispatch_d(int K, int S, int V, int ar, const PipeLaunch& a) {
  RMA_PIPE_CASE(12, 3, kArFast5)
  RMA_PIPE_CASE(16, 8, kArFast5)
  RMA_PIPE_CASE(24, 8, kArFast5)
  RMA_PIPE_CASE(8, 4, kArFast5)
  RMA_PIPE_CASE(8, 1, kArFast5)
  RMA_PIPE_CASE(16, 4, kArFast5Perm)
  RMA_PIPE_CASE(20, 4, kArFast5Perm)
  RMA_PIPE_CASE(24, 4, kArFast5Perm)
  return false;
}

}  // namespace pipe
}  // namespace rma
