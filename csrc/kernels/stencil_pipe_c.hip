// Instantiations of the any-K pipelined kernel (stencil_pipe.h), unit c:
// fast5 arithmetic, K = 13..24 (default stage split). Split over several units so the build compiles them in parallel.
#include "stencil_pipe.h"

namespace rma {
namespace pipe {

bool dispatch_c(int K, int S, int V, int ar, const PipeLaunch& a) {
  RMA_PIPE_CASE(13, 4, kArFast5)
  RMA_PIPE_CASE(14, 4, kArFast5)
  RMA_PIPE_CASE(15, 4, kArFast5)
  RMA_PIPE_CASE(16, 4, kArFast5)
  RMA_PIPE_CASE(17, 4, kArFast5)
  RMA_PIPE_CASE(18, 4, kArFast5)
  RMA_PIPE_CASE(19, 4, kArFast5)
  RMA_PIPE_CASE(20, 4, kArFast5)
  RMA_PIPE_CASE(21, 4, kArFast5)
  RMA_PIPE_CASE(22, 4, kArFast5)
  RMA_PIPE_CASE(23, 4, kArFast5)
  RMA_PIPE_CASE(24, 4, kArFast5)
  return false;
}

}  // namespace pipe
}  // namespace rma
