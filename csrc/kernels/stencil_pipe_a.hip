// Instantiations of the any-K pipelined kernel (stencil_pipe.h), unit a:
// canonical flux arithmetic, K = 1..24 (default stage split). Split over several units so the build compiles them in parallel.
#include "stencil_pipe.h"

namespace rma {
namespace pipe {

bool dispatch_a(int K, int S, int V, int ar, const PipeLaunch& a) {
  RMA_PIPE_CASE(1, 1, kArCanon)
  RMA_PIPE_CASE(2, 1, kArCanon)
  RMA_PIPE_CASE(3, 1, kArCanon)
  RMA_PIPE_CASE(4, 1, kArCanon)
  RMA_PIPE_CASE(5, 2, kArCanon)
  RMA_PIPE_CASE(6, 2, kArCanon)
  RMA_PIPE_CASE(7, 2, kArCanon)
  RMA_PIPE_CASE(8, 2, kArCanon)
  RMA_PIPE_CASE(9, 2, kArCanon)
  RMA_PIPE_CASE(10, 4, kArCanon)
  RMA_PIPE_CASE(11, 4, kArCanon)
  RMA_PIPE_CASE(12, 4, kArCanon)
  RMA_PIPE_CASE(13, 4, kArCanon)
  RMA_PIPE_CASE(14, 4, kArCanon)
  RMA_PIPE_CASE(15, 4, kArCanon)
  RMA_PIPE_CASE(16, 4, kArCanon)
  RMA_PIPE_CASE(17, 4, kArCanon)
  RMA_PIPE_CASE(18, 4, kArCanon)
  RMA_PIPE_CASE(19, 4, kArCanon)
  RMA_PIPE_CASE(20, 4, kArCanon)
  RMA_PIPE_CASE(21, 4, kArCanon)
  RMA_PIPE_CASE(22, 4, kArCanon)
  RMA_PIPE_CASE(23, 4, kArCanon)
  RMA_PIPE_CASE(24, 4, kArCanon)
  return false;
}

}  // namespace pipe
}  // namespace rma
