// Instantiations of the any-K pipelined kernel (stencil_pipe.h), unit b:
// fast5 arithmetic, K = 1..12 (default stage split). Split over several units so the build compiles them in parallel.
#include "stencil_pipe.h"

namespace rma {
namespace pipe {

bool dispatch_b(int K, int S, int V, int ar, const PipeLaunch& a) {
  RMA_PIPE_CASE(1, 1, kArFast5)
  RMA_PIPE_CASE(2, 1, kArFast5)
  RMA_PIPE_CASE(3, 1, kArFast5)
  RMA_PIPE_CASE(4, 1, kArFast5)
  RMA_PIPE_CASE(5, 2, kArFast5)
  RMA_PIPE_CASE(6, 2, kArFast5)
  RMA_PIPE_CASE(7, 2, kArFast5)
  RMA_PIPE_CASE(8, 2, kArFast5)
  RMA_PIPE_CASE(9, 2, kArFast5)
  RMA_PIPE_CASE(10, 4, kArFast5)
  RMA_PIPE_CASE(11, 4, kArFast5)
  RMA_PIPE_CASE(12, 4, kArFast5)
  return false;
}

}  // namespace pipe
}  // namespace rma
