// Instantiations of the any-K pipelined kernel (stencil_pipe.h), unit d:
// fast5 arithmetic, alternative stage splits for sweeps. Split over several units so the build compiles them in parallel.
#include "stencil_pipe.h"

namespace rma {
namespace pipe {

bool dispatch_d(int K, int S, int V, bool canon, const PipeLaunch& a) {
  RMA_PIPE_CASE(12, 3, false)
  RMA_PIPE_CASE(16, 8, false)
  RMA_PIPE_CASE(24, 8, false)
  RMA_PIPE_CASE(8, 4, false)
  RMA_PIPE_CASE(8, 1, false)
  return false;
}

}  // namespace pipe
}  // namespace rma
