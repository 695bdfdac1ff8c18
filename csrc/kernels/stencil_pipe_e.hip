// Instantiations of the any-K pipelined kernel (stencil_pipe.h), unit e:
// fast5 arithmetic with two column waves per stage (C = 2, V = 4): 8-wave
// blocks of ~500 input columns whose inner stage boundary recomputes 2*Hp
// columns instead of a second strip's 2K. An experiment, not the default:
// 8 % less arithmetic at K=24 but one block per CU (152 KB LDS), whose per-row
// barrier no second block hides: 85.2 vs 80.9 ms per K=24 pass at 101376^2,
// 65.7 vs 55.4 ms at K=16 (profiles/pass_sweep_cols2_r2.json).
#include "stencil_pipe.h"

namespace rma {
namespace pipe {

#define RMA_PIPE2_CASE(KK, SS, CC)          \
  if (K == KK && S == SS && ar == CC) {     \
    if (V != 4) return false;               \
    launch<KK, SS, 4, CC, 2>(a);            \
    return true;                            \
  }

bool dispatch_e(int K, int S, int V, int ar, const PipeLaunch& a) {
  RMA_PIPE2_CASE(16, 4, kArFast5)
  RMA_PIPE2_CASE(20, 4, kArFast5)
  RMA_PIPE2_CASE(24, 4, kArFast5)
  return false;
}

}  // namespace pipe
}  // namespace rma
