// Host-side kernel-selection rules of the stencil launchers: which
// pipelined (K, stages, arithmetic, cols) instantiations exist, the cells per
// lane a launch runs, the one-step march kernel's strip width. Plain host code
// (moved out of stencil_pipe.hip / stencil.hip) so the executor's planning
// compiles and runs without HIP, e.g. in tests/native/executor_selftest.cpp
// under ThreadSanitizer / AddressSanitizer.
#include <cstdint>

#include "pipe_arith.h"
#include "rma/kernels.h"

namespace rma {

int pipe_default_stages(int K) {
  // Waves per strip: 1, 2 or 4 only. A block of 3, 5 or 6 waves puts two of
  // its stages on one SIMD (waves are dealt round-robin over the 4 SIMDs of a
  // CU) and the per-row barrier then runs the whole block at that SIMD's pace:
  // K=17..20 with 5 stages took 103-118 ms per pass at 101376^2 against 76 ms
  // for K=20 on 4 stages of 5 levels (profiles/pass_sweep_r2.json). Deeper
  // stages amortise the per-row barrier and hand-off: K=24 on 4 stages of 6
  // levels (2 waves per SIMD) has the lowest time per step of all depths.
  if (K <= 4) return 1;
  if (K <= 9) return 2;  // K=9 on 4 stages would leave the last one empty
  return 4;
}

bool pipe_has(int K, int S, int arith) {
  if (K < 1 || K > kPipeMaxK) return false;
  if (arith == pipe::kArFast5Perm) return S == 4 && (K == 16 || K == 20 || K == 24);
  if (arith == pipe::kArFast5Reg) return S == 4 && K >= 10 && K <= 24;
  if (arith == pipe::kArDiagOneRow) return S == 4 && (K == 20 || K == 24);
  if (pipe::ar_split(arith)) return S == 4 && (K == 20 || K == 24);
  if (arith == pipe::kArFast5RegU3) return S == 4 && K >= 17 && K <= 20;
  if (arith == pipe::kArFast5RegIso) return S == 4 && (K == 20 || K == 24);
  if (arith == pipe::kArDiagS0) return S == 4 && K == 20;
  if (arith == pipe::kArFast5RegW1) return S == 4 && (K == 20 || K == 24);
  if (arith == pipe::kArFast5RegMask || arith == pipe::kArFast5RegMaskCtl ||
      arith == pipe::kArFast5RegNoSB || arith == pipe::kArFast5RegRot)
    return S == 4 && (K == 20 || K == 24);
  if (arith == pipe::kArDiagHalfBarrier) return S == 4 && K == 20;
  if (arith == pipe::kArFast5RegU6S) return S == 4 && (K == 21 || K == 24);
  if (arith == pipe::kArFast5RegSP || arith == pipe::kArFast5RegSP2 ||
      arith == pipe::kArFast5RegPrio || arith == pipe::kArFast5RegPrioNR)
    return S == 4 && (K == 20 || K == 24);
  if (S == pipe_default_stages(K)) return true;
  // alternative stage splits instantiated for sweeps (csrc/lab/stencil_pipe_lab.hip)
  return (K == 12 && S == 3) || (K == 16 && S == 8) || (K == 24 && S == 8) ||
         (K == 8 && S == 4) || (K == 8 && S == 1);
}

bool pipe_has_cols(int K, int S, int arith, int cols) {
  if (cols <= 1) return pipe_has(K, S, arith);
  if (cols != 2 || S != 4) return false;
  if (arith == pipe::kArFast5 || arith == pipe::kArFast5Reg) return K == 16 || K == 20 || K == 24;
  return arith == pipe::kArFast5RegRot && (K == 20 || K == 24);
}

int pipe_default_cols(int K, int S, int arith) {
  // one column wave: the 2-column blocks (csrc/lab/stencil_pipe_lab.hip) do 6-8 % less
  // arithmetic but run one 8-wave block per CU and lose more to the unhidden
  // per-row barrier: ring kernel 5-20 % (profiles/pass_sweep_cols2_r2.json), piper
  // +5.3 % at K=20 and +11.9 % at K=24 with the rotated map, +34-38 % wait cycles
  // (profiles/r6/cols2_piper.md)
  (void)K;
  (void)S;
  (void)arith;
  return 1;
}

int pipe_vec(int K, int stages, int arith, int64_t nx, int requested, bool aligned16) {
  const int S = stages > 0 ? stages : pipe_default_stages(K);
  if (requested == 5 && nx % 5 == 0 && pipe::pipe_has_v5(K, S, arith)) return 5;
  if (aligned16 && nx % 2 == 0) return (requested >= 4 && nx % 4 == 0) ? 4 : 2;
  return 1;
}

int stencil_vec(int64_t nx, const StencilTuning& tune) {
  // cells per lane: 16-byte rows need an even nx; V=4 also needs nx % 4 == 0
  // (a clamped lane past the row end must still load its own cells)
  if (nx % 2) return 1;
  if (tune.vec == 4 && nx % 4 == 0) return 4;
  return 2;
}

int stencil_strip_cells(int64_t nx, const StencilTuning& tune) {
  constexpr int kWave = 64;
  return kWave * stencil_vec(nx, tune);
}

}  // namespace rma
