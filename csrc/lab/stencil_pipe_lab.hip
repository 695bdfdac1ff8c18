// librma_lab.so, pipelined unit: members of the any-K pipelined family
// (stencil_pipe.h) that the executor never runs, kept for sweeps:
//   * alternative stage splits (K=12 S=3, K=16/24 S=8, K=8 S=4/1), fast5;
//   * kernel 11 "pipeb": fast5 with the lane moves by ds_bpermute on the LDS
//     pipe instead of DPP (an energy / issue experiment, K = 16, 20, 24);
//   * two column waves per stage (C = 2, V = 4, fast5 K = 16, 20, 24): 8-wave
//     blocks of ~500 input columns whose inner stage boundary recomputes 2*Hp
//     columns instead of a second strip's 2K. 8 % less arithmetic at K=24 but
//     one block per CU (152 KB LDS), whose per-row barrier no second block
//     hides: 85.2 vs 80.9 ms per K=24 pass at 101376^2, 65.7 vs 55.4 ms at
//     K=16 (profiles/pass_sweep_cols2_r2.json); the same with piper's register
//     factors (K = 16, 20, 24; piper_rot at 20, 24), round 6: VALU -5.9 % but
//     +34-38 % wait cycles, 70.8 vs 67.2 ms at K=20 (profiles/r6/cols2_piper.md);
//   * 5 cells per lane (fast5, K = 16..20, stencil_pipe5_lab.hip);
//   * a diagnosis variant with one factor-ring read per stage and row (wrong
//     results; what the ring reads cost: -5 % per K=24 pass, SUMMARY_r3);
//   * piper6 / piper7: register factors with the split 6-operation form for
//     anisotropic grids (one full-mantissa constant multiplier instead of
//     two; kernels 14 / 15, bitwise equal to each other and to
//     stencil6_rects_cpu), K = 20, 24;
//   * piper_u3 (kernel 16): piper with the row loop unrolled by 3 in every
//     stage (the round-3 kernel; the core's K = 17..20 unroll by 6), A/B;
//   * piper_iso (kernel 17): piper with fma(1, U+D, t) as an add, for
//     ry == 1 exactly (bitwise equal to piper there), K = 20, 24;
//   * piper_mask (kernel 20): piper whose lanes outside a level's valid cone
//     skip the level under EXEC (bitwise equal to piper), K = 20, 24.
#include "../kernels/lab_hooks.h"

namespace rma {
namespace pipe {
namespace {

bool dispatch_alt(int K, int S, int V, int ar, const PipeLaunch& a) {
  RMA_PIPE_CASE(12, 3, kArFast5)
  RMA_PIPE_CASE(16, 8, kArFast5)
  RMA_PIPE_CASE(24, 8, kArFast5)
  RMA_PIPE_CASE(8, 4, kArFast5)
  RMA_PIPE_CASE(8, 1, kArFast5)
  RMA_PIPE_CASE(16, 4, kArFast5Perm)
  RMA_PIPE_CASE(20, 4, kArFast5Perm)
  RMA_PIPE_CASE(24, 4, kArFast5Perm)
  RMA_PIPE_CASE(20, 4, kArDiagOneRow)
  RMA_PIPE_CASE(24, 4, kArDiagOneRow)
  RMA_PIPE_CASE(20, 4, kArFast6Reg)
  RMA_PIPE_CASE(24, 4, kArFast6Reg)
  RMA_PIPE_CASE(20, 4, kArFast7Reg)
  RMA_PIPE_CASE(24, 4, kArFast7Reg)
  RMA_PIPE_CASE(17, 4, kArFast5RegU3)
  RMA_PIPE_CASE(18, 4, kArFast5RegU3)
  RMA_PIPE_CASE(19, 4, kArFast5RegU3)
  RMA_PIPE_CASE(20, 4, kArFast5RegU3)
  RMA_PIPE_CASE(20, 4, kArFast5RegIso)
  RMA_PIPE_CASE(24, 4, kArFast5RegIso)
  RMA_PIPE_CASE(20, 4, kArDiagS0)
  RMA_PIPE_CASE(20, 4, kArFast5RegW1)
  RMA_PIPE_CASE(24, 4, kArFast5RegW1)
  RMA_PIPE_CASE(20, 4, kArFast5RegMask)
  RMA_PIPE_CASE(24, 4, kArFast5RegMask)
  RMA_PIPE_CASE(20, 4, kArFast5RegMaskCtl)
  RMA_PIPE_CASE(24, 4, kArFast5RegMaskCtl)
  RMA_PIPE_CASE(20, 4, kArFast5RegNoSB)
  RMA_PIPE_CASE(24, 4, kArFast5RegNoSB)
  RMA_PIPE_CASE(20, 4, kArFast5RegRot)
  RMA_PIPE_CASE(24, 4, kArFast5RegRot)
  RMA_PIPE_CASE(20, 4, kArDiagHalfBarrier)
  RMA_PIPE_CASE(21, 4, kArFast5RegU6S)
  RMA_PIPE_CASE(24, 4, kArFast5RegU6S)
  RMA_PIPE_CASE(20, 4, kArFast5RegSP)
  RMA_PIPE_CASE(24, 4, kArFast5RegSP)
  RMA_PIPE_CASE(20, 4, kArFast5RegSP2)
  RMA_PIPE_CASE(24, 4, kArFast5RegSP2)
  RMA_PIPE_CASE(20, 4, kArFast5RegPrio)
  RMA_PIPE_CASE(24, 4, kArFast5RegPrio)
  RMA_PIPE_CASE(20, 4, kArFast5RegPrioNR)
  RMA_PIPE_CASE(24, 4, kArFast5RegPrioNR)
  return false;
}


#define RMA_PIPE2_CASE(KK, SS, CC)          \
  if (K == KK && S == SS && ar == CC) {     \
    if (V != 4) return false;               \
    launch<KK, SS, 4, CC, 2>(a);            \
    return true;                            \
  }

bool dispatch_cols2(int K, int S, int V, int ar, const PipeLaunch& a) {
  RMA_PIPE2_CASE(16, 4, kArFast5)
  RMA_PIPE2_CASE(20, 4, kArFast5)
  RMA_PIPE2_CASE(24, 4, kArFast5)
  RMA_PIPE2_CASE(16, 4, kArFast5Reg)
  RMA_PIPE2_CASE(20, 4, kArFast5Reg)
  RMA_PIPE2_CASE(24, 4, kArFast5Reg)
  RMA_PIPE2_CASE(20, 4, kArFast5RegRot)
  RMA_PIPE2_CASE(24, 4, kArFast5RegRot)
  return false;
}

}  // namespace

bool dispatch_v5(int K, int S, int V, int ar, const PipeLaunch& a);  // stencil_pipe5_lab.hip

}  // namespace pipe

namespace lab {
bool pipe(int K, int S, int V, int C, int arith, const pipe::PipeLaunch& a) {
  if (C == 2) return pipe::dispatch_cols2(K, S, V, arith, a);
  return V == 5 ? pipe::dispatch_v5(K, S, V, arith, a) : pipe::dispatch_alt(K, S, V, arith, a);
}
}  // namespace lab
}  // namespace rma
