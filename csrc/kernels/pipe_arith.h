// Arithmetic variants of the stage-pipelined K-step kernel (stencil_pipe.h
// template parameter Ar) and the host-side predicates over them. Host-safe (no
// HIP): the kernel-selection rules (kernel_select.cpp) compile with any host
// compiler, e.g. the sanitizer builds of tests/native.
#pragma once

namespace rma {
namespace pipe {

constexpr int kArFast5 = 0, kArCanon = 1, kArFast5Perm = 2, kArFast5Reg = 3;
// diagnosis only (lab, WRONG results): every level of a stage uses the factor
// row of its level 1, i.e. one LDS ring row read per stage and iteration
// instead of H; measures what the ring reads cost (energy / time)
constexpr int kArDiagOneRow = 4;
// register factors with the split form for anisotropic grids (dx != dy):
//   T2 = fma(g, fma(ry, fma(-2, c, U+D), fma(-2, c, L+R)), c)
// one full-mantissa constant multiplier (ry) instead of two (ry, -2(1+ry)):
// the deep passes are power-capped and the multiplier toggling of the
// constants costs ~2 % (profiles/SUMMARY_r3.md section 1). kArFast7Reg is
// the same form with the -2c done as (c + c) and two subtractions (2c is
// exact, so both round once: bitwise equal). A different rounding than the
// 5-operation form; CPU twin stencil6_rects_cpu.
constexpr int kArFast6Reg = 5, kArFast7Reg = 6;
// lab A/B: kArFast5Reg with the row loop unrolled by 3 in every stage (the
// round-3 piper; see kU6 below), bitwise equal to piper
constexpr int kArFast5RegU3 = 7;
// isotropic grids (ry = (dx/dy)^2 == 1 exactly, e.g. N = 1, the 2x2 grid):
// fma(ry, U+D, t) as the add (U+D) + t -- bitwise the same (1 * x is exact,
// one rounding either way), one fp64 multiplier use fewer per update; the
// host selects it only when ry == 1 (kernel 17 "piper_iso")
constexpr int kArFast5RegIso = 8;
// diagnosis only (lab, WRONG results): piper whose stage 0 runs H-1 levels
// (stage 0 also streams T / 1/Cp and forms the factors: is it the block's
// critical path at the per-row barrier?)
constexpr int kArDiagS0 = 9;
// lab: piper at ONE wave per SIMD (one 4-wave block per CU, up to 512
// registers incl. AGPRs) with the row loop unrolled by 6 also at H = 6 (K =
// 21..24, which spill 39 VGPRs at 2 waves per SIMD): no factor-row moves
// against no second block to hide the per-row barrier
constexpr int kArFast5RegW1 = 10;
// lab: piper with the lanes outside the level's valid cone masked off. Level l
// of a strip window is valid on columns [l, W - l) only (each level loses one
// column per side); a lane whose V cells all lie outside skips that level's
// arithmetic under EXEC (its registers keep stale values no valid output reads).
// ~7 % of the lane-updates of a K=20 pass: does an EXEC-masked lane save the
// power-capped pass its energy? Bitwise equal to piper.
constexpr int kArFast5RegMask = 11;
// its control: the same asm statement under the full EXEC (the schedule's cost alone)
constexpr int kArFast5RegMaskCtl = 12;
// lab: piper without the sched_barriers between the phases of a level's
// arithmetic (the scheduler free to overlap levels), A/B of the schedule
constexpr int kArFast5RegNoSB = 13;
// lab: piper with the stage -> wave map rotated by 2 in odd blocks (waves are
// dealt to SIMDs in order, so two co-resident blocks of the same parity put
// both stage-0 waves, the heaviest, on one SIMD): A/B of the SIMD balance
constexpr int kArFast5RegRot = 14;
// diagnosis only (lab, WRONG results: the hand-off rows race): piper with the
// row barrier on every other row only -- the most that fewer barriers could buy
constexpr int kArDiagHalfBarrier = 15;
// lab: piper unrolled by 6 also at H = 6 (K = 21..24), accepting the spills
// (~10-17 scratch accesses per 6 rows and stage instead of ~44-64 row moves)
constexpr int kArFast5RegU6S = 16;
// lab: piper with the levels software-pipelined: level j+1's lane moves, L+R
// and fma(mkc, c, L+R) (which read only the previous row iteration's values)
// are issued while level j's chain U+D -> fma(ry) -> fma(g) runs, so the chain
// after a new row lands is 3 dependent operations instead of 5 plus the lane
// moves. Same operations and rounding as piper (bitwise). kArFast5RegSP: one
// sched_barrier per level; kArFast5RegSP2: none.
constexpr int kArFast5RegSP = 17, kArFast5RegSP2 = 18;
// lab: wave priority for the heaviest stage. Stage 0 (HBM stream, factor
// formation, ~7 % more VALU and ~15x the SALU of a middle stage; ISA budget
// profiles/r5/isa_budget.md) paces its block at every row barrier.
// kArFast5RegPrio: the rotated stage map of kArFast5RegRot (odd blocks' stage
// 0 on SIMD 2, so each SIMD hosts at most one stage-0 wave) plus s_setprio 2
// on stage-0 waves, so the SIMD issues for them first; kArFast5RegPrioNR: the
// priority without the rotation (both stage-0 waves share SIMD 0: control).
constexpr int kArFast5RegPrio = 19, kArFast5RegPrioNR = 20;
constexpr bool ar_reg(int Ar) {
  return Ar == kArFast5Reg || Ar == kArFast6Reg || Ar == kArFast7Reg || Ar == kArFast5RegU3 ||
         Ar == kArFast5RegIso || Ar == kArDiagS0 || Ar == kArFast5RegW1 || Ar == kArFast5RegMask ||
         Ar == kArFast5RegMaskCtl || Ar == kArFast5RegNoSB || Ar == kArFast5RegRot ||
         Ar == kArDiagHalfBarrier || Ar == kArFast5RegU6S || Ar == kArFast5RegSP ||
         Ar == kArFast5RegSP2 || Ar == kArFast5RegPrio || Ar == kArFast5RegPrioNR;
}
constexpr bool ar_split(int Ar) { return Ar == kArFast6Reg || Ar == kArFast7Reg; }

// 5 cells per lane: fast5, S = 4, K = 16..20, in the lab library
// (csrc/lab/stencil_pipe5_lab.hip)
inline bool pipe_has_v5(int K, int S, int ar) {
  return ar == kArFast5 && S == 4 && K >= 16 && K <= 20;
}

}  // namespace pipe
}  // namespace rma
