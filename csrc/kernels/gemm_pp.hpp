// Ping-pong 8-wave MFMA main loop (gfx950): the 256x256-class tiles of the GEMM / convolution
// kernels.
//
// Why a second main loop: the 2-phase loop of gemm_core.hpp (one barrier per 64-deep k-step,
// every fragment read up front) is latency-bound at one workgroup per CU — its 256x256 tile tops
// out at ~1.1 PF on 4096^3 (profiles/r2_gemm_lab_tiles_schedules.jsonl) because every wave waits
// for its own LDS reads, and the glds stage, before its MFMAs.  This loop follows the CDNA4
// two-waves-per-SIMD structure (MI355X_MICROARCH.md "Two waves per SIMD"; cdna_hip_programming.md
// §5 "256^2 8-phase template"):
//
//  * 512 threads = 8 waves, WM x WN = 2 x 4.  Waves 0-3 ("group 0") and 4-7 ("group 1") sit one
//    per SIMD each, so every SIMD holds one wave of each group.
//  * A k-step (BK = 64) is cut into 4 PHASES, one output quadrant each (the wave tile is
//    (BM/WM) x (BN/WN); quadrant (h, g) = the wave's m-half h x n-half g: QM x QN 16x16 MFMA tiles
//    x 2 k-substeps = 16 MFMAs at 256x256).  A phase = {LDS fragment reads; one half-tile of
//    LDS-DMA; counted vmcnt} BARRIER {MFMAs} BARRIER.
//  * Group 1 runs one barrier behind group 0 (one extra s_barrier before the loop), so between
//    any two barriers one group issues MFMAs while the other issues its LDS reads and DMAs: the
//    matrix pipe of every SIMD is fed by alternating waves and the reads never sit in front of
//    the wave's own MFMAs.
//  * Operands are staged in HALF tiles: A-half h = tile rows [h*BM/2, +BM/2), B-half g = tile
//    columns [g*BN/2, +BN/2) — each one a standard operand-policy tile of R = BM/2 (BN/2) rows
//    loaded by 8 waves, so every gemm_core.hpp policy (dense, im2col, dgrad gathers, MC
//    transposed images) plugs in unchanged.  The wave's rows are therefore NOT contiguous: its
//    quadrant h rows are h*BM/2 + wr*(BM/2/WM) + [0, BM/2/WM) (see row()/col() below; the
//    epilogues take this map as a template argument).
//  * Fragment reuse: quadrants run in the order (0,0) (0,1) (1,1) (1,0), so a k-step reads
//    A-half 0 + B-half 0 (phase 0), B-half 1 (phase 1), A-half 1 (phase 2) and nothing in phase 3.
//  * Half-tile DMA schedule (2 LDS stages, stage = tile & 1), phase q of tile t issues:
//      q0: B-half 1 of t+1   q1: A-half 1 of t+1   q2: A-half 0 of t+2   q3: B-half 0 of t+2
//    Every half is overwritten >= 2 phases after its last read (the WAR distance the staggered
//    barriers need) and is needed >= 5 phases after it is issued; the wait at phase x retires
//    everything issued at phases <= x-4 (vmcnt = DMAs of the halves issued in x-3..x), i.e. the
//    data a phase reads was waited for one phase earlier, before a barrier the reader passes.
//    The prologue is the same schedule run for phases -6..-1.
#pragma once
#include "gemm_core.hpp"

namespace mipipe {
namespace gk {

constexpr int kPPPrio = 1;     // s_setprio(1) around each MFMA cluster
constexpr int kPPStagger = 2;  // group 1 one barrier behind (ping-pong); off = lockstep
constexpr int kPPDefault = kPPPrio | kPPStagger;

// s_waitcnt vmcnt(n) for a wave-uniform runtime n in [0, MAX] (scalar branches to immediates)
template <int MAX>
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
  if constexpr (MAX <= 0) {
    wait_vmcnt<0>();
  } else {
    if (n >= MAX) wait_vmcnt<MAX>();
    else wait_vmcnt_rt<MAX - 1>(n);
  }
}

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int BM, int BN, class OpA, class OpB, int WM = 2, int WN = 4, int V = kPPDefault>
struct MainLoopPP {
  static constexpr int NW = WM * WN;
  static_assert(NW == 8, "ping-pong: 8 waves, two per SIMD");
  static constexpr int HM = BM / 2, HN = BN / 2;
  static constexpr int QM = HM / WM / 16;  // 16-row tiles per wave per quadrant
  static constexpr int QN = HN / WN / 16;
  static constexpr int MT = 2 * QM, NT = 2 * QN;
  static constexpr int HA = HM * BK * 2;  // bytes of one A half-tile image
  static constexpr int HB = HN * BK * 2;
  static constexpr int OFF_A0 = 0, OFF_A1 = HA, OFF_B0 = 2 * HA, OFF_B1 = 2 * HA + HB;
  static constexpr int STAGE_BYTES = 2 * (HA + HB);
  static constexpr int LDS_BYTES = 2 * STAGE_BYTES;
  static constexpr int NIA = OpA::NI;  // LDS-DMA instructions per wave per A / B half tile
  static constexpr int NIB = OpB::NI;
  static constexpr int FULL_INFLIGHT = 2 * (NIA + NIB);  // 4 phases: 2 A halves + 2 B halves
  static constexpr bool PRIO = (V & kPPPrio) != 0;
  static constexpr bool STAGGER = (V & kPPStagger) != 0;
  static_assert(OpA::NI * 8 * NW == HM || !OpA::KC, "A half policy: R = BM/2 rows, 8 waves");
  static_assert(OpB::NI * 8 * NW == HN || !OpB::KC, "B half policy: R = BN/2 rows, 8 waves");
  static_assert(QM >= 1 && QN >= 1, "tile too small for the wave grid");
  static_assert(!HasXform<OpA>::value && !HasXform<OpB>::value, "folded BN: 4-wave loops only");

  // tile-local row / column of accumulator (i, j) of wave (wr, wc), before the lane offset
  __device__ static uint32_t row(int wr, int i) {
    return (uint32_t)((i / QM) * HM + wr * (QM * 16) + (i % QM) * 16);
  }
  __device__ static uint32_t col(int wc, int j) {
    return (uint32_t)((j / QN) * HN + wc * (QN * 16) + (j % QN) * 16);
  }

  template <class Op>
  __device__ static void half(Op& op, char* dst, int kt, int wave) {
    op.prep(kt);
    if (is_tail(op, kt)) {  // wave-uniform: the last k-step of a K % 64 != 0 operand only
#pragma unroll
      for (int j = 0; j < Op::NI; ++j) dma16<true>(op, kt, j, dst + (wave * Op::NI + j) * 1024);
      tail_block_end();
    } else {
#pragma unroll
      for (int j = 0; j < Op::NI; ++j) dma16<false>(op, kt, j, dst + (wave * Op::NI + j) * 1024);
    }
  }

  // DMA of global phase x (x >= -6; compile-time phase-in-tile Q = x & 3)
  template <int Q>
  __device__ static void issue(char* smem, OpA (&a)[2], OpB (&b)[2], int kt0, int nk, int t,
                               int wave) {
    const int tt = t + 1 + (Q >> 1);  // tile of the half issued in this phase
    if (tt >= nk) return;
    char* st = smem + (tt & 1) * STAGE_BYTES;
    if constexpr (Q == 0) half(b[1], st + OFF_B1, kt0 + tt, wave);
    else if constexpr (Q == 1) half(a[1], st + OFF_A1, kt0 + tt, wave);
    else if constexpr (Q == 2) half(a[0], st + OFF_A0, kt0 + tt, wave);
    else half(b[0], st + OFF_B0, kt0 + tt, wave);
  }

  // DMA instructions in flight that the wait at phase x may leave: those of the halves issued in
  // phases x-3..x (phase q issues a B half for q = 0, 3 and an A half for q = 1, 2)
  __device__ static int inflight(int x, int nk) {
    const int last = 4 * nk - 7;  // phase of the final DMA (A-half 1 of the last tile)
    int n = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int y = x - d;
      const int q = (y + 8) & 3;
      if (y <= last) n += (q == 1 || q == 2) ? NIA : NIB;
    }
    return n;
  }

  template <int Q>
  __device__ static void mfma_quadrant(f32x4 (&acc)[MT][NT], const bf16x8 (&af)[2][QM],
                                       const bf16x8 (&bf)[2][QN]) {
    constexpr int H = (Q == 0 || Q == 1) ? 0 : 1;  // m-half
    constexpr int G = (Q == 0 || Q == 3) ? 0 : 1;  // n-half
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < QM; ++i)
#pragma unroll
        for (int j = 0; j < QN; ++j)
          acc[H * QM + i][G * QN + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              bf[ks][j], af[ks][i], acc[H * QM + i][G * QN + j], 0, 0, 0);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  }

  __device__ static void read_a(bf16x8 (&af)[2][QM], const char* img, uint32_t arow, int lane) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < QM; ++i)
        af[ks][i] = FragLoader<OpA::KC, HM>::load(img, arow + i * 16, ks, lane);
  }
  __device__ static void read_b(bf16x8 (&bf)[2][QN], const char* img, uint32_t bcol, int lane) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < QN; ++j)
        bf[ks][j] = FragLoader<OpB::KC, HN>::load(img, bcol + j * 16, ks, lane);
  }

  template <bool FULL, int Q>
  __device__ static void phase_dma(char* smem, OpA (&a)[2], OpB (&b)[2], int kt0, int nk, int t,
                                   int wave) {
    if constexpr (FULL) {
      char* st = smem + ((t + 1 + (Q >> 1)) & 1) * STAGE_BYTES;
      const int kt = kt0 + t + 1 + (Q >> 1);
      if constexpr (Q == 0) half(b[1], st + OFF_B1, kt, wave);
      else if constexpr (Q == 1) half(a[1], st + OFF_A1, kt, wave);
      else if constexpr (Q == 2) half(a[0], st + OFF_A0, kt, wave);
      else half(b[0], st + OFF_B0, kt, wave);
      wait_vmcnt<FULL_INFLIGHT>();
    } else {
      issue<Q>(smem, a, b, kt0, nk, t, wave);
      wait_vmcnt_rt<FULL_INFLIGHT>(inflight(4 * t + Q, nk));
    }
  }

  template <bool FULL>
  __device__ static void tile_body(char* smem, OpA (&a)[2], OpB (&b)[2], int kt0, int nk, int t,
                                   f32x4 (&acc)[MT][NT], bf16x8 (&af)[2][QM],
                                   bf16x8 (&bf0)[2][QN], bf16x8 (&bf1)[2][QN], uint32_t arow,
                                   uint32_t bcol, int wave, int lane) {
    const char* st = smem + (t & 1) * STAGE_BYTES;
    // phase 0: quadrant (0,0)
    read_a(af, st + OFF_A0, arow, lane);
    read_b(bf0, st + OFF_B0, bcol, lane);
    phase_dma<FULL, 0>(smem, a, b, kt0, nk, t, wave);
    pp_barrier();
    mfma_quadrant<0>(acc, af, bf0);
    pp_barrier();
    // phase 1: quadrant (0,1)
    read_b(bf1, st + OFF_B1, bcol, lane);
    phase_dma<FULL, 1>(smem, a, b, kt0, nk, t, wave);
    pp_barrier();
    mfma_quadrant<1>(acc, af, bf1);
    pp_barrier();
    // phase 2: quadrant (1,1)
    read_a(af, st + OFF_A1, arow, lane);
    phase_dma<FULL, 2>(smem, a, b, kt0, nk, t, wave);
    pp_barrier();
    mfma_quadrant<2>(acc, af, bf1);
    pp_barrier();
    // phase 3: quadrant (1,0)
    phase_dma<FULL, 3>(smem, a, b, kt0, nk, t, wave);
    pp_barrier();
    mfma_quadrant<3>(acc, af, bf0);
    pp_barrier();
  }

  // a[h] / b[g]: the half-tile policies, initialised with origins m0 + h*HM / n0 + g*HN
  __device__ static void run(char* smem, OpA (&a)[2], OpB (&b)[2], int kt0, int kt1,
                             f32x4 (&acc)[MT][NT], int wave, int lane) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = kt1 - kt0;
    if (nk <= 0) return;
    const int wr = wave / WN, wc = wave % WN;
    const uint32_t arow = wr * (QM * 16), bcol = wc * (QN * 16);
    const bool late = STAGGER && wave >= NW / 2;  // wave-uniform (wave is readfirstlane'd)
    // prologue: the steady-state DMA schedule for phases -6..-1
    issue<2>(smem, a, b, kt0, nk, -2, wave);
    issue<3>(smem, a, b, kt0, nk, -2, wave);
    issue<0>(smem, a, b, kt0, nk, -1, wave);
    issue<1>(smem, a, b, kt0, nk, -1, wave);
    issue<2>(smem, a, b, kt0, nk, -1, wave);
    issue<3>(smem, a, b, kt0, nk, -1, wave);
    wait_vmcnt_rt<FULL_INFLIGHT>(inflight(-1, nk));
    pp_barrier();
    if (late) pp_barrier();
    bf16x8 af[2][QM], bf0[2][QN], bf1[2][QN];
    int t = 0;
    // steady state: every phase issues its half tile and waits with the full in-flight count
    for (; t + 2 < nk; ++t) tile_body<true>(smem, a, b, kt0, nk, t, acc, af, bf0, bf1, arow, bcol, wave, lane);
    // the last two tiles: DMAs stop, the waits count down to 0
    for (; t < nk; ++t) tile_body<false>(smem, a, b, kt0, nk, t, acc, af, bf0, bf1, arow, bcol, wave, lane);
    if (STAGGER && !late) pp_barrier();
    // the epilogue reuses the stage buffers
    __syncthreads();
  }
};

}  // namespace gk
}  // namespace mipipe
