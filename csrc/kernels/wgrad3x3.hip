// 3x3 / stride-1 / pad-1 convolution weight-gradient with the input patch resident in LDS.
//
//   dW[co][kh][kw][ci] += sum_{n,ho,wo} dy[n][ho][wo][co] * x[n][ho+kh-1][wo+kw-1][ci]
//
// The generic weight-grad (conv_wgrad.hip) is an implicit GEMM whose B operand is im2col(x):
// every input element is fetched once per filter tap (9x through L2) and every block re-reads
// dy for each of its N tiles.  Here a k-step is a group of R consecutive output rows of ONE
// image (R*W <= 64 pixels, padded to 64 MFMA k-slots); the block stages
//   * the dy rows   [64 slots][64 co]                (8 KB, the A operand), and
//   * the x patch   [(R+2) rows][(W+2) cols][64 ci]  (<= 24 KB, zero halo)
// and all 9 taps read their B fragments from the SAME patch: tap (kh, kw) is the patch shifted
// by kh*(W+2) + kw pixels.  Both operands are k(pixel)-major, so fragments come from
// ds_read_b64_tr_b16 transposed reads (guide T10) whose per-lane row addresses make the tap
// shift free; the patch uses the MC chunk swizzle (row-parity / row-bit-3 XOR), which is
// bank-conflict-free for any tap shift of the {k..k+3, k+8..k+11} row sets one read touches.
//
// Block = 64 co x 64 ci x 9 taps (4 waves; wave w owns ci [16w, 16w+16) for all 64 co and 9 taps:
// 36 accumulators, A fragments shared by the 9 taps).  The reduction over pixels is split over
// S blocks per tile; each writes its fp32 partial tile to a workspace slice and a fixed-order
// sum adds the slices into dW (det.hip splitk_sum) — deterministic in both modes.
#include <cstdlib>
#include <utility>

#include "conv_common.hpp"

namespace mipipe {
namespace w3 {

using gk::BK;
using gk::glds16;
using gk::mc_off;
using gk::mc_swz;
using gk::wait_vmcnt;

constexpr int TM = 64;           // co per block
constexpr int TC = 64;           // ci per block
constexpr int kSlots = 64;       // MFMA k-slots (pixels) per k-step
constexpr int kDyBytes = kSlots * TM * 2;            // 8 KB
constexpr int kPatchPix = 192;                       // >= (R+2)*(W+2) for every supported shape
constexpr int kPatchBytes = kPatchPix * TC * 2;      // 24 KB
constexpr int kStage = kDyBytes + kPatchBytes;       // 32 KB
// 3 LDS stages, two k-steps of loads in flight (counted vmcnt): with the 36 accumulator tiles
// the kernel runs one wave per SIMD, so the prefetch depth, not other waves, hides HBM latency
constexpr int kStages = 3;

struct Geo {
  int N, H, W, Ci, Co;
  int R;        // output rows per k-step
  int G;        // k-step groups per image = ceil(H / R)
  int PW;       // patch width W + 2
  int steps;    // N * G
  int per;      // k-steps per split
  long ws_stride;  // floats per workspace slice (Co * 9 * Ci)
};

// patch pixel of MFMA slot k (tap (0,0)); slots beyond R*W reuse a row above (finite values,
// multiplied by the zero dy rows of those slots)
__device__ __forceinline__ int slot_pix(int k, int W, int RW, int PW) {
  const int kk = k < RW ? k : k - W * ((k - RW) / W + 1);
  const int r = kk / W;
  return r * PW + (kk - r * W);
}

// Transposed LDS read as inline asm: hipcc's waitcnt pass cannot tell these reads from the
// LDS-DMA writes into the OTHER stage buffers and drains vmcnt(0) before them (measured in the
// .s: 2 of 3 k-steps), which would serialise the 2-deep prefetch.  Ordering against the DMA is
// the counted vmcnt + barrier at the top of each k-step; ordering against the MFMAs is an
// explicit lgkmcnt wait + sched_barrier per unit (guide §5.4 rule 18).
__device__ __forceinline__ s16x4 tr_read(uint32_t lds_addr) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(lds_addr) : "memory");
  return v;
}
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  static_assert(N >= 0 && N <= 15, "lgkmcnt range");
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ bf16x8 join(s16x4 lo, s16x4 hi) {
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// The 18 (ks, tap) units of one k-step, software-pipelined LOOK units deep: both k halves' A
// fragments are requested first, then B(0..LOOK-1); unit u requests B(u+LOOK) and waits until
// only the reads issued after B(u) are outstanding (LDS returns in order), so its MFMAs overlap
// the next LOOK units' reads.  All counts are compile-time immediates (lgkmcnt <= 15).
template <int CB>
struct Frags {
  s16x4 a_lo[2][CB], a_hi[2][CB];
  s16x4 b_lo[18], b_hi[18];
};
template <int LOOK>
__device__ constexpr int unit_allowed(int u) {
  return 2 * ((u + LOOK < 18 ? u + LOOK : 17) - u);
}

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

template <int LOOK, int U, int CB, class FB>
__device__ __forceinline__ void unit(Frags<CB>& f, f32x4 (&acc)[9][CB], FB& issueB) {
  constexpr int ks = U / 9, t = U % 9;
  if constexpr (U + LOOK <= 17) issueB(U + LOOK);
  wait_lgkm<unit_allowed<LOOK>(U)>();
  const bf16x8 bf = join(f.b_lo[U], f.b_hi[U]);
#pragma unroll
  for (int i = 0; i < CB; ++i)
    acc[t][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf, join(f.a_lo[ks][i], f.a_hi[ks][i]),
                                                        acc[t][i], 0, 0, 0);
}
template <int LOOK, int CB, class FB, int... U>
__device__ __forceinline__ void units(Frags<CB>& f, f32x4 (&acc)[9][CB], FB& issueB,
                                      std::integer_sequence<int, U...>) {
  (unit<LOOK, U, CB>(f, acc, issueB), ...);
}

// NW = 4: wave w owns ci [16w, 16w+16) x all 64 co (4 co blocks, 36 accumulator tiles, one wave
//         per SIMD — the register file holds the tiles, the 3-stage prefetch hides latency);
// NW = 8: wave w owns ci [16(w&3), +16) x co [32(w>>2), +32) (2 co blocks, 18 tiles): two waves
//         per SIMD hide each other's LDS / barrier latency at 2x the A-fragment reads.
template <int NW>
__global__ __launch_bounds__(64 * NW, NW / 4) void wgrad3x3_kernel(
    const __bf16* __restrict__ dy, const __bf16* __restrict__ x, float* __restrict__ ws, Geo g,
    BnCollect col) {
  constexpr int CB = 16 / NW;                  // co blocks (16 co) per wave
  constexpr int DYI = 8 / NW;                  // dy-image glds per wave per stage
  constexpr int PTI = kPatchPix / (NW * 8);    // patch glds per wave per stage
  constexpr int LOADS = DYI + PTI;
  constexpr int LOOK = NW == 8 ? 6 : 5;
  static_assert(PTI * NW * 8 == kPatchPix && DYI * NW == 8, "staging split");
  // one __shared__ array per stage, indexed statically (the k-loop is unrolled by kStages): the
  // compiler can then prove that the LDS-DMA into stage s+2 does not alias the ds_reads of stage
  // s and keeps the counted vmcnt (one runtime-indexed array makes it wait vmcnt(0) before the
  // first ds_read of every k-step, draining the prefetch)
  __shared__ __attribute__((aligned(16))) char smem0[kStage];
  __shared__ __attribute__((aligned(16))) char smem1[kStage];
  __shared__ __attribute__((aligned(16))) char smem2[kStage];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (col.rep != nullptr && blockIdx.x == 0 && blockIdx.y == 0) gk::bn_collect_block<64 * NW>(col);
  const int tilesC = g.Ci / TC;
  const int tile = blockIdx.x;
  const int co0 = (tile / tilesC) * TM, ci0 = (tile % tilesC) * TC;
  const int s0 = blockIdx.y * g.per;
  const int s1 = min(g.steps, s0 + g.per);
  const int W = g.W, H = g.H, PW = g.PW, RW = g.R * g.W;
  const __bf16* zero = reinterpret_cast<const __bf16*>(gk::g_conv_zero);
  const int wci = wave & 3;                       // this wave's 16-ci quarter
  const int wco = NW == 8 ? (wave >> 2) * 32 : 0;  // this wave's first co

  // ---- staging: dy image MC [64 slots][64 co] (8 px per wave-instruction); x patch [pix][64 ci]
  // with the same chunk swizzle.  A lane's pixel per glds is loop-invariant, only the image /
  // row-group base moves, so the element offsets are precomputed (32-bit: the host checks
  // numel < 2^31) and each k-step adds one base and selects the zero page for halo /
  // out-of-image rows — a few VALU ops per glds instead of a division and a 64-bit multiply.
  int dy_rel[DYI], dy_slot[DYI];
#pragma unroll
  for (int i = 0; i < DYI; ++i) {
    dy_slot[i] = (wave * DYI + i) * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ (int)mc_swz<64>((uint32_t)dy_slot[i]);
    dy_rel[i] = dy_slot[i] * g.Co + co0 + ch * 8;
  }
  int pt_rel[PTI], pt_r[PTI];
  uint32_t wi_ok = 0;
#pragma unroll
  for (int i = 0; i < PTI; ++i) {
    const int p = (wave * PTI + i) * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ (int)mc_swz<64>((uint32_t)p);
    const int r = p / PW;
    const int wi = p - r * PW - 1;
    pt_r[i] = r;
    pt_rel[i] = (r * W + wi) * g.Ci + ci0 + ch * 8;
    wi_ok |= ((unsigned)wi < (unsigned)W ? 1u : 0u) << i;
  }
  auto stage = [&](char* buf, int step) {
    const int n = step / g.G, grp = step - n * g.G;
    const int ho0 = grp * g.R;
    const int rows = min(g.R, H - ho0);
    const int P = rows * W;
    const int dy0 = (n * H + ho0) * W * g.Co;
#pragma unroll
    for (int i = 0; i < DYI; ++i) {
      const void* src = dy_slot[i] < P ? (const void*)(dy + dy0 + dy_rel[i]) : (const void*)zero;
      glds16(src, buf + (wave * DYI + i) * 1024);
    }
    char* pb = buf + kDyBytes;
    const int x0 = (n * H + ho0 - 1) * W * g.Ci;  // patch row 0 = image row ho0 - 1
    const int rlo = ho0 == 0 ? 1 : 0;                // patch rows that exist in the image
    const int rhi = min(rows + 2, H - ho0 + 1);
#pragma unroll
    for (int i = 0; i < PTI; ++i) {
      const bool ok = ((wi_ok >> i) & 1u) & (pt_r[i] >= rlo) & (pt_r[i] < rhi);
      const void* src = ok ? (const void*)(x + x0 + pt_rel[i]) : (const void*)zero;
      glds16(src, pb + (wave * PTI + i) * 1024);
    }
  };

  // ---- fragment geometry: slots this lane's transposed reads start at (k0 and k0 + 4)
  const int grp16 = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  const int bchunk = wci * 2 + (pq >> 1);  // this wave's ci block: 16 cols = 2 chunks
  const int bhalf = pq & 1;
  // LDS byte offsets (from a stage's base) of every transposed read of a k-step: A (dy image,
  // the MC loader's lane map) per [ks][co block][half], B (patch) per [unit][half]
  uint32_t aoff[2][CB][2], boff[18][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int k0 = ks * 32 + 8 * grp16 + q;
    const int pp0 = slot_pix(k0, W, RW, PW), pp1 = slot_pix(k0 + 4, W, RW, PW);
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const uint32_t c = (uint32_t)((wco >> 3) + i * 2 + (pq >> 1));
      aoff[ks][i][0] = mc_off<64>((uint32_t)k0, c) + 8 * bhalf;
      aoff[ks][i][1] = mc_off<64>((uint32_t)k0 + 4, c) + 8 * bhalf;
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int toff = (t / 3) * PW + (t % 3);
      boff[ks * 9 + t][0] = kDyBytes + mc_off<64>((uint32_t)(pp0 + toff), (uint32_t)bchunk) + 8 * bhalf;
      boff[ks * 9 + t][1] = kDyBytes + mc_off<64>((uint32_t)(pp1 + toff), (uint32_t)bchunk) + 8 * bhalf;
    }
  }

  f32x4 acc[9][CB];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < CB; ++i) acc[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one k-step reading stage buffer `cur` (while step+2 is staged into `nxt`)
  auto kstep = [&](const char* cur, char* nxt, int step) {
    // Branch-free schedule (a join of "staged" / "not staged" paths makes hipcc's waitcnt pass
    // drain vmcnt(0) before the next ds_read): the stage two k-steps ahead is always issued,
    // past the end it re-stages the last k-step into a buffer nobody reads again, so exactly one
    // younger stage is in flight at every wait.
    wait_vmcnt<LOADS>();  // this wave's loads of `step` landed
    // every wave's loads of `step` landed, and every wave finished reading step-1's buffer
    __builtin_amdgcn_s_waitcnt((7 << 4) | (0 << 8) | 15 | (3 << 14));  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    stage(nxt, min(step + 2, s1 - 1));
    const uint32_t base = lds_u32(cur);
    Frags<CB> f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < CB; ++i) {
        f.a_lo[ks][i] = tr_read(base + aoff[ks][i][0]);
        f.a_hi[ks][i] = tr_read(base + aoff[ks][i][1]);
      }
    auto issueB = [&](int u) {
      f.b_lo[u] = tr_read(base + boff[u][0]);
      f.b_hi[u] = tr_read(base + boff[u][1]);
    };
#pragma unroll
    for (int u = 0; u < LOOK; ++u) issueB(u);
    __builtin_amdgcn_s_setprio(1);
    units<LOOK>(f, acc, issueB, std::make_integer_sequence<int, 18>{});
    __builtin_amdgcn_s_setprio(0);
  };

  if (s0 < s1) {
    stage(smem0, s0);
    stage(smem1, min(s0 + 1, s1 - 1));
    for (int step = s0; step < s1; step += kStages) {  // buffers: step % 3 -> smem0/1/2
      kstep(smem0, smem2, step);
      if (step + 1 < s1) kstep(smem1, smem0, step + 1);
      if (step + 2 < s1) kstep(smem2, smem1, step + 2);
    }
    wait_vmcnt<0>();  // the trailing dummy stages
  }
  // ---- partial tile -> workspace slice blockIdx.y: lane holds C[co][ci..ci+3] per (tap, i)
  float* out = ws + (long)blockIdx.y * g.ws_stride;
  const int ci = ci0 + wci * 16 + 4 * (lane >> 4);
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int co = co0 + wco + i * 16 + (lane & 15);
      *reinterpret_cast<float4*>(out + ((long)co * 9 + t) * g.Ci + ci) =
          make_float4(acc[t][i][0], acc[t][i][1], acc[t][i][2], acc[t][i][3]);
    }
}

}  // namespace w3

bool g_wgrad3x3 = [] {
  const char* v = getenv("MIPIPE_WGRAD3");
  return v == nullptr || atoi(v) != 0;
}();

int g_wgrad3x3_waves = [] {
  const char* v = getenv("MIPIPE_WGRAD3_WAVES");
  return v != nullptr && atoi(v) == 4 ? 4 : 8;
}();

bool conv_wgrad3x3_supported(const ConvShape& s) {
  if (s.f32 || s.KH != 3 || s.KW != 3 || s.stride != 1 || s.pad != 1) return false;
  if ((s.stride_w != 0 && s.stride_w != 1) || (s.pad_w >= 0 && s.pad_w != 1)) return false;
  if (s.Ci % w3::TC != 0 || s.Co % w3::TM != 0 || s.W > 62 || s.W < 1) return false;
  const int R = std::min(s.H, w3::kSlots / s.W);
  if (R < 1 || (R + 2) * (s.W + 2) > w3::kPatchPix) return false;
  return (long)s.N * s.H * s.W * std::max(s.Ci, s.Co) < (1ll << 31);
}

// splits used for a shape (workspace slices): about one block per CU in total (one 4-wave block
// fits a CU: 96 KB of LDS, ~350 VGPR+AGPR per lane)
int conv_wgrad3x3_splits(const ConvShape& s, int splits_req) {
  const int R = std::min(s.H, w3::kSlots / s.W);
  const int steps = s.N * ((s.H + R - 1) / R);
  const int tiles = (s.Co / w3::TM) * (s.Ci / w3::TC);
  int S = splits_req > 0 ? splits_req : std::max(1, 256 / tiles);
  S = std::min(S, steps);
  const int per = (steps + S - 1) / S;
  return (steps + per - 1) / per;
}

void conv_wgrad3x3(const void* dy, const void* x, float* dw, const ConvShape& s, hipStream_t st,
                   float* ws, int splits, const BnCollect* col) {
  w3::Geo g;
  g.N = s.N; g.H = s.H; g.W = s.W; g.Ci = s.Ci; g.Co = s.Co;
  g.R = std::min(s.H, w3::kSlots / s.W);
  g.G = (s.H + g.R - 1) / g.R;
  g.PW = s.W + 2;
  g.steps = s.N * g.G;
  const int S = std::max(1, splits);
  g.per = (g.steps + S - 1) / S;
  g.ws_stride = (long)s.Co * 9 * s.Ci;
  const int tiles = (s.Co / w3::TM) * (s.Ci / w3::TC);
  BnCollect c{};
  if (col != nullptr) c = *col;
  if (g_wgrad3x3_waves == 4)
    hipLaunchKernelGGL(w3::wgrad3x3_kernel<4>, dim3(tiles, S), dim3(256), 0, st,
                       (const __bf16*)dy, (const __bf16*)x, ws, g, c);
  else
    hipLaunchKernelGGL(w3::wgrad3x3_kernel<8>, dim3(tiles, S), dim3(512), 0, st,
                       (const __bf16*)dy, (const __bf16*)x, ws, g, c);
  splitk_sum(ws, S, g.ws_stride, dw, st);
}

}  // namespace mipipe
