// Implicit-GEMM convolution (forward, data-grad, weight-grad) for NHWC bf16 / fp32 on gfx950.
//
//   forward : M = N*Ho*Wo, N = Co, K = KH*KW*Ci   A = im2col(x) (gathered rows), B = W[Co][K]
//   dgrad   : M = N*H*W,   N = Ci, K = KH*KW*Co   A = gather(dy), B = W viewed [K=(tap,co)][Ci]
//   wgrad   : M = Co, N = KH*KW*Ci, K = N*Ho*Wo  A = dy^T (k-major), B = im2col(x)^T, split-K
//
// Forward fuses the BatchNorm batch-statistics reduction into its epilogue (shifted per-channel
// sum / sum-of-squares of the fp32 accumulators), so BN never re-reads y for statistics.
// 1x1 / stride-1 / pad-0 convolutions take the dense-operand fast path (no gather math).
//
// Every kernel is a template over a TILE CONFIG (block tile, LDS stages, wave grid).  The host
// picks the config per problem: the measured table (conv_tune.cpp: per-shape autotuning, the
// cudnn.benchmark analogue) when one exists, else the heuristic in default_*_cfg().  The three
// ops live in separate translation units (conv_fwd.hip / conv_dgrad.hip / conv_wgrad.hip).
#pragma once
#include "epilogue.hpp"
#include "gemm_pp.hpp"
#include "launchers.hpp"

namespace mipipe {
namespace gk {

// zero page for padding taps / out-of-range rows (one per translation unit: no -fgpu-rdc)
static __device__ __attribute__((aligned(64))) uint4 g_conv_zero[8];

// Block tile BM x BN, NS LDS stages, WM x WN waves (wave tile (BM/WM) x (BN/WN)).
// PP: the ping-pong 8-wave main loop of gemm_pp.hpp (2 LDS stages of half tiles; accumulators
// in its half-tile row/column map, which the epilogues take as HALVES).
template <int BM_, int BN_, int NS_, int WM_, int WN_, bool PP_ = false>
struct Tile {
  static constexpr int BM = BM_, BN = BN_, NS = NS_, WM = WM_, WN = WN_;
  static constexpr int NW = WM * WN;
  static constexpr int THREADS = 64 * NW;
  static constexpr bool PP = PP_;
};

// The config table.  Ids are stable (they key the tuning table).
//  0: 128x128, 2 stages, 2x2 waves   — general default
//  1: 128x128, 1 stage               — short-K / memory-bound (3 blocks per CU)
//  2: 128x64,  2 stages              — narrow N (<= 64 channels)
//  3: 256x128, 2 stages, 4x2 waves   — large M: 85 FLOP per L2 byte (128x128: 64)
//  4: 256x128, 3 stages, 4x2 waves   — same, two k-steps of loads in flight (counted vmcnt)
//  5: 128x256, 2 stages, 2x4 waves   — large N
//  6: 256x256, 2 stages, 4x2 waves   — 64x128 wave tiles, 128 FLOP per L2 byte
//  7: 256x64,  2 stages, 4x1 waves   — large M, narrow N
//  8: 64x128,  2 stages, 2x2 waves   — narrow M (weight-grad of <= 64 output channels)
//  9: 128x64,  1 stage               — short-K streaming convs (one or two k-steps, large M):
//     24.6 KB of LDS -> 6 blocks per CU to keep more epilogue traffic in flight
// 10: 64x128,  1 stage               — same for narrow M
// 11: 256x256, ping-pong 2x4 waves    — large GEMMs: 1.38 PF on 4096^3 vs 1.22 PF for config 6
//     (tools/gemm_lab/pp_lab.hip, profiles/r4_pp_lab_v1.jsonl)
// 12: 256x128, ping-pong 2x4 waves    — large M, medium N
// 13: 128x256, ping-pong 2x4 waves    — medium M, large N
// 14: 128x128, ping-pong 2x4 waves    — the 8-wave schedule for mid-size convs whose 256-wide
//     tiles leave CUs idle (e.g. 14x14x256 3x3: 196 tiles of 256x256 for 256 CUs); 64 KB of LDS,
//     two blocks per CU
typedef Tile<128, 128, 2, 2, 2> T0;
typedef Tile<128, 128, 1, 2, 2> T1;
typedef Tile<128, 64, 2, 2, 2> T2;
typedef Tile<256, 128, 2, 4, 2> T3;
typedef Tile<256, 128, 3, 4, 2> T4;
typedef Tile<128, 256, 2, 2, 4> T5;
typedef Tile<256, 256, 2, 4, 2> T6;
typedef Tile<256, 64, 2, 4, 1> T7;
typedef Tile<64, 128, 2, 2, 2> T8;
typedef Tile<128, 64, 1, 2, 2> T9;
typedef Tile<64, 128, 1, 2, 2> T10;
typedef Tile<256, 256, 2, 2, 4, true> T11;
typedef Tile<256, 128, 2, 2, 4, true> T12;
typedef Tile<128, 256, 2, 2, 4, true> T13;
typedef Tile<128, 128, 2, 2, 4, true> T14;
constexpr int kNumTiles = 15;
static_assert(kNumTiles == kConvTileConfigs, "launchers.hpp tile count");

// fp32 operands run the split-bf16x3 loop (3 LDS images): 4-wave tiles only.
template <class T>
constexpr bool tile_ok_for(int cfg) {
  return std::is_same<T, float>::value ? (cfg == 0 || cfg == 2 || cfg == 8)
                                       : (cfg >= 0 && cfg < kNumTiles);
}

template <class T, class C>
constexpr int main_lds_bytes() {
  return std::is_same<T, float>::value  // split-bf16x3 images, one or two stages
             ? f32_stages<C::BM, C::BN>() * 3 * (C::BM + C::BN) * BK * 2
             : C::NS * (C::BM + C::BN) * BK * 2;
}
template <class T, class C>
constexpr int lds_bytes_out() {
  constexpr int a = main_lds_bytes<T, C>();
  constexpr int b = kEpiLdsBytes<C::BM, C::BN, T, C::WM>();
  return a > b ? a : b;
}
template <class T, class C>
constexpr int lds_bytes_f32out() {
  constexpr int a = main_lds_bytes<T, C>();
  constexpr int b = kEpiF32Rows<C::BM, C::BN, C::PP>() * (C::BN * 4 + 16);
  return a > b ? a : b;
}

// Operand-policy families: template <int R, int NW> using type = <policy over R rows, NW waves>.
// bf16 operands take the buffer-descriptor policies (KCDenseBuf / MCDenseBuf / KCIm2colBuf:
// fixed per-lane voffsets, k-step in soffset); fp32 operands feed the split-bf16x3 loop through
// registers and keep the pointer policies.  MIPIPE_NO_BUF_OPERANDS (compile-time) restores the
// pointer policies everywhere (A/B).
#ifdef MIPIPE_NO_BUF_OPERANDS
constexpr bool kBufOperands = false;
#else
constexpr bool kBufOperands = true;
#endif
template <class T>
constexpr bool use_buf() { return kBufOperands && !std::is_same<T, float>::value; }
template <class T> struct PolKCDense {
  template <int R, int NW>
  using type = typename std::conditional<use_buf<T>(), KCDenseBuf<R, T, NW>, KCDense<R, T, NW>>::type;
};
template <class T> struct PolMCDense {
  template <int R, int NW>
  using type = typename std::conditional<use_buf<T>(), MCDenseBuf<R, T, NW>, MCDense<R, T, NW>>::type;
};
// the buffer im2col needs the ALIGNED tap-uniform k-steps and a <= 32-tap mask; the host sends
// larger filters (KH*KW > 32) down the unaligned pointer path (conv_fwd.hip)
template <bool AL, class T> struct PolKCIm2col {
  template <int R, int NW>
  using type = typename std::conditional<AL && use_buf<T>(), KCIm2colBuf<R, T, NW>,
                                         KCIm2col<R, AL, T, NW>>::type;
};
// the buffer data-grad operands need Co % 64 == 0 (ALIGNED) and <= 32 class taps
template <bool AL, class T> struct PolKCDgrad {
  template <int R, int NW>
  using type = typename std::conditional<AL && use_buf<T>(), KCDgradBuf<R, T, NW>,
                                         KCDgrad<R, AL, T, NW>>::type;
};
template <bool AL, class T> struct PolMCDgradW {
  template <int R, int NW>
  using type = typename std::conditional<AL && use_buf<T>(), MCDgradWBuf<R, T, NW>,
                                         MCDgradW<R, T, NW>>::type;
};
// folded BatchNorm on the input (bf16 dense convs only: the buffer policies + fragment transform)
template <class T> struct PolKCDenseBN {
  template <int R, int NW>
  using type = KCDenseBufBN<R, T, NW>;
};
template <class T> struct PolMCDenseBN {
  template <int R, int NW>
  using type = MCDenseBufBN<R, T, NW>;
};
// channels of the folded-BN (scale, bias) LDS table (float2 each) of a BNIN forward
constexpr int kBnInMaxK = kConvBnInMaxK;
template <class T> struct PolMCIm2colT {
  template <int R, int NW>
  using type = typename std::conditional<use_buf<T>(), MCIm2colTBuf<R, T, NW>, MCIm2colT<R, T, NW>>::type;
};

// The main loop of tile config C over k-steps [kt0, kt1).  Operand policies come from the
// families PA / PB; ia(op, row_origin) / ib(op, col_origin) initialise one policy instance.
// Ping-pong tiles stage half tiles: two instances per operand (origins +0 and +BM/2 / +BN/2).
template <class T, class C, class PA, class PB, int V = kLoopDefault, class IA, class IB>
__device__ __forceinline__ void run_main_loop(char* smem, IA&& ia, IB&& ib, uint32_t m0,
                                              uint32_t n0, int kt0, int kt1,
                                              f32x4 (&acc)[C::BM / C::WM / 16][C::BN / C::WN / 16],
                                              int wave, int lane) {
  if constexpr (C::PP) {
    static_assert(!std::is_same<T, float>::value, "ping-pong tiles are bf16-only");
    typedef typename PA::template type<C::BM / 2, C::NW> OA;
    typedef typename PB::template type<C::BN / 2, C::NW> OB;
    OA a[2];
    OB b[2];
    ia(a[0], m0);
    ia(a[1], m0 + C::BM / 2);
    ib(b[0], n0);
    ib(b[1], n0 + C::BN / 2);
    MainLoopPP<C::BM, C::BN, OA, OB, C::WM, C::WN>::run(smem, a, b, kt0, kt1, acc, wave, lane);
  } else {
    typedef typename PA::template type<C::BM, C::NW> OA;
    typedef typename PB::template type<C::BN, C::NW> OB;
    OA a;
    OB b;
    ia(a, m0);
    ib(b, n0);
    MainLoopFor<T, C::BM, C::BN, OA, OB, C::NS, C::WM, C::WN, V>::type::run(smem, a, b, kt0, kt1,
                                                                            acc, wave, lane);
  }
}
// Minimum resident blocks per CU promised to the register allocator.
template <class T, class C>
constexpr int conv_occ() {
  // (asking 5-6 blocks of the single-stage half-size tiles 9/10 spills: they need ~100 VGPRs)
  // (8-wave tiles: one block per CU, two for the 64 KB 128x128 ping-pong tile)
  // (two-stage fp32 tiles: 144 KB of LDS, one block per CU -> the register budget of one)
  if (std::is_same<T, float>::value && f32_stages<C::BM, C::BN>() == 2) return 1;
  return C::NW == 8 ? (C::BM * C::BN <= 128 * 128 ? 2 : 1)
                    : ((C::NS == 1 && !std::is_same<T, float>::value) ? 3 : 2);
}

// DGRAD_EPI: the same im2col main loop run as a stride-1 data-grad (x = dy, w = the tap-flipped
// [Ci][KH][KW][Co] weight, pad = K-1-pad) with the data-grad epilogue and its fusions.
// SPLIT: split-K plan — blockIdx.y runs k-steps [y*e.split_kt, (y+1)*e.split_kt) and writes its
// fp32 partial tile to slice y of e.split_ws; conv_splitk_finish_kernel runs the epilogue.
template <class T, class C, bool SPLIT>
constexpr int conv_fwd_lds_bytes() {
  return SPLIT && lds_bytes_f32out<T, C>() > lds_bytes_out<T, C>() ? lds_bytes_f32out<T, C>()
                                                                   : lds_bytes_out<T, C>();
}
// BNIN: folded BatchNorm on the input (dense bf16, non-ping-pong tiles, K <= kBnInMaxK): x holds
// y and the A fragments are transformed to relu(y*e.in_scale + e.in_bias) after their LDS read
// (the (scale, bias) table sits in LDS behind the stage buffers).
template <class T, class C, bool BNIN>
constexpr int bnin_lds_bytes() {
  return BNIN ? main_lds_bytes<T, C>() + kBnInMaxK * 8 : 0;
}
template <class C, bool DENSE, bool ALIGNED, class T, bool DGRAD_EPI = false, bool SPLIT = false,
          bool BNIN = false>
__global__ __launch_bounds__(C::THREADS, (conv_occ<T, C>())) void conv_fwd_kernel(
    const T* __restrict__ x, const T* __restrict__ w, ConvGeom g, uint32_t M,
    uint32_t tilesN, EpiParams e) {
  constexpr int BM = C::BM, BN = C::BN;
  static_assert(!BNIN || (DENSE && !C::PP && !SPLIT && !DGRAD_EPI), "folded-BN forward variant");
  typedef typename std::conditional<
      BNIN, PolKCDenseBN<T>,
      typename std::conditional<DENSE, PolKCDense<T>, PolKCIm2col<ALIGNED, T>>::type>::type PA;
  constexpr int kLds = conv_fwd_lds_bytes<T, C, SPLIT>() > bnin_lds_bytes<T, C, BNIN>()
                           ? conv_fwd_lds_bytes<T, C, SPLIT>()
                           : bnin_lds_bytes<T, C, BNIN>();
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  uint32_t ntile = gridDim.x;
  if constexpr (!DGRAD_EPI) {
    if (e.fl_wt != nullptr) {  // trailing blocks: the data-grad's flipped weight
      if (blockIdx.x >= e.fl_tiles) {
        if (SPLIT && blockIdx.y != 0) return;  // once, not per split
        flip_block<T, C::THREADS>(e, blockIdx.x - e.fl_tiles, smem);
        return;
      }
      ntile = e.fl_tiles;
    }
  }
  const uint32_t id = xcd_remap(blockIdx.x, ntile);
  const uint32_t tm = id / tilesN, tn = id % tilesN;
  const uint32_t m0 = tm * BM, n0 = tn * BN;
  const uint32_t K = (uint32_t)(g.KH * g.KW * g.C);
  const int nk = (int)((K + BK - 1) / BK);
  int kt0 = 0, kt1 = nk;
  if constexpr (SPLIT) {
    kt0 = (int)blockIdx.y * e.split_kt;
    kt1 = min(nk, kt0 + e.split_kt);
  }
  char* bn_tab = smem + main_lds_bytes<T, C>();
  if constexpr (BNIN) {  // (ordered before the first fragment read by the main loop's barrier)
    float2* tab = reinterpret_cast<float2*>(bn_tab);
    for (int c = threadIdx.x; c < nk * BK; c += C::THREADS)
      tab[c] = (uint32_t)c < K ? make_float2(e.in_scale[c], e.in_bias[c]) : make_float2(0.f, 0.f);
  }
  auto ia = [&](auto& a, uint32_t origin) {
    if constexpr (DENSE) a.init(x, g.C, M, K, origin, wave, lane, g_conv_zero);
    else a.init(x, g, M, origin, wave, lane, g_conv_zero);
    if constexpr (BNIN) a.tab = bn_tab;
  };
  auto ib = [&](auto& b, uint32_t origin) { b.init(w, K, e.N, K, origin, wave, lane, g_conv_zero); };
  f32x4 acc[BM / C::WM / 16][BN / C::WN / 16];
  run_main_loop<T, C, PA, PolKCDense<T>>(smem, ia, ib, m0, n0, kt0, kt1, acc, wave, lane);
  if constexpr (SPLIT) {
    EpiParams ws{};  // this split's partial tile -> slice blockIdx.y ([splits][M][N], pitch N)
    ws.C = e.split_ws;
    ws.ldc = e.N;
    ws.M = M;
    ws.N = e.N;
    ws.det_rows = 1;
    epilogue_f32<BM, BN, true, C::WM, C::WN, C::PP>(smem, acc, ws, m0, n0, wave, lane);
  } else {
    epilogue_out<BM, BN, DGRAD_EPI, T, C::WM, C::WN, false, C::PP>(smem, acc, e, m0, n0, 0, wave,
                                                                   lane);
  }
}

// Finish of a split-K conv plan: each lane sums its accumulator positions over the splits in
// slice order (every slice's loads of a position issued together), then the block runs the
// regular output epilogue on the sum — BatchNorm statistics, bias / ReLU, the data-grad row remap
// and BN-backward fusions — exactly as the unsplit kernel would have on its accumulators.
template <class T, class C>
constexpr int finish_lds_bytes() {
  constexpr int a = kEpiLdsBytes<C::BM, C::BN, T, C::WM>();
  constexpr int b = 16 * (C::THREADS + 8) * 4;  // the BN-backward column-sum rows
  return a > b ? a : b;
}
template <class C, class T, bool FUSE>
__global__ __launch_bounds__(C::THREADS) void conv_splitk_finish_kernel(
    const float* __restrict__ ws, int S, uint32_t tilesN, EpiParams e) {
  constexpr int BM = C::BM, BN = C::BN, WM = C::WM, WN = C::WN;
  constexpr int MT = BM / WM / 16, NT = BN / WN / 16;
  __shared__ __attribute__((aligned(16))) char smem[finish_lds_bytes<T, C>()];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t tm = blockIdx.x / tilesN, tn = blockIdx.x % tilesN;
  const uint32_t m0 = tm * BM, n0 = tn * BN;
  const int wr = wave / WN, wc = wave % WN;
  typedef AccMap<BM, BN, WM, WN, false> Map;
  const uint32_t lr = lane & 15, lc = (lane >> 4) * 4;
  const long slice = (long)e.M * e.N;
  long off[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const uint32_t m = min(m0 + Map::row(wr, i) + lr, e.M - 1);  // clamped: masked later
      const uint32_t n = n0 + Map::col(wc, j) + lc;
      off[i][j] = (long)m * e.N + (n < e.N ? n : 0);
    }
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const float4 v = *reinterpret_cast<const float4*>(ws + off[i][j]);
      acc[i][j] = f32x4{v.x, v.y, v.z, v.w};
    }
  for (int s = 1; s < S; ++s) {  // slice order: deterministic
    const float* wsl = ws + s * slice;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const float4 v = *reinterpret_cast<const float4*>(wsl + off[i][j]);
        acc[i][j] += f32x4{v.x, v.y, v.z, v.w};
      }
  }
  epilogue_out<BM, BN, FUSE, T, WM, WN, false, false>(smem, acc, e, m0, n0, 0, wave, lane);
}

// TWO: BN-backward fusion of a two-branch block output (dense bf16 data-grads only)
template <class C, bool DENSE, bool ALIGNED, class T, bool TWO = false>
__global__ __launch_bounds__(C::THREADS, (conv_occ<T, C>())) void conv_dgrad_kernel(
    const T* __restrict__ dy, const T* __restrict__ w, int Ho, int Wo, int Co, int taps,
    FastDiv fCo, DgradClass cls, uint32_t M, uint32_t tilesN, EpiParams e) {
  constexpr int BM = C::BM, BN = C::BN;
  typedef typename std::conditional<DENSE, PolKCDense<T>, PolKCDgrad<ALIGNED, T>>::type PA;
  typedef typename std::conditional<DENSE, PolMCDense<T>, PolMCDgradW<ALIGNED, T>>::type PB;
  __shared__ __attribute__((aligned(16))) char smem[lds_bytes_out<T, C>()];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t id = xcd_remap(blockIdx.x, gridDim.x);
  const uint32_t tm = id / tilesN, tn = id % tilesN;
  const uint32_t m0 = tm * BM, n0 = tn * BN;
  const uint32_t Ci = e.N;
  const uint32_t K = (uint32_t)(cls.ntaps * Co);
  const int nk = (int)((K + BK - 1) / BK);
  auto ia = [&](auto& a, uint32_t origin) {
    if constexpr (DENSE) a.init(dy, Co, M, K, origin, wave, lane, g_conv_zero);
    else a.init(dy, Ho, Wo, Co, fCo, cls, M, origin, wave, lane, g_conv_zero);
  };
  auto ib = [&](auto& b, uint32_t origin) {
    if constexpr (DENSE) b.init(w, Ci, Ci, K, origin, wave, lane, g_conv_zero);
    else b.init(w, (uint32_t)Co, (uint32_t)taps, Ci, fCo, cls, origin, wave, lane, g_conv_zero);
  };
  f32x4 acc[BM / C::WM / 16][BN / C::WN / 16];
  run_main_loop<T, C, PA, PB>(smem, ia, ib, m0, n0, 0, nk, acc, wave, lane);
  epilogue_out<BM, BN, true, T, C::WM, C::WN, TWO, C::PP>(smem, acc, e, m0, n0, 0, wave, lane);
}

// ATOMIC: split-K partial tiles added with fp32 atomics; else the block owns its output tile
// (no split) and adds it with a plain read-modify-write (e.rmw) or writes a workspace slice.
// BNIN: folded BatchNorm on the input (dense bf16, 4-wave tiles): x holds y and the B fragments
// are transformed to relu(y*e.in_scale + e.in_bias) after their LDS read.
template <class C, bool DENSE, class T, bool ATOMIC = true, bool BNIN = false>
__global__ __launch_bounds__(C::THREADS, (conv_occ<T, C>())) void conv_wgrad_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, ConvGeom g, uint32_t tilesN,
    int kt_per_split, EpiParams e) {
  constexpr int BM = C::BM, BN = C::BN;
  static_assert(!BNIN || (DENSE && !C::PP), "folded-BN weight-grad variant");
  typedef typename std::conditional<
      BNIN, PolMCDenseBN<T>,
      typename std::conditional<DENSE, PolMCDense<T>, PolMCIm2colT<T>>::type>::type PB;
  __shared__ __attribute__((aligned(16))) char smem[lds_bytes_f32out<T, C>()];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t id = xcd_remap(blockIdx.x, gridDim.x);
  const uint32_t tm = id / tilesN, tn = id % tilesN;
  const uint32_t m0 = tm * BM, n0 = tn * BN;
  const uint32_t Co = e.M;
  const uint32_t K = (uint32_t)(g.N * g.Ho * g.Wo);
  const int nk = (int)((K + BK - 1) / BK);
  const int kt0 = blockIdx.y * kt_per_split;
  const int kt1 = min(nk, kt0 + kt_per_split);
  if (e.col.rep != nullptr && blockIdx.x == 0 && blockIdx.y == 0) bn_collect_block<C::THREADS>(e.col);
  auto ia = [&](auto& a, uint32_t origin) { a.init(dy, Co, Co, K, origin, wave, lane, g_conv_zero); };
  auto ib = [&](auto& b, uint32_t origin) {
    if constexpr (DENSE) b.init(x, g.C, g.C, K, origin, wave, lane, g_conv_zero);
    else b.init(x, g, origin, wave, lane, g_conv_zero, kt0);  // (the buffer policy starts at kt0)
    if constexpr (BNIN) {
      b.g_sc = e.in_scale;
      b.g_bi = e.in_bias;
      b.origin = origin;
      b.ncols = (uint32_t)g.C;
    }
  };
  f32x4 acc[BM / C::WM / 16][BN / C::WN / 16];
  run_main_loop<T, C, PolMCDense<T>, PB>(smem, ia, ib, m0, n0, kt0, kt1, acc, wave, lane);
  epilogue_f32<BM, BN, ATOMIC, C::WM, C::WN, C::PP>(smem, acc, e, m0, n0, wave, lane);
}

}  // namespace gk

// ------------------------------------------------------------------------------------ host
inline gk::ConvGeom make_geom(const ConvShape& s) {
  gk::ConvGeom g;
  g.stride_w = s.stride_w > 0 ? s.stride_w : s.stride;
  g.pad_w = s.pad_w >= 0 ? s.pad_w : s.pad;
  g.N = s.N; g.H = s.H; g.W = s.W; g.C = s.Ci; g.Ho = s.Ho; g.Wo = s.Wo;
  g.KH = s.KH; g.KW = s.KW; g.stride = s.stride; g.pad = s.pad;
  g.fHoWo = FastDiv((uint32_t)(s.Ho * s.Wo));
  g.fWo = FastDiv((uint32_t)s.Wo);
  g.fC = FastDiv((uint32_t)s.Ci);
  g.fKW = FastDiv((uint32_t)s.KW);
  return g;
}

inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

inline bool is_dense(const ConvShape& s) { return conv_is_dense(s); }

// Dispatch a runtime config id to a compile-time tile: f(Tile) for valid ids.
// NO_WIDE: the op cannot stage a 256x256 fp32 tile in LDS (weight-grad): id 6 runs as 3.
template <class T, bool NO_WIDE = false, class F>
inline void with_tile(int cfg, F&& f) {
  using namespace gk;
  if constexpr (std::is_same<T, float>::value) {
    if (cfg == 2) f(T2{});
    else if (cfg == 8) f(T8{});
    else f(T0{});
  } else {
    switch (cfg) {
      case 1: f(T1{}); break;
      case 2: f(T2{}); break;
      case 3: f(T3{}); break;
      case 4: f(T4{}); break;
      case 5: f(T5{}); break;
      case 6:
        if constexpr (NO_WIDE) f(T3{});
        else f(T6{});
        break;
      case 7: f(T7{}); break;
      case 8: f(T8{}); break;
      case 9: f(T9{}); break;
      case 10: f(T10{}); break;
      case 11: f(T11{}); break;
      case 12: f(T12{}); break;
      case 13: f(T13{}); break;
      case 14: f(T14{}); break;
      default: f(T0{}); break;
    }
  }
}

// Heuristic tile choice when the tuning table has no entry (measured round-1 rules).
int default_fwd_cfg(const ConvShape& s);
int default_dgrad_cfg(const ConvShape& s, long K_class);
int default_wgrad_cfg(const ConvShape& s);

}  // namespace mipipe
