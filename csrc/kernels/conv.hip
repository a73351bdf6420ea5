// Implicit-GEMM convolution (forward, data-grad, weight-grad) for NHWC bf16 on gfx950.
//
//   forward : M = N*Ho*Wo, N = Co, K = KH*KW*Ci   A = im2col(x) (gathered rows), B = W[Co][K]
//   dgrad   : M = N*H*W,   N = Ci, K = KH*KW*Co   A = gather(dy), B = W viewed [K=(tap,co)][Ci]
//   wgrad   : M = Co, N = KH*KW*Ci, K = N*Ho*Wo  A = dy^T (k-major), B = im2col(x)^T, split-K
//
// Forward fuses the BatchNorm batch-statistics reduction into its epilogue (shifted per-channel
// sum / sum-of-squares of the fp32 accumulators), so BN never re-reads y for statistics.
// 1x1 / stride-1 / pad-0 convolutions take the dense-operand fast path (no gather math).
#include "epilogue.hpp"
#include "launchers.hpp"

namespace mipipe {
namespace gk {

__device__ __attribute__((aligned(64))) uint4 g_conv_zero[8];

// NS = LDS stages.  NS = 1 is used when the whole reduction is one k-step (K <= 64, e.g. the
// 64-channel 1x1 convs of layer1): half the LDS, so 3 blocks fit per CU instead of 2 and the
// block-level overlap of loads with epilogues hides these memory-bound layers' latency.
// LDS of a conv kernel: the main loop's stages, or the epilogue's staged tile + statistics.
template <class T, int BM, int BN, class OpA, class OpB, int NS>
constexpr int lds_bytes_out() {
  constexpr int a = MainLoopFor<T, BM, BN, OpA, OpB, NS>::LDS_BYTES;
  constexpr int b = kEpiLdsBytes<BM, BN, T>();
  return a > b ? a : b;
}
template <class T, int BM, int BN, class OpA, class OpB>
constexpr int lds_bytes_f32out() {
  constexpr int a = MainLoopFor<T, BM, BN, OpA, OpB, 2>::LDS_BYTES;
  constexpr int b = BM * (BN * 4 + 16);
  return a > b ? a : b;
}
// Occupancy hint: NS = 1 (bf16 single stage) fits 3 blocks per CU; 2 otherwise.
template <class T, int NS>
constexpr int conv_occ() { return (NS == 1 && !std::is_same<T, float>::value) ? 3 : 2; }

template <int BM, int BN, bool DENSE, int NS = 2, bool ALIGNED = false, class T = __bf16>
__global__ __launch_bounds__(256, (conv_occ<T, NS>())) void conv_fwd_kernel(
    const T* __restrict__ x, const T* __restrict__ w, ConvGeom g, uint32_t M,
    uint32_t tilesN, EpiParams e) {
  typedef typename std::conditional<DENSE, KCDense<BM, T>, KCIm2col<BM, ALIGNED, T>>::type OpA;
  typedef KCDense<BN, T> OpB;
  __shared__ __attribute__((aligned(16))) char smem[lds_bytes_out<T, BM, BN, OpA, OpB, NS>()];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t id = xcd_remap(blockIdx.x, gridDim.x);
  const uint32_t tm = id / tilesN, tn = id % tilesN;
  const uint32_t m0 = tm * BM, n0 = tn * BN;
  const uint32_t K = (uint32_t)(g.KH * g.KW * g.C);
  const int nk = (int)((K + BK - 1) / BK);
  OpA a;
  if constexpr (DENSE) a.init(x, g.C, M, K, m0, wave, lane, g_conv_zero);
  else a.init(x, g, M, m0, wave, lane, g_conv_zero);
  OpB b;
  b.init(w, K, e.N, K, n0, wave, lane, g_conv_zero);
  f32x4 acc[BM / 32][BN / 32];
  MainLoopFor<T, BM, BN, OpA, OpB, NS>::type::run(smem, a, b, 0, nk, acc, wave, lane);
  epilogue_out<BM, BN, false, T>(smem, acc, e, m0, n0, 0, wave, lane);
}

template <int BM, int BN, bool DENSE, int NS = 2, bool ALIGNED = false, class T = __bf16>
__global__ __launch_bounds__(256, (conv_occ<T, NS>())) void conv_dgrad_kernel(
    const T* __restrict__ dy, const T* __restrict__ w, int Ho, int Wo, int Co, int taps,
    FastDiv fCo, DgradClass cls, uint32_t M, uint32_t tilesN, EpiParams e) {
  typedef typename std::conditional<DENSE, KCDense<BM, T>, KCDgrad<BM, ALIGNED, T>>::type OpA;
  typedef typename std::conditional<DENSE, MCDense<BN, T>, MCDgradW<BN, T>>::type OpB;
  __shared__ __attribute__((aligned(16))) char smem[lds_bytes_out<T, BM, BN, OpA, OpB, NS>()];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t id = xcd_remap(blockIdx.x, gridDim.x);
  const uint32_t tm = id / tilesN, tn = id % tilesN;
  const uint32_t m0 = tm * BM, n0 = tn * BN;
  const uint32_t Ci = e.N;
  const uint32_t K = (uint32_t)(cls.ntaps * Co);
  const int nk = (int)((K + BK - 1) / BK);
  OpA a;
  OpB b;
  if constexpr (DENSE) {
    a.init(dy, Co, M, K, m0, wave, lane, g_conv_zero);
    b.init(w, Ci, Ci, K, n0, wave, lane, g_conv_zero);
  } else {
    a.init(dy, Ho, Wo, Co, fCo, cls, M, m0, wave, lane, g_conv_zero);
    b.init(w, (uint32_t)Co, (uint32_t)taps, Ci, fCo, cls, n0, wave, lane, g_conv_zero);
  }
  f32x4 acc[BM / 32][BN / 32];
  MainLoopFor<T, BM, BN, OpA, OpB, NS>::type::run(smem, a, b, 0, nk, acc, wave, lane);
  epilogue_out<BM, BN, true, T>(smem, acc, e, m0, n0, 0, wave, lane);
}

template <int BM, int BN, bool DENSE, class T = __bf16>
__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(const T* __restrict__ dy,
                                                             const T* __restrict__ x,
                                                             ConvGeom g, uint32_t tilesN,
                                                             int kt_per_split, EpiParams e) {
  typedef MCDense<BM, T> OpA;
  typedef typename std::conditional<DENSE, MCDense<BN, T>, MCIm2colT<BN, T>>::type OpB;
  __shared__ __attribute__((aligned(16))) char smem[lds_bytes_f32out<T, BM, BN, OpA, OpB>()];
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
  OpA a;
  a.init(dy, Co, Co, K, m0, wave, lane, g_conv_zero);
  OpB b;
  if constexpr (DENSE) b.init(x, g.C, g.C, K, n0, wave, lane, g_conv_zero);
  else b.init(x, g, n0, wave, lane, g_conv_zero);
  f32x4 acc[BM / 32][BN / 32];
  MainLoopFor<T, BM, BN, OpA, OpB, 2>::type::run(smem, a, b, kt0, kt1, acc, wave, lane);
  epilogue_f32<BM, BN, true>(smem, acc, e, m0, n0, wave, lane);
}

}  // namespace gk

using namespace gk;

static ConvGeom make_geom(int N, int H, int W, int C, int Ho, int Wo, int KH, int KW, int stride,
                          int pad, int stride_w = 0, int pad_w = -1) {
  ConvGeom g;
  g.stride_w = stride_w > 0 ? stride_w : stride;
  g.pad_w = pad_w >= 0 ? pad_w : pad;
  g.N = N; g.H = H; g.W = W; g.C = C; g.Ho = Ho; g.Wo = Wo;
  g.KH = KH; g.KW = KW; g.stride = stride; g.pad = pad;
  g.fHoWo = FastDiv((uint32_t)(Ho * Wo));
  g.fWo = FastDiv((uint32_t)Wo);
  g.fC = FastDiv((uint32_t)C);
  g.fKW = FastDiv((uint32_t)KW);
  return g;
}

static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

static bool is_dense(const ConvShape& s) {
  return s.KH == 1 && s.KW == 1 && s.stride == 1 && s.pad == 0 && s.pad_w <= 0 &&
         (s.stride_w == 0 || s.stride_w == 1);
}

int conv_fwd_stat_rows(const ConvShape& s) {
  (void)s;
  return kStatReplicas;
}

#define MIPIPE_LAUNCH(kern, grid, ...) hipLaunchKernelGGL((kern), (grid), dim3(256), 0, st, __VA_ARGS__)

template <class T>
static void conv_fwd_t(const void* x, const void* w, void* y, float* st_sum, float* st_sq,
                       const float* st_shift, const ConvShape& s, hipStream_t st,
                       const float* bias, bool relu) {
  constexpr bool F = std::is_same<T, float>::value;  // fp32: one main loop (no NS=1 variants)
  ConvGeom g = make_geom(s.N, s.H, s.W, s.Ci, s.Ho, s.Wo, s.KH, s.KW, s.stride, s.pad, s.stride_w, s.pad_w);
  uint32_t M = (uint32_t)s.N * s.Ho * s.Wo;
  EpiParams e{};
  e.C = y; e.ldc = s.Co; e.M = M; e.N = s.Co; e.bias = bias; e.act = relu ? 1 : 0;
  e.st_sum = st_sum; e.st_sq = st_sq; e.st_shift = st_shift; e.st_R = g_stat_rows;
  const bool dense = is_dense(s);
  const T* xp = (const T*)x;
  const T* wp = (const T*)w;
  if (s.Co <= 64) {
    uint32_t tN = cdiv(s.Co, 64), tiles = cdiv(M, 128) * tN;
    if (dense) MIPIPE_LAUNCH((conv_fwd_kernel<128, 64, true, 2, false, T>), dim3(tiles), xp, wp, g, M, tN, e);
    else if (s.Ci % BK == 0) MIPIPE_LAUNCH((conv_fwd_kernel<128, 64, false, 2, true, T>), dim3(tiles), xp, wp, g, M, tN, e);
    else MIPIPE_LAUNCH((conv_fwd_kernel<128, 64, false, 2, false, T>), dim3(tiles), xp, wp, g, M, tN, e);
  } else {
    uint32_t tN = cdiv(s.Co, 128), tiles = cdiv(M, 128) * tN;
    if (!F && dense && s.Ci <= g_ns1_max_k) MIPIPE_LAUNCH((conv_fwd_kernel<128, 128, true, 1, false, T>), dim3(tiles), xp, wp, g, M, tN, e);
    else if (dense) MIPIPE_LAUNCH((conv_fwd_kernel<128, 128, true, 2, false, T>), dim3(tiles), xp, wp, g, M, tN, e);
    else if (!F && s.Ci % BK == 0 && (long)s.KH * s.KW * s.Ci <= g_ns1_max_k_gather) MIPIPE_LAUNCH((conv_fwd_kernel<128, 128, false, 1, true, T>), dim3(tiles), xp, wp, g, M, tN, e);
    else if (s.Ci % BK == 0) MIPIPE_LAUNCH((conv_fwd_kernel<128, 128, false, 2, true, T>), dim3(tiles), xp, wp, g, M, tN, e);
    else MIPIPE_LAUNCH((conv_fwd_kernel<128, 128, false, 2, false, T>), dim3(tiles), xp, wp, g, M, tN, e);
  }
}

void conv_fwd(const void* x, const void* w, void* y, float* st_sum, float* st_sq,
              const float* st_shift, const ConvShape& s, hipStream_t st, const float* bias,
              bool relu) {
  if (s.f32) conv_fwd_t<float>(x, w, y, st_sum, st_sq, st_shift, s, st, bias, relu);
  else conv_fwd_t<__bf16>(x, w, y, st_sum, st_sq, st_shift, s, st, bias, relu);
}

template <class T>
static void conv_dgrad_t(const void* dy, const void* w, void* dx, const ConvShape& s,
                         hipStream_t st, const DgradFusion* fz) {
  constexpr bool F = std::is_same<T, float>::value;
  const bool dense = is_dense(s);
  const T* dyp = (const T*)dy;
  const T* wp = (const T*)w;
  const int S = s.stride;
  const int PW = s.pad_w >= 0 ? s.pad_w : s.pad;  // horizontal padding
  FastDiv fCo((uint32_t)s.Co);
  for (int ph = 0; ph < S; ++ph) {
    for (int pw = 0; pw < S; ++pw) {
      DgradClass c{};
      c.ph = ph; c.pw = pw;
      c.Hc = (s.H - ph + S - 1) / S;
      c.Wc = (s.W - pw + S - 1) / S;
      if (c.Hc <= 0 || c.Wc <= 0) continue;
      // taps reaching this phase: kh = (ph + pad) mod S + S*a, kw likewise
      c.S = S; c.KW = s.KW;
      c.kh0 = (ph + s.pad) % S;
      c.kw0 = (pw + PW) % S;
      int nkh = c.kh0 < s.KH ? (s.KH - c.kh0 + S - 1) / S : 0;
      int nkw = c.kw0 < s.KW ? (s.KW - c.kw0 + S - 1) / S : 0;
      c.nkw = std::max(nkw, 1);
      c.ntaps = nkh * nkw;
      c.dh0 = (ph + s.pad - c.kh0) / S;
      c.dw0 = (pw + PW - c.kw0) / S;
      c.fnkw = FastDiv((uint32_t)c.nkw);
      c.fHcWc = FastDiv((uint32_t)(c.Hc * c.Wc));
      c.fWc = FastDiv((uint32_t)c.Wc);
      uint32_t M = (uint32_t)s.N * c.Hc * c.Wc;
      EpiParams e{};
      e.C = dx; e.ldc = s.Ci; e.M = M; e.N = s.Ci;
      if (fz != nullptr) {
        e.addend = fz->addend;
        e.bnr_y = fz->bn_y;
        e.bnr_mean = fz->bn_mean; e.bnr_invstd = fz->bn_invstd;
        e.bnr_scale = fz->bn_scale; e.bnr_bias = fz->bn_bias; e.bnr_rep = fz->bn_rep; e.st_R = g_stat_rows;
        e.bnr_z = fz->bn_z;
      }
      if (S > 1) {
        e.rm_s = S; e.rm_ph = ph; e.rm_pw = pw; e.rm_H = s.H; e.rm_W = s.W;
        e.rm_Hc = c.Hc; e.rm_Wc = c.Wc; e.rm_fHcWc = c.fHcWc; e.rm_fWc = c.fWc;
      }
      int taps = s.KH * s.KW;
      if (s.Ci <= 64) {
        uint32_t tN = cdiv(s.Ci, 64), tiles = cdiv(M, 128) * tN;
        if (dense) MIPIPE_LAUNCH((conv_dgrad_kernel<128, 64, true, 2, false, T>), dim3(tiles), dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
        else if (s.Co % BK == 0) MIPIPE_LAUNCH((conv_dgrad_kernel<128, 64, false, 2, true, T>), dim3(tiles), dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
        else MIPIPE_LAUNCH((conv_dgrad_kernel<128, 64, false, 2, false, T>), dim3(tiles), dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
      } else {
        uint32_t tN = cdiv(s.Ci, 128), tiles = cdiv(M, 128) * tN;
        if (!F && dense && s.Co <= g_ns1_max_k) MIPIPE_LAUNCH((conv_dgrad_kernel<128, 128, true, 1, false, T>), dim3(tiles), dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
        else if (dense) MIPIPE_LAUNCH((conv_dgrad_kernel<128, 128, true, 2, false, T>), dim3(tiles), dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
        else if (!F && s.Co % BK == 0 && (long)c.ntaps * s.Co <= g_ns1_max_k_gather) MIPIPE_LAUNCH((conv_dgrad_kernel<128, 128, false, 1, true, T>), dim3(tiles), dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
        else if (s.Co % BK == 0) MIPIPE_LAUNCH((conv_dgrad_kernel<128, 128, false, 2, true, T>), dim3(tiles), dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
        else MIPIPE_LAUNCH((conv_dgrad_kernel<128, 128, false, 2, false, T>), dim3(tiles), dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
      }
    }
  }
}

void conv_dgrad(const void* dy, const void* w, void* dx, const ConvShape& s, hipStream_t st,
                const DgradFusion* fz) {
  if (s.f32) conv_dgrad_t<float>(dy, w, dx, s, st, fz);
  else conv_dgrad_t<__bf16>(dy, w, dx, s, st, fz);
}

static int pick_splits(uint32_t tiles, int nk, int Ci) {
  // measured (tools/sweep_splitk.py): ~512 workgroups is best for most ResNet-50 wgrads; narrow
  // inputs (Ci <= 64: the 7x7 stem and layer1 3x3) prefer ~1.5x more
  int target = Ci <= 64 ? g_splitk_target * 3 / 2 : g_splitk_target;
  int splits = (int)std::max<uint32_t>(1, target / std::max<uint32_t>(1, tiles));
  int max_splits = std::max(1, nk / 4);
  return std::min(splits, max_splits);
}

template <class T>
static void conv_wgrad_t(const void* dy, const void* x, float* dw, const ConvShape& s,
                         hipStream_t st) {
  ConvGeom g = make_geom(s.N, s.H, s.W, s.Ci, s.Ho, s.Wo, s.KH, s.KW, s.stride, s.pad, s.stride_w, s.pad_w);
  uint32_t Ntot = (uint32_t)(s.KH * s.KW * s.Ci);
  EpiParams e{};
  e.C = dw; e.ldc = Ntot; e.M = s.Co; e.N = Ntot;
  const bool dense = is_dense(s);
  long K = (long)s.N * s.Ho * s.Wo;
  int nk = (int)cdiv(K, BK);
  const T* dyp = (const T*)dy;
  const T* xp = (const T*)x;
  if (s.Co <= 64) {
    uint32_t tN = cdiv(Ntot, 128), tiles = cdiv(s.Co, 64) * tN;
    int splits = pick_splits(tiles, nk, s.Ci), per = (int)cdiv(nk, splits);
    splits = (int)cdiv(nk, per);
    if (dense) MIPIPE_LAUNCH((conv_wgrad_kernel<64, 128, true, T>), dim3(tiles, splits), dyp, xp, g, tN, per, e);
    else MIPIPE_LAUNCH((conv_wgrad_kernel<64, 128, false, T>), dim3(tiles, splits), dyp, xp, g, tN, per, e);
  } else {
    uint32_t tN = cdiv(Ntot, 128), tiles = cdiv(s.Co, 128) * tN;
    int splits = pick_splits(tiles, nk, s.Ci), per = (int)cdiv(nk, splits);
    splits = (int)cdiv(nk, per);
    if (dense) MIPIPE_LAUNCH((conv_wgrad_kernel<128, 128, true, T>), dim3(tiles, splits), dyp, xp, g, tN, per, e);
    else MIPIPE_LAUNCH((conv_wgrad_kernel<128, 128, false, T>), dim3(tiles, splits), dyp, xp, g, tN, per, e);
  }
}

void conv_wgrad(const void* dy, const void* x, float* dw, const ConvShape& s, hipStream_t st) {
  if (s.f32) conv_wgrad_t<float>(dy, x, dw, s, st);
  else conv_wgrad_t<__bf16>(dy, x, dw, s, st);
}

}  // namespace mipipe
