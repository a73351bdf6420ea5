// Convolution forward: implicit GEMM over a tile config (conv_common.hpp), BN-statistics or
// bias/ReLU epilogue.
#include "conv_common.hpp"

namespace mipipe {
using namespace gk;

int conv_fwd_stat_rows(const ConvShape& s) {
  (void)s;
  return kStatReplicas;
}

int default_fwd_cfg(const ConvShape& s) {
  const bool dense = is_dense(s);
  const bool ns1 = !s.f32 && (dense ? s.Ci <= g_ns1_max_k
                                    : (s.Ci % BK == 0 && (long)s.KH * s.KW * s.Ci <= g_ns1_max_k_gather));
  if (s.Co <= 64) return 2;
  return ns1 ? 1 : 0;
}

static int resolve_fwd_cfg(const ConvShape& s, int cfg) {
  cfg = conv_plan_tile(cfg);
  const bool ok = s.f32 ? tile_ok_for<float>(cfg) : tile_ok_for<__bf16>(cfg);
  return ok ? cfg : default_fwd_cfg(s);
}

void conv_tile_dims(int cfg, bool f32, int* bm, int* bn) {
  auto f = [&](auto tile) {
    *bm = decltype(tile)::BM;
    *bn = decltype(tile)::BN;
  };
  if (f32) with_tile<float>(conv_plan_tile(cfg), f);
  else with_tile<__bf16>(conv_plan_tile(cfg), f);
}

long conv_fwd_split_ws_elems(const ConvShape& s, int cfg) {
  const int nk = (int)cdiv((uint64_t)s.KH * s.KW * s.Ci, BK);
  int S, kps;
  conv_split_geometry(nk, conv_plan_splits(cfg), &S, &kps);
  return S > 1 ? (long)S * s.N * s.Ho * s.Wo * s.Co : 0;
}

int conv_fwd_tiles_m(const ConvShape& s, int cfg) {
  cfg = resolve_fwd_cfg(s, cfg);
  int bm = 128;
  auto f = [&](auto tile) { bm = decltype(tile)::BM; };
  if (s.f32) with_tile<float>(cfg, f);
  else with_tile<__bf16>(cfg, f);
  return (int)cdiv((uint64_t)s.N * s.Ho * s.Wo, bm);
}

template <class T>
static void conv_fwd_t(const void* x, const void* w, void* y, float* st_sum, float* st_sq,
                       const float* st_shift, const ConvShape& s, hipStream_t st,
                       const float* bias, bool relu, int cfg, int det_rows, void* wflip,
                       float* split_ws, const float* in_scale, const float* in_bias) {
  ConvGeom g = make_geom(s);
  const uint32_t M = (uint32_t)s.N * s.Ho * s.Wo;
  EpiParams e{};
  e.C = y; e.ldc = s.Co; e.M = M; e.N = s.Co; e.bias = bias; e.act = relu ? 1 : 0;
  e.st_sum = st_sum; e.st_sq = st_sq; e.st_shift = st_shift; e.st_R = g_stat_rows;
  e.det_rows = det_rows;
  e.nt = (g_nt_store & 1) && (long)M * s.Co * (s.f32 ? 4 : 2) > g_nt_min_bytes;
  uint32_t nflip = 0;
  if (wflip != nullptr && dgrad_preflip_ok(s)) {
    e.fl_w = w; e.fl_wt = wflip;
    e.fl_Co = s.Co; e.fl_KH = s.KH; e.fl_KW = s.KW; e.fl_Ci = s.Ci;
    dgrad_flip_plan(s, e.fl);
    nflip = e.fl.nblk;
  }
  const bool dense = is_dense(s);
  // bf16 ALIGNED runs the buffer im2col (KCIm2colBuf: <= 32 taps in its bit mask)
  const bool aligned = s.Ci % BK == 0 && (s.f32 || s.KH * s.KW <= 32);
  const T* xp = (const T*)x;
  const T* wp = (const T*)w;
  const int nk = (int)cdiv((uint64_t)s.KH * s.KW * s.Ci, BK);
  int S, kps;
  conv_split_geometry(nk, split_ws != nullptr ? conv_plan_splits(cfg) : 1, &S, &kps);
  cfg = resolve_fwd_cfg(s, cfg);
  if (in_scale != nullptr) {  // folded input BN: dense bf16, 4-wave tiles, no split
    e.in_scale = in_scale;
    e.in_bias = in_bias;
    if (cfg >= 11) cfg = default_fwd_cfg(s);
    S = 1;
  }
  with_tile<T>(cfg, [&](auto tile) {
    typedef decltype(tile) C;
    const uint32_t tN = cdiv(s.Co, C::BN), tiles = cdiv(M, C::BM) * tN;
    EpiParams ee = e;
    ee.fl_tiles = tiles;
    const dim3 block(C::THREADS);
    // (the 256x256 4-wave tile cannot stage its fp32 partial tile in LDS: never split)
    constexpr bool kSplitOk = !(C::BM == 256 && C::BN == 256 && !C::PP);
    if constexpr (kSplitOk) if (S > 1) {  // split-K plan: partial tiles into the workspace, then the finish launch
      ee.split_kt = kps;
      ee.split_ws = split_ws;
      const dim3 grid(tiles + nflip, S);
      if (dense)
        hipLaunchKernelGGL((conv_fwd_kernel<C, true, false, T, false, true>), grid, block, 0, st, xp, wp, g, M, tN, ee);
      else if (aligned)
        hipLaunchKernelGGL((conv_fwd_kernel<C, false, true, T, false, true>), grid, block, 0, st, xp, wp, g, M, tN, ee);
      else
        hipLaunchKernelGGL((conv_fwd_kernel<C, false, false, T, false, true>), grid, block, 0, st, xp, wp, g, M, tN, ee);
      hipLaunchKernelGGL((conv_splitk_finish_kernel<C, T, false>), dim3(tiles), block, 0, st,
                         (const float*)split_ws, S, tN, e);
      return;
    }
    const dim3 grid(tiles + nflip);
    if constexpr (!C::PP && std::is_same<T, __bf16>::value) {
      if (in_scale != nullptr) {  // (host checks: dense, K <= kBnInMaxK)
        hipLaunchKernelGGL((conv_fwd_kernel<C, true, false, T, false, false, true>), grid, block, 0, st, xp, wp, g, M, tN, ee);
        return;
      }
    }
    if (dense)
      hipLaunchKernelGGL((conv_fwd_kernel<C, true, false, T>), grid, block, 0, st, xp, wp, g, M, tN, ee);
    else if (aligned)
      hipLaunchKernelGGL((conv_fwd_kernel<C, false, true, T>), grid, block, 0, st, xp, wp, g, M, tN, ee);
    else
      hipLaunchKernelGGL((conv_fwd_kernel<C, false, false, T>), grid, block, 0, st, xp, wp, g, M, tN, ee);
  });
}

void conv_fwd(const void* x, const void* w, void* y, float* st_sum, float* st_sq,
              const float* st_shift, const ConvShape& s, hipStream_t st, const float* bias,
              bool relu, int cfg, int det_rows, void* wflip, float* split_ws,
              const float* in_scale, const float* in_bias) {
  if (s.f32) conv_fwd_t<float>(x, w, y, st_sum, st_sq, st_shift, s, st, bias, relu, cfg, det_rows, wflip, split_ws, nullptr, nullptr);
  else conv_fwd_t<__bf16>(x, w, y, st_sum, st_sq, st_shift, s, st, bias, relu, cfg, det_rows, wflip, split_ws, in_scale, in_bias);
}

}  // namespace mipipe
