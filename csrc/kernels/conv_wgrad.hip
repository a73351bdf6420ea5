// Convolution weight-grad: dw[Co][(kh,kw,ci)] += dy^T im2col(x), split-K over output pixels with
// fp32 atomics into the (flat DDP bucket) gradient.
#include "conv_common.hpp"

namespace mipipe {
using namespace gk;

int default_wgrad_cfg(const ConvShape& s) { return s.Co <= 64 ? 8 : 0; }

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
                         hipStream_t st, int cfg) {
  ConvGeom g = make_geom(s);
  const uint32_t Ntot = (uint32_t)(s.KH * s.KW * s.Ci);
  EpiParams e{};
  e.C = dw; e.ldc = Ntot; e.M = s.Co; e.N = Ntot;
  const bool dense = is_dense(s);
  const long K = (long)s.N * s.Ho * s.Wo;
  const int nk = (int)cdiv(K, BK);
  const T* dyp = (const T*)dy;
  const T* xp = (const T*)x;
  if (!tile_ok_for<T>(cfg)) cfg = default_wgrad_cfg(s);
  with_tile<T, true>(cfg, [&](auto tile) {
    typedef decltype(tile) C;
    const uint32_t tN = cdiv(Ntot, C::BN), tiles = cdiv(s.Co, C::BM) * tN;
    int splits = pick_splits(tiles, nk, s.Ci), per = (int)cdiv(nk, splits);
    splits = (int)cdiv(nk, per);
    const dim3 grid(tiles, splits), block(C::THREADS);
    if (dense)
      hipLaunchKernelGGL((conv_wgrad_kernel<C, true, T>), grid, block, 0, st, dyp, xp, g, tN, per, e);
    else
      hipLaunchKernelGGL((conv_wgrad_kernel<C, false, T>), grid, block, 0, st, dyp, xp, g, tN, per, e);
  });
}

void conv_wgrad(const void* dy, const void* x, float* dw, const ConvShape& s, hipStream_t st,
                int cfg) {
  if (s.f32) conv_wgrad_t<float>(dy, x, dw, s, st, cfg);
  else conv_wgrad_t<__bf16>(dy, x, dw, s, st, cfg);
}

}  // namespace mipipe
