// Convolution weight-grad: dw[Co][(kh,kw,ci)] += dy^T im2col(x), split-K over output pixels with
// fp32 atomics into the (flat DDP bucket) gradient — or, unsplit, one block per output tile with
// a plain read-modify-write (no atomics).  The (tile, split count) plan is tuned per shape.
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

static int resolve_wgrad_cfg(const ConvShape& s, int cfg) {
  const bool ok = s.f32 ? tile_ok_for<float>(cfg) : tile_ok_for<__bf16>(cfg);
  return ok ? cfg : default_wgrad_cfg(s);
}

template <class C>
static void wgrad_grid(const ConvShape& s, uint32_t& tN, uint32_t& tiles, int& splits, int& per,
                       int splits_req) {
  const uint32_t Ntot = (uint32_t)(s.KH * s.KW * s.Ci);
  const int nk = (int)cdiv((uint64_t)s.N * s.Ho * s.Wo, BK);
  tN = cdiv(Ntot, C::BN);
  tiles = cdiv(s.Co, C::BM) * tN;
  splits = splits_req > 0 ? std::min(splits_req, nk) : pick_splits(tiles, nk, s.Ci);
  per = (int)cdiv(nk, splits);
  splits = (int)cdiv(nk, per);
}

int conv_wgrad_splits(const ConvShape& s, int cfg, int splits_req) {
  cfg = resolve_wgrad_cfg(s, cfg);
  int splits = 1;
  auto f = [&](auto tile) {
    uint32_t tN, tiles;
    int per;
    wgrad_grid<decltype(tile)>(s, tN, tiles, splits, per, splits_req);
  };
  if (s.f32) with_tile<float, true>(cfg, f);
  else with_tile<__bf16, true>(cfg, f);
  return splits;
}

template <class T>
static void conv_wgrad_t(const void* dy, const void* x, float* dw, const ConvShape& s,
                         hipStream_t st, int cfg, float* ws, int splits_req,
                         const BnCollect* col, const float* in_scale, const float* in_bias) {
  ConvGeom g = make_geom(s);
  const uint32_t Ntot = (uint32_t)(s.KH * s.KW * s.Ci);
  EpiParams e{};
  e.C = dw; e.ldc = Ntot; e.M = s.Co; e.N = Ntot;
  if (col != nullptr) e.col = *col;
  const bool dense = is_dense(s);
  const T* dyp = (const T*)dy;
  const T* xp = (const T*)x;
  cfg = resolve_wgrad_cfg(s, cfg);
  if (in_scale != nullptr) {  // folded input BN: dense bf16, 4-wave tiles
    e.in_scale = in_scale;
    e.in_bias = in_bias;
    if (cfg >= 11) cfg = default_wgrad_cfg(s);
  }
  int splits_used = 1;
  if (ws != nullptr) {  // deterministic: partial tiles to the workspace, summed in split order
    e.C = ws;
    e.det_rows = 1;
  }
  with_tile<T, true>(cfg, [&](auto tile) {
    typedef decltype(tile) C;
    uint32_t tN, tiles;
    int splits, per;
    wgrad_grid<C>(s, tN, tiles, splits, per, splits_req);
    splits_used = splits;
    const dim3 grid(tiles, splits), block(C::THREADS);
    EpiParams ee = e;
    // unsplit (and not the deterministic workspace path): the block owns its output tile ->
    // non-atomic read-modify-write; the ATOMIC template also carries the workspace-slice store
    const bool atomic = splits > 1 || ws != nullptr;
    if (!atomic) ee.rmw = 1;
    if constexpr (!C::PP && std::is_same<T, __bf16>::value) {
      if (in_scale != nullptr) {  // (host checks: dense)
        if (atomic) hipLaunchKernelGGL((conv_wgrad_kernel<C, true, T, true, true>), grid, block, 0, st, dyp, xp, g, tN, per, ee);
        else hipLaunchKernelGGL((conv_wgrad_kernel<C, true, T, false, true>), grid, block, 0, st, dyp, xp, g, tN, per, ee);
        return;
      }
    }
    if (dense) {
      if (atomic) hipLaunchKernelGGL((conv_wgrad_kernel<C, true, T, true>), grid, block, 0, st, dyp, xp, g, tN, per, ee);
      else hipLaunchKernelGGL((conv_wgrad_kernel<C, true, T, false>), grid, block, 0, st, dyp, xp, g, tN, per, ee);
    } else {
      if (atomic) hipLaunchKernelGGL((conv_wgrad_kernel<C, false, T, true>), grid, block, 0, st, dyp, xp, g, tN, per, ee);
      else hipLaunchKernelGGL((conv_wgrad_kernel<C, false, T, false>), grid, block, 0, st, dyp, xp, g, tN, per, ee);
    }
  });
  if (ws != nullptr) splitk_sum(ws, splits_used, (long)s.Co * Ntot, dw, st);
}

void conv_wgrad(const void* dy, const void* x, float* dw, const ConvShape& s, hipStream_t st,
                int cfg, float* ws, int splits, const BnCollect* col, const float* in_scale,
                const float* in_bias) {
  if (s.f32) conv_wgrad_t<float>(dy, x, dw, s, st, cfg, ws, splits, col, nullptr, nullptr);
  else conv_wgrad_t<__bf16>(dy, x, dw, s, st, cfg, ws, splits, col, in_scale, in_bias);
}

}  // namespace mipipe
