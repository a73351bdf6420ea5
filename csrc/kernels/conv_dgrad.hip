// Convolution data-grad: one implicit GEMM per stride parity class (sub-pixel decomposition,
// no structurally-zero MFMA work), with the dgrad epilogue fusions (residual addend, BN-backward
// reductions of the producing BN+ReLU).
#include "conv_common.hpp"

namespace mipipe {
using namespace gk;

int default_dgrad_cfg(const ConvShape& s, long K_class) {
  const bool dense = is_dense(s);
  const bool ns1 = !s.f32 && (dense ? s.Co <= g_ns1_max_k
                                    : (s.Co % BK == 0 && K_class <= g_ns1_max_k_gather));
  if (s.Ci <= 64) return 2;
  return ns1 ? 1 : 0;
}

// The parity classes of a stride-S dgrad: (class descriptor, rows M) in launch order.
template <class F>
static void for_each_class(const ConvShape& s, F&& f) {
  const int S = s.stride;
  const int PW = s.pad_w >= 0 ? s.pad_w : s.pad;  // horizontal padding
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
      f(c, (uint32_t)s.N * c.Hc * c.Wc);
    }
  }
}

static int resolve_dgrad_cfg(const ConvShape& s, int cfg, long K_class) {
  const bool ok = s.f32 ? tile_ok_for<float>(cfg) : tile_ok_for<__bf16>(cfg);
  return ok ? cfg : default_dgrad_cfg(s, K_class);
}

int conv_dgrad_tiles_m(const ConvShape& s, int cfg_in) {
  int total = 0;
  for_each_class(s, [&](const DgradClass& c, uint32_t M) {
    const int cfg = resolve_dgrad_cfg(s, cfg_in, (long)c.ntaps * s.Co);
    int bm = 128;
    auto f = [&](auto tile) { bm = decltype(tile)::BM; };
    if (s.f32) with_tile<float>(cfg, f);
    else with_tile<__bf16>(cfg, f);
    total += (int)cdiv(M, bm);
  });
  return total;
}

template <class T>
static void conv_dgrad_t(const void* dy, const void* w, void* dx, const ConvShape& s,
                         hipStream_t st, const DgradFusion* fz, int cfg_in) {
  const bool dense = is_dense(s);
  const bool aligned = s.Co % BK == 0;
  const T* dyp = (const T*)dy;
  const T* wp = (const T*)w;
  const int S = s.stride;
  FastDiv fCo((uint32_t)s.Co);
  int row0 = 0;  // deterministic mode: first partial row of this class
  for_each_class(s, [&](const DgradClass& c, uint32_t M) {
      EpiParams e{};
      e.C = dx; e.ldc = s.Ci; e.M = M; e.N = s.Ci;
      if (fz != nullptr) {
        e.addend = fz->addend;
        e.bnr_y = fz->bn_y;
        e.bnr_mean = fz->bn_mean; e.bnr_invstd = fz->bn_invstd;
        e.bnr_scale = fz->bn_scale; e.bnr_bias = fz->bn_bias; e.bnr_rep = fz->bn_rep; e.st_R = g_stat_rows;
        e.bnr_z = fz->bn_z;
        e.bnr_mask = fz->bn_mask;
        e.bnr_y2 = fz->bn_y2;
        e.bnr_mean2 = fz->bn_mean2;
        e.bnr_invstd2 = fz->bn_invstd2;
        e.det_rows = fz->det_rows;
        e.det_row0 = row0;
      }
      if (S > 1) {
        e.rm_s = S; e.rm_ph = c.ph; e.rm_pw = c.pw; e.rm_H = s.H; e.rm_W = s.W;
        e.rm_Hc = c.Hc; e.rm_Wc = c.Wc; e.rm_fHcWc = c.fHcWc; e.rm_fWc = c.fWc;
      }
      const int taps = s.KH * s.KW;
      const int cfg = resolve_dgrad_cfg(s, cfg_in, (long)c.ntaps * s.Co);
      with_tile<T>(cfg, [&](auto tile) {
        typedef decltype(tile) C;
        const uint32_t tN = cdiv(s.Ci, C::BN), tiles = cdiv(M, C::BM) * tN;
        row0 += (int)cdiv(M, C::BM);
        const dim3 grid(tiles), block(C::THREADS);
        if (e.bnr_y2 != nullptr) {  // two-branch block output (host checks: dense, bf16)
          if constexpr (std::is_same<T, __bf16>::value)
            hipLaunchKernelGGL((conv_dgrad_kernel<C, true, false, T, true>), grid, block, 0, st, dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
        } else if (dense)
          hipLaunchKernelGGL((conv_dgrad_kernel<C, true, false, T>), grid, block, 0, st, dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
        else if (aligned)
          hipLaunchKernelGGL((conv_dgrad_kernel<C, false, true, T>), grid, block, 0, st, dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
        else
          hipLaunchKernelGGL((conv_dgrad_kernel<C, false, false, T>), grid, block, 0, st, dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
      });
  });
}

void conv_dgrad(const void* dy, const void* w, void* dx, const ConvShape& s, hipStream_t st,
                const DgradFusion* fz, int cfg) {
  if (s.f32) conv_dgrad_t<float>(dy, w, dx, s, st, fz, cfg);
  else conv_dgrad_t<__bf16>(dy, w, dx, s, st, fz, cfg);
}

}  // namespace mipipe
