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

// ----------------------------------------------------------------------------------------
// Stride-1 data-grads as forward convolutions.  With stride 1 there is a single parity class
// and dx = conv(dy, flip(W)ᵀ, pad = K-1-pad): the forward kernel's im2col A operand (dy rows
// gathered per tap, K-contiguous) and its K-contiguous weight operand replace the data-grad
// gather and the N-contiguous (transposed-read) weight operand.  Measured per shape by the tile
// tuner on the ResNet-50 b256 3x3 layers (tools/r2/tune_dump.py): the dgrad main loop ran at
// 15-23 % of the dense bf16 peak where the forward loop runs at 26-35 %.
bool conv_dgrad_fwd_style(const ConvShape& s) {
  const bool s1 = s.stride == 1 && (s.stride_w == 0 || s.stride_w == 1);
  return s1 && !is_dense(s);
}

template <class T>
__global__ __launch_bounds__(256) void conv_weight_flip_kernel(const T* __restrict__ w,
                                                               T* __restrict__ wt, int Co, int KH,
                                                               int KW, int Ci) {
  // wt[ci][kh][kw][co] = w[co][KH-1-kh][KW-1-kw][ci]; one thread per output element
  const long total = (long)Co * KH * KW * Ci;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int co = (int)(i % Co);
    long r = i / Co;
    const int kw = (int)(r % KW);
    r /= KW;
    const int kh = (int)(r % KH);
    const int ci = (int)(r / KH);
    wt[i] = w[(((long)co * KH + (KH - 1 - kh)) * KW + (KW - 1 - kw)) * Ci + ci];
  }
}

void conv_weight_flip(const void* w, void* wt, int Co, int KH, int KW, int Ci, bool f32,
                      hipStream_t st) {
  const long total = (long)Co * KH * KW * Ci;
  const int grid = (int)std::min<long>((total + 255) / 256, 2048);
  if (f32)
    hipLaunchKernelGGL((conv_weight_flip_kernel<float>), dim3(grid), dim3(256), 0, st,
                       (const float*)w, (float*)wt, Co, KH, KW, Ci);
  else
    hipLaunchKernelGGL((conv_weight_flip_kernel<__bf16>), dim3(grid), dim3(256), 0, st,
                       (const __bf16*)w, (__bf16*)wt, Co, KH, KW, Ci);
}

template <class T>
static void conv_dgrad_fwd_t(const void* dy, const void* wflip, void* dx, const ConvShape& s,
                             hipStream_t st, const DgradFusion* fz, int cfg_in) {
  ConvShape s2 = s;  // the forward convolution dy -> dx
  s2.H = s.Ho; s2.W = s.Wo; s2.Ci = s.Co; s2.Co = s.Ci;
  s2.Ho = s.H; s2.Wo = s.W;
  s2.stride = 1; s2.stride_w = 0;
  s2.pad = s.KH - 1 - s.pad;
  s2.pad_w = s.KW - 1 - (s.pad_w >= 0 ? s.pad_w : s.pad);
  const ConvGeom g = make_geom(s2);
  const uint32_t M = (uint32_t)s.N * s.H * s.W;
  EpiParams e{};
  e.C = dx; e.ldc = s.Ci; e.M = M; e.N = s.Ci;
  if (fz != nullptr) {
    e.addend = fz->addend;
    e.bnr_y = fz->bn_y;
    e.bnr_mean = fz->bn_mean; e.bnr_invstd = fz->bn_invstd;
    e.bnr_scale = fz->bn_scale; e.bnr_bias = fz->bn_bias; e.bnr_rep = fz->bn_rep; e.st_R = g_stat_rows;
    e.bnr_z = fz->bn_z;
    e.bnr_mask = fz->bn_mask;
    e.det_rows = fz->det_rows;
    e.det_row0 = 0;
  }
  const bool aligned = s.Co % BK == 0;
  const T* dyp = (const T*)dy;
  const T* wp = (const T*)wflip;
  const int cfg = resolve_dgrad_cfg(s, cfg_in, (long)s.KH * s.KW * s.Co);
  with_tile<T>(cfg, [&](auto tile) {
    typedef decltype(tile) C;
    const uint32_t tN = cdiv(s.Ci, C::BN), tiles = cdiv(M, C::BM) * tN;
    const dim3 grid(tiles), block(C::THREADS);
    if (aligned)
      hipLaunchKernelGGL((conv_fwd_kernel<C, false, true, T, true>), grid, block, 0, st, dyp, wp, g, M, tN, e);
    else
      hipLaunchKernelGGL((conv_fwd_kernel<C, false, false, T, true>), grid, block, 0, st, dyp, wp, g, M, tN, e);
  });
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
                const DgradFusion* fz, int cfg, const void* w_flip) {
  if (w_flip != nullptr && conv_dgrad_fwd_style(s) && (fz == nullptr || fz->bn_y2 == nullptr)) {
    if (s.f32) conv_dgrad_fwd_t<float>(dy, w_flip, dx, s, st, fz, cfg);
    else conv_dgrad_fwd_t<__bf16>(dy, w_flip, dx, s, st, fz, cfg);
    return;
  }
  if (s.f32) conv_dgrad_t<float>(dy, w, dx, s, st, fz, cfg);
  else conv_dgrad_t<__bf16>(dy, w, dx, s, st, fz, cfg);
}

}  // namespace mipipe
