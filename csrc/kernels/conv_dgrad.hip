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
  cfg = conv_plan_tile(cfg);
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
// Data-grads as forward convolutions.  A stride-S data-grad splits into S² parity classes; the
// class (ph, pw) is a STRIDE-1 convolution of dy with the taps kh = kh0 + S·a, kw = kw0 + S·b,
// flipped: dx[S·i+ph][S·j+pw] = Σ_{a',b'} dy[i - pad_h + a'][j - pad_w + b'] · W'[a'][b'] with
// W'[ci][a'][b'][co] = W[co][kh0 + S(nkh-1-a')][kw0 + S(nkw-1-b')][ci] and pad = nk-1-d0.  The
// forward kernel's im2col A operand (dy rows gathered per tap, K-contiguous) and K-contiguous
// weight operand then replace the data-grad gather and its N-contiguous (transposed-read)
// weight operand; the epilogue (row remap of the class, BN-backward fusions) is unchanged.
// Measured per shape by the tile tuner on the ResNet-50 b256 3x3 layers (tools/r2/tune_dump.py):
// the dgrad main loop ran at 15-23 % of the dense bf16 peak where the forward loop runs at
// 26-35 %; switching the stride-1 3x3s: 10.84k -> 11.24k img/s.
bool conv_dgrad_fwd_style(const ConvShape& s, bool dense_too) {
  const bool sq = s.stride_w == 0 || s.stride_w == s.stride;
  return sq && (dense_too || !is_dense(s));
}

int dgrad_fwd_style_mode() {
  static const int mode = [] {
    const char* v = getenv("MIPIPE_DGRAD_FWD");
    return v == nullptr ? 1 : atoi(v);
  }();
  return mode;
}

// workspace of a split plan: the largest forward-style class's splits x rows x Ci (classes run
// one after another on the stream and reuse it)
long conv_dgrad_split_ws_elems(const ConvShape& s, int cfg) {
  if (conv_plan_splits(cfg) <= 1 || dgrad_fwd_style_mode() <= 0 ||
      !conv_dgrad_fwd_style(s, dgrad_fwd_style_mode() >= 2))
    return 0;
  long need = 0;
  for_each_class(s, [&](const DgradClass& c, uint32_t M) {
    if (c.ntaps <= 0) return;
    const int nk = (int)cdiv((uint64_t)c.ntaps * s.Co, BK);
    int S, kps;
    conv_split_geometry(nk, conv_plan_splits(cfg), &S, &kps);
    if (S > 1) need = std::max(need, (long)S * M * s.Ci);
  });
  return need;
}

bool dgrad_preflip_ok(const ConvShape& s) {
  const int mode = dgrad_fwd_style_mode();
  return mode > 0 && s.stride <= 2 && s.KH * s.KW > 1 && conv_dgrad_fwd_style(s, mode >= 2);
}

void dgrad_flip_plan(const ConvShape& s, FlipPlan& p) {
  p = FlipPlan{};
  p.S = s.stride;
  long off = 0;
  const uint32_t tiles = cdiv(s.Ci, 64) * cdiv(s.Co, 64);
  for_each_class(s, [&](const DgradClass& c, uint32_t) {
    if (c.ntaps <= 0 || p.ncls >= 4) return;
    const int nkh = c.kh0 < s.KH ? (s.KH - c.kh0 + c.S - 1) / c.S : 0;
    FlipClass& f = p.cls[p.ncls++];
    f.kh0 = c.kh0; f.kw0 = c.kw0; f.nkh = nkh; f.nkw = c.nkw;
    f.off = off;
    f.b0 = p.nblk;
    off += (long)s.Ci * c.ntaps * s.Co;  // conv_dgrad_t's flip_off progression
    p.nblk += tiles * (uint32_t)(nkh * c.nkw);
  });
}

// Tap-flipped sub-kernel as 64x64 LDS-tiled transposes, one per tap: wt[ci][a][b][co] =
// w[co][kh0 + S(nkh-1-a)][kw0 + S(nkw-1-b)][ci].  Reads run along ci and writes along co (both
// coalesced; the one-thread-per-element gather it replaces cost ~7 us per call).
template <class T>
__global__ __launch_bounds__(256) void conv_weight_flip_kernel(const T* __restrict__ w,
                                                               T* __restrict__ wt, int Co, int KH,
                                                               int KW, int Ci, int kh0, int kw0,
                                                               int S, int nkh, int nkw) {
  __shared__ T tile[64][65];
  const int ci0 = blockIdx.x * 64, co0 = blockIdx.y * 64, tap = blockIdx.z;
  const int a = tap / nkw, b = tap % nkw;
  const int kh = kh0 + S * (nkh - 1 - a), kw = kw0 + S * (nkw - 1 - b);
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  // all 16 loads in flight at once: a launch this small is one memory latency, not sixteen
  T v[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int co = co0 + ty + 4 * u, ci = ci0 + tx;
    v[u] = (co < Co && ci < Ci) ? w[(((long)co * KH + kh) * KW + kw) * Ci + ci] : T(0.f);
  }
#pragma unroll
  for (int u = 0; u < 16; ++u) tile[ty + 4 * u][tx] = v[u];
  __syncthreads();
  const long taps = (long)nkh * nkw;
#pragma unroll
  for (int r = ty; r < 64; r += 4) {
    const int ci = ci0 + r, co = co0 + tx;
    if (co < Co && ci < Ci) wt[((long)ci * taps + tap) * Co + co] = tile[tx][r];
  }
}

template <class T>
static void weight_flip(const T* w, T* wt, const ConvShape& s, const DgradClass& c, int nkh,
                        hipStream_t st) {
  const dim3 grid((s.Ci + 63) / 64, (s.Co + 63) / 64, nkh * c.nkw);
  hipLaunchKernelGGL((conv_weight_flip_kernel<T>), grid, dim3(256), 0, st, w, wt, s.Co, s.KH,
                     s.KW, s.Ci, c.kh0, c.kw0, c.S, nkh, c.nkw);
}

template <class T>
static void conv_dgrad_t(const void* dy, const void* w, void* dx, const ConvShape& s,
                         hipStream_t st, const DgradFusion* fz, int cfg_in, void* wflip,
                         bool preflipped, float* split_ws) {
  const bool dense = is_dense(s);
  long flip_off = 0;  // this class's slice of the flipped-weight workspace
  const bool aligned = s.Co % BK == 0;
  const T* dyp = (const T*)dy;
  const T* wp = (const T*)w;
  const int S = s.stride;
  FastDiv fCo((uint32_t)s.Co);
  int row0 = 0;  // deterministic mode: first partial row of this class
  for_each_class(s, [&](const DgradClass& c, uint32_t M) {
      EpiParams e{};
      e.C = dx; e.ldc = s.Ci; e.M = M; e.N = s.Ci;
      e.nt = ((g_nt_store >> 1) & 1) &&
             (long)s.N * s.H * s.W * s.Ci * (s.f32 ? 4 : 2) > g_nt_min_bytes;
      e.ntl = (g_nt_store >> 8) & 1;
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
      const int nkh = c.kh0 < s.KH ? (s.KH - c.kh0 + S - 1) / S : 0;
      if (wflip != nullptr && c.ntaps > 0 && e.bnr_y2 == nullptr) {
        // this class as a stride-1 forward convolution of dy (see conv_dgrad_fwd_style)
        T* wt = (T*)wflip + flip_off;
        flip_off += (long)s.Ci * c.ntaps * s.Co;
        // preflipped: the forward launch wrote it (conv_fwd's trailing blocks, dgrad_flip_plan)
        if (!preflipped) weight_flip<T>(wp, wt, s, c, nkh, st);
        ConvShape s2 = s;
        s2.H = s.Ho; s2.W = s.Wo; s2.Ci = s.Co; s2.Co = s.Ci;
        s2.Ho = c.Hc; s2.Wo = c.Wc;
        s2.KH = nkh; s2.KW = c.nkw;
        s2.stride = 1; s2.stride_w = 0;
        s2.pad = nkh - 1 - c.dh0;
        s2.pad_w = c.nkw - 1 - c.dw0;
        const ConvGeom g2 = make_geom(s2);
        const bool dense2 = dense && S == 1;
        int SK = 1, kps = 0;
        conv_split_geometry((int)cdiv((uint64_t)c.ntaps * s.Co, BK),
                            split_ws != nullptr ? conv_plan_splits(cfg_in) : 1, &SK, &kps);
        with_tile<T>(cfg, [&](auto tile) {
          typedef decltype(tile) C;
          const uint32_t tN = cdiv(s.Ci, C::BN), tiles = cdiv(M, C::BM) * tN;
          row0 += (int)cdiv(M, C::BM);
          const dim3 grid(tiles), block(C::THREADS);
          constexpr bool kSplitOk = !(C::BM == 256 && C::BN == 256 && !C::PP);  // (see conv_fwd)
          if constexpr (kSplitOk) if (SK > 1) {  // split-K plan (see conv_fwd): partial tiles, then the finish launch
            EpiParams es = e;
            es.split_kt = kps;
            es.split_ws = split_ws;
            const dim3 g2d(tiles, SK);
            if (dense2)
              hipLaunchKernelGGL((conv_fwd_kernel<C, true, false, T, true, true>), g2d, block, 0, st, dyp, wt, g2, M, tN, es);
            else if (aligned && (s.f32 || nkh * c.nkw <= 32))
              hipLaunchKernelGGL((conv_fwd_kernel<C, false, true, T, true, true>), g2d, block, 0, st, dyp, wt, g2, M, tN, es);
            else
              hipLaunchKernelGGL((conv_fwd_kernel<C, false, false, T, true, true>), g2d, block, 0, st, dyp, wt, g2, M, tN, es);
            hipLaunchKernelGGL((conv_splitk_finish_kernel<C, T, true>), dim3(tiles), block, 0, st,
                               (const float*)split_ws, SK, tN, e);
            return;
          }
          if (dense2)
            hipLaunchKernelGGL((conv_fwd_kernel<C, true, false, T, true>), grid, block, 0, st, dyp, wt, g2, M, tN, e);
          else if (aligned && (s.f32 || nkh * c.nkw <= 32))  // bf16: buffer im2col tap mask
            hipLaunchKernelGGL((conv_fwd_kernel<C, false, true, T, true>), grid, block, 0, st, dyp, wt, g2, M, tN, e);
          else
            hipLaunchKernelGGL((conv_fwd_kernel<C, false, false, T, true>), grid, block, 0, st, dyp, wt, g2, M, tN, e);
        });
        return;
      }
      with_tile<T>(cfg, [&](auto tile) {
        typedef decltype(tile) C;
        const uint32_t tN = cdiv(s.Ci, C::BN), tiles = cdiv(M, C::BM) * tN;
        row0 += (int)cdiv(M, C::BM);
        const dim3 grid(tiles), block(C::THREADS);
        if (e.bnr_y2 != nullptr) {
  // two-branch block output (host checks: dense, bf16)
          if constexpr (std::is_same<T, __bf16>::value)
            hipLaunchKernelGGL((conv_dgrad_kernel<C, true, false, T, true>), grid, block, 0, st, dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
        } else if (dense)
          hipLaunchKernelGGL((conv_dgrad_kernel<C, true, false, T>), grid, block, 0, st, dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
        else if (aligned && (s.f32 || c.ntaps <= 32))  // bf16: buffer operands' tap mask
          hipLaunchKernelGGL((conv_dgrad_kernel<C, false, true, T>), grid, block, 0, st, dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
        else
          hipLaunchKernelGGL((conv_dgrad_kernel<C, false, false, T>), grid, block, 0, st, dyp, wp, s.Ho, s.Wo, s.Co, taps, fCo, c, M, tN, e);
      });
  });
}

void conv_dgrad(const void* dy, const void* w, void* dx, const ConvShape& s, hipStream_t st,
                const DgradFusion* fz, int cfg, void* w_flip, bool preflipped, float* split_ws) {
  preflipped = preflipped && w_flip != nullptr && dgrad_preflip_ok(s);
  if (s.f32) conv_dgrad_t<float>(dy, w, dx, s, st, fz, cfg, w_flip, preflipped, split_ws);
  else conv_dgrad_t<__bf16>(dy, w, dx, s, st, fz, cfg, w_flip, preflipped, split_ws);
}

}  // namespace mipipe
