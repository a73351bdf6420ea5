// Direct-convolution and normalisation kernels for the rest of the torchvision model zoo
// (task.py:50-52 scans the whole registry for ``--arch``): grouped / depthwise convolutions
// (ResNeXt, MobileNetV2, MNASNet, ShuffleNetV2), non-square kernels and padding (Inception-v3),
// BatchNorm with any channel count and ReLU6 (ShuffleNetV2 x1.0 has 58-channel branches;
// MobileNetV2 clamps at 6), and k x k average pooling (DenseNet transitions, Inception pools).
//
// Design: these ops are memory / latency bound — a depthwise 3x3 conv does 9 MACs per loaded
// element, a 4-channel-per-group ResNeXt conv 36 — so they are direct NHWC kernels with the
// channel index fastest across the wavefront (every global access of a wave is one contiguous
// run of channels), fp32 accumulation, bf16 storage.  Depthwise convs with C % 8 == 0 (all of
// MobileNetV2 / MNASNet) take 8-channel 16-byte vector paths (cdna guide G13: hipcc does not
// vectorise scalar bf16 accesses).  Dense (groups = 1, C % 8 == 0, square) convs never come
// here: they run on the MFMA implicit-GEMM kernels of conv.hip.
//
// Weight layout matches conv.hip: [Co][KH][KW][Ci/groups] (the channels_last parameter); the
// vector depthwise kernels read a taps-major copy wt[KH*KW][C] made by the host binding.
#include "common.hpp"
#include "launchers.hpp"

namespace mipipe {

__device__ __forceinline__ float act_apply(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}

// derivative of the activation expressed through its OUTPUT z (relu: z > 0; relu6: 0 < z < 6)
__device__ __forceinline__ bool act_pass(float z, int act) {
  if (act == 1) return z > 0.f;
  if (act == 2) return z > 0.f && z < 6.f;
  return true;
}

static int grid_for(long work, int per_block = 256, int cap = 8192) {
  long g = (work + per_block - 1) / per_block;
  return (int)std::max<long>(1, std::min<long>(g, cap));
}

// ------------------------------------------------------------------------ grouped conv fwd
// One thread per output element, co fastest: a wave stores 64 consecutive channels of one
// pixel; the group's input channels are read as a contiguous run.
template <class T>
__global__ __launch_bounds__(256) void gconv_fwd_kernel(
    const T* __restrict__ x, const T* __restrict__ w, const float* __restrict__ bias,
    T* __restrict__ y, GConvShape s, int act) {
  const int Cig = s.Ci / s.groups, Cog = s.Co / s.groups;
  const long total = (long)s.N * s.Ho * s.Wo * s.Co;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int co = (int)(t % s.Co);
    const long pix = t / s.Co;
    const int wo = (int)(pix % s.Wo);
    const long r = pix / s.Wo;
    const int ho = (int)(r % s.Ho);
    const int n = (int)(r / s.Ho);
    const int ci0 = (co / Cog) * Cig;
    float acc = bias ? bias[co] : 0.f;
    for (int kh = 0; kh < s.KH; ++kh) {
      const int hi = ho * s.sh - s.ph + kh;
      if (hi < 0 || hi >= s.H) continue;
      for (int kw = 0; kw < s.KW; ++kw) {
        const int wi = wo * s.sw - s.pw + kw;
        if (wi < 0 || wi >= s.W) continue;
        const T* xp = x + (((long)n * s.H + hi) * s.W + wi) * s.Ci + ci0;
        const T* wp = w + (((long)co * s.KH + kh) * s.KW + kw) * Cig;
        for (int c = 0; c < Cig; ++c) acc += to_f32(xp[c]) * to_f32(wp[c]);
      }
    }
    y[t] = from_f32<T>(act_apply(acc, act));
  }
}

// ------------------------------------------------------------------------ grouped conv dgrad
// dx[n,hi,wi,ci] = sum over taps and the group's output channels; a gather (no atomics).
// ``z`` (optional): the conv's OUTPUT when an activation was fused in forward: dy is masked by
// act'(z) on the fly (the masked gradient is never materialised).
template <class T>
__global__ __launch_bounds__(256) void gconv_dgrad_kernel(
    const T* __restrict__ dy, const T* __restrict__ w, const T* __restrict__ z,
    T* __restrict__ dx, GConvShape s, int act) {
  const int Cig = s.Ci / s.groups, Cog = s.Co / s.groups;
  const long total = (long)s.N * s.H * s.W * s.Ci;
  const long wstride = (long)s.KH * s.KW * Cig;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int ci = (int)(t % s.Ci);
    const long pix = t / s.Ci;
    const int wi = (int)(pix % s.W);
    const long r = pix / s.W;
    const int hi = (int)(r % s.H);
    const int n = (int)(r / s.H);
    const int g = ci / Cig, cil = ci - g * Cig, co0 = g * Cog;
    float acc = 0.f;
    for (int kh = 0; kh < s.KH; ++kh) {
      const int hn = hi + s.ph - kh;
      if (hn < 0 || hn % s.sh) continue;
      const int ho = hn / s.sh;
      if (ho >= s.Ho) continue;
      for (int kw = 0; kw < s.KW; ++kw) {
        const int wn = wi + s.pw - kw;
        if (wn < 0 || wn % s.sw) continue;
        const int wo = wn / s.sw;
        if (wo >= s.Wo) continue;
        const long o = (((long)n * s.Ho + ho) * s.Wo + wo) * s.Co + co0;
        const T* wp = w + (((long)co0 * s.KH + kh) * s.KW + kw) * Cig + cil;
        for (int j = 0; j < Cog; ++j) {
          float gv = to_f32(dy[o + j]);
          if (z != nullptr && !act_pass(to_f32(z[o + j]), act)) gv = 0.f;
          acc += gv * to_f32(wp[j * wstride]);
        }
      }
    }
    dx[t] = from_f32<T>(acc);
  }
}

// ------------------------------------------------------------------------ grouped conv wgrad
// dw[co,kh,kw,cil] += sum over (n, ho, wo).  Thread e owns one weight element of tap
// blockIdx.z, ordered (co, cil) so a wave's dy / x loads are contiguous channel runs;
// blockIdx.y splits the (n, ho) rows and the partial sums land in dw with fp32 atomics
// (dw = zeroed buffer, or the parameter's slice of the flat gradient bucket).  Optional act/z
// mask as in dgrad; optional dbias (Σ masked dy per co, accumulated by the tap-0 threads).
template <class T>
__global__ __launch_bounds__(256) void gconv_wgrad_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ z,
    float* __restrict__ dw, float* __restrict__ dbias, GConvShape s, int act, int rows_per) {
  const int Cig = s.Ci / s.groups, Cog = s.Co / s.groups;
  const long nW = (long)s.Co * Cig;  // per tap
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int tap = blockIdx.z;
  if (e >= nW) return;
  const int kh = tap / s.KW, kw = tap - kh * s.KW;
  const int co = (int)(e / Cig), cil = (int)(e - (long)co * Cig);
  const int ci = (co / Cog) * Cig + cil;
  const long R = (long)s.N * s.Ho;
  const long r0 = (long)blockIdx.y * rows_per;
  const long r1 = r0 + rows_per < R ? r0 + rows_per : R;
  const bool do_bias = dbias != nullptr && tap == 0 && cil == 0;
  float acc = 0.f, accb = 0.f;
  for (long r = r0; r < r1; ++r) {
    const int ho = (int)(r % s.Ho);
    const int n = (int)(r / s.Ho);
    const int hi = ho * s.sh - s.ph + kh;
    const bool hok = hi >= 0 && hi < s.H;
    if (!hok && !do_bias) continue;
    const T* dyr = dy + r * s.Wo * s.Co + co;
    const T* zr = z ? z + r * s.Wo * s.Co + co : nullptr;
    const T* xr = x + ((long)n * s.H + (hok ? hi : 0)) * s.W * s.Ci + ci;
    for (int wo = 0; wo < s.Wo; ++wo) {
      float gv = to_f32(dyr[(long)wo * s.Co]);
      if (zr != nullptr && !act_pass(to_f32(zr[(long)wo * s.Co]), act)) gv = 0.f;
      accb += gv;
      const int wi = wo * s.sw - s.pw + kw;
      if (hok && wi >= 0 && wi < s.W) acc += gv * to_f32(xr[(long)wi * s.Ci]);
    }
  }
  atomicAdd(dw + (((long)co * s.KH + kh) * s.KW + kw) * Cig + cil, acc);
  if (do_bias) atomicAdd(dbias + co, accb);
}

// ------------------------------------------------------------------------ depthwise, C % 8 == 0
template <class T>
__device__ __forceinline__ void mask8(const T* z, int act, float* g) {
  float zv[8];
  load8(z, zv);
#pragma unroll
  for (int q = 0; q < 8; ++q)
    if (!act_pass(zv[q], act)) g[q] = 0.f;
}

// 8 channels of one output pixel per thread: per tap one 16-B activation load and one 16-B
// weight load (taps-major weights), 8 FMAs.
template <class T>
__global__ __launch_bounds__(256) void dwconv_fwd_v8_kernel(
    const T* __restrict__ x, const T* __restrict__ wt, const float* __restrict__ bias,
    T* __restrict__ y, GConvShape s, int act) {
  const int C = s.Co, cg = C / 8;
  const long total = (long)s.N * s.Ho * s.Wo * cg;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(t % cg);
    const long pix = t / cg;
    const int wo = (int)(pix % s.Wo);
    const long r = pix / s.Wo;
    const int ho = (int)(r % s.Ho);
    const int n = (int)(r / s.Ho);
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = bias ? bias[c8 * 8 + q] : 0.f;
    for (int kh = 0; kh < s.KH; ++kh) {
      const int hi = ho * s.sh - s.ph + kh;
      if (hi < 0 || hi >= s.H) continue;
      for (int kw = 0; kw < s.KW; ++kw) {
        const int wi = wo * s.sw - s.pw + kw;
        if (wi < 0 || wi >= s.W) continue;
        float xv[8], wv[8];
        load8(x + (((long)n * s.H + hi) * s.W + wi) * C + c8 * 8, xv);
        load8(wt + (long)(kh * s.KW + kw) * C + c8 * 8, wv);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += xv[q] * wv[q];
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = act_apply(acc[q], act);
    store8(y + pix * C + c8 * 8, acc);
  }
}

// 3x3 depthwise forward with every tap's loads issued unconditionally (clamped in-image
// coordinates, out-of-image taps zeroed by a select): the generic kernel's `continue` on the
// bounds made hipcc branch around each tap's loads and drain vmcnt(0) per tap.
template <class T>
__global__ __launch_bounds__(256) void dwconv3_fwd_v8_kernel(
    const T* __restrict__ x, const T* __restrict__ wt, const float* __restrict__ bias,
    T* __restrict__ y, GConvShape s, int act) {
  const int C = s.Co, cg = C / 8;
  const long total = (long)s.N * s.Ho * s.Wo * cg;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(t % cg);
    const long pix = t / cg;
    const int wo = (int)(pix % s.Wo);
    const long r = pix / s.Wo;
    const int ho = (int)(r % s.Ho);
    const int n = (int)(r / s.Ho);
    float xv[9][8];
    bool ok[9];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int hi = ho * s.sh - s.ph + kh, wi = wo * s.sw - s.pw + kw;
        ok[kh * 3 + kw] = (unsigned)hi < (unsigned)s.H && (unsigned)wi < (unsigned)s.W;
        const int hc = min(max(hi, 0), s.H - 1), wc = min(max(wi, 0), s.W - 1);
        load8(x + (((long)n * s.H + hc) * s.W + wc) * C + c8 * 8, xv[kh * 3 + kw]);
      }
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = bias ? bias[c8 * 8 + q] : 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      float wv[8];
      load8(wt + (long)k * C + c8 * 8, wv);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += ok[k] ? xv[k][q] * wv[q] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = act_apply(acc[q], act);
    store8(y + pix * C + c8 * 8, acc);
  }
}

template <class T>
__global__ __launch_bounds__(256) void dwconv_dgrad_v8_kernel(
    const T* __restrict__ dy, const T* __restrict__ wt, const T* __restrict__ z,
    T* __restrict__ dx, GConvShape s, int act) {
  const int C = s.Ci, cg = C / 8;
  const long total = (long)s.N * s.H * s.W * cg;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(t % cg);
    const long pix = t / cg;
    const int wi = (int)(pix % s.W);
    const long r = pix / s.W;
    const int hi = (int)(r % s.H);
    const int n = (int)(r / s.H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int kh = 0; kh < s.KH; ++kh) {
      const int hn = hi + s.ph - kh;
      if (hn < 0 || hn % s.sh) continue;
      const int ho = hn / s.sh;
      if (ho >= s.Ho) continue;
      for (int kw = 0; kw < s.KW; ++kw) {
        const int wn = wi + s.pw - kw;
        if (wn < 0 || wn % s.sw) continue;
        const int wo = wn / s.sw;
        if (wo >= s.Wo) continue;
        const long o = (((long)n * s.Ho + ho) * s.Wo + wo) * C + c8 * 8;
        float g[8], wv[8];
        load8(dy + o, g);
        if (z != nullptr) mask8(z + o, act, g);
        load8(wt + (long)(kh * s.KW + kw) * C + c8 * 8, wv);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += g[q] * wv[q];
      }
    }
    store8(dx + pix * C + c8 * 8, acc);
  }
}

// 256 threads = (lane row lr, channel group c8) pairs with lanes = 256 / (C/8) rows; the output
// positions of blockIdx.y's (n, ho) row range are strided over the lanes.  Per-block partials
// are reduced through LDS, then one fp32 atomic per weight element per block lands in dw
// ([C][KH][KW], the parameter layout).  blockIdx.z = tap; tap-0 blocks also reduce dbias.
template <class T>
__global__ __launch_bounds__(256) void dwconv_wgrad_v8_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ z,
    float* __restrict__ dw, float* __restrict__ dbias, GConvShape s, int act, int rows_per) {
  __shared__ float red[256 * 9];  // stride 9: conflict-free column reads
  const int C = s.Co, cg = C / 8;
  const int lanes = 256 / cg;
  const int tid = threadIdx.x;
  const int c8 = tid % cg, lr = tid / cg;
  const int tap = blockIdx.z, kh = tap / s.KW, kw = tap - kh * s.KW, taps = s.KH * s.KW;
  const bool do_bias = dbias != nullptr && tap == 0;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float accb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (lr < lanes) {
    const long R = (long)s.N * s.Ho;
    const long r0 = (long)blockIdx.y * rows_per;
    const long r1 = r0 + rows_per < R ? r0 + rows_per : R;
    for (long p = r0 * s.Wo + lr; p < r1 * s.Wo; p += lanes) {
      const int wo = (int)(p % s.Wo);
      const long r = p / s.Wo;
      const int ho = (int)(r % s.Ho), n = (int)(r / s.Ho);
      const int hi = ho * s.sh - s.ph + kh, wi = wo * s.sw - s.pw + kw;
      const bool ok = hi >= 0 && hi < s.H && wi >= 0 && wi < s.W;
      if (!ok && !do_bias) continue;
      float g[8];
      load8(dy + p * C + c8 * 8, g);
      if (z != nullptr) mask8(z + p * C + c8 * 8, act, g);
      if (do_bias) {
#pragma unroll
        for (int q = 0; q < 8; ++q) accb[q] += g[q];
      }
      if (ok) {
        float xv[8];
        load8(x + (((long)n * s.H + hi) * s.W + wi) * C + c8 * 8, xv);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += g[q] * xv[q];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) red[tid * 9 + q] = acc[q];
  __syncthreads();
  if (tid < cg) {
    float sum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int l = 0; l < lanes; ++l)
#pragma unroll
      for (int q = 0; q < 8; ++q) sum[q] += red[(l * cg + tid) * 9 + q];
#pragma unroll
    for (int q = 0; q < 8; ++q) atomicAdd(dw + (long)(tid * 8 + q) * taps + tap, sum[q]);
  }
  if (do_bias) {  // block-uniform branch
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) red[tid * 9 + q] = accb[q];
    __syncthreads();
    if (tid < cg) {
      float sum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int l = 0; l < lanes; ++l)
#pragma unroll
        for (int q = 0; q < 8; ++q) sum[q] += red[(l * cg + tid) * 9 + q];
#pragma unroll
      for (int q = 0; q < 8; ++q) atomicAdd(dbias + tid * 8 + q, sum[q]);
    }
  }
}

void gconv_fwd(const void* x, const void* w, const float* bias, void* y, const GConvShape& s,
               int act, hipStream_t st, bool f32) {
  auto run = [&](auto tag) {
    typedef decltype(tag) T;
    long work = (long)s.N * s.Ho * s.Wo * s.Co;
    hipLaunchKernelGGL((gconv_fwd_kernel<T>), dim3(grid_for(work)), dim3(256), 0, st, (const T*)x,
                       (const T*)w, bias, (T*)y, s, act);
  };
  if (f32) run(float{});
  else run(__bf16{});
}

void gconv_dgrad(const void* dy, const void* w, const void* z, void* dx, const GConvShape& s,
                 int act, hipStream_t st, bool f32) {
  auto run = [&](auto tag) {
    typedef decltype(tag) T;
    long work = (long)s.N * s.H * s.W * s.Ci;
    hipLaunchKernelGGL((gconv_dgrad_kernel<T>), dim3(grid_for(work)), dim3(256), 0, st,
                       (const T*)dy, (const T*)w, (const T*)z, (T*)dx, s, act);
  };
  if (f32) run(float{});
  else run(__bf16{});
}

void gconv_wgrad(const void* dy, const void* x, const void* z, float* dw, float* dbias,
                 const GConvShape& s, int act, hipStream_t st, bool f32) {
  auto run = [&](auto tag) {
    typedef decltype(tag) T;
    const long nW = (long)s.Co * (s.Ci / s.groups);
    const int bx = (int)((nW + 255) / 256);
    const int taps = s.KH * s.KW;
    const long R = (long)s.N * s.Ho;
    // ~2048 workgroups in total, every split at least 4 rows of (n, ho)
    long splits = std::max<long>(1, 2048 / std::max<long>(1, (long)bx * taps));
    splits = std::min<long>(splits, std::max<long>(1, R / 4));
    splits = std::min<long>(splits, 65535);
    const int rows_per = (int)((R + splits - 1) / splits);
    const int by = (int)((R + rows_per - 1) / rows_per);
    hipLaunchKernelGGL((gconv_wgrad_kernel<T>), dim3(bx, by, taps), dim3(256), 0, st, (const T*)dy,
                       (const T*)x, (const T*)z, dw, dbias, s, act, rows_per);
  };
  if (f32) run(float{});
  else run(__bf16{});
}

void dwconv_fwd(const void* x, const void* wt, const float* bias, void* y, const GConvShape& s,
                int act, hipStream_t st, bool f32) {
  auto run = [&](auto tag) {
    typedef decltype(tag) T;
    long work = (long)s.N * s.Ho * s.Wo * (s.Co / 8);
    if (s.KH == 3 && s.KW == 3)
      hipLaunchKernelGGL((dwconv3_fwd_v8_kernel<T>), dim3(grid_for(work)), dim3(256), 0, st,
                         (const T*)x, (const T*)wt, bias, (T*)y, s, act);
    else
      hipLaunchKernelGGL((dwconv_fwd_v8_kernel<T>), dim3(grid_for(work)), dim3(256), 0, st,
                         (const T*)x, (const T*)wt, bias, (T*)y, s, act);
  };
  if (f32) run(float{});
  else run(__bf16{});
}

void dwconv_dgrad(const void* dy, const void* wt, const void* z, void* dx, const GConvShape& s,
                  int act, hipStream_t st, bool f32) {
  auto run = [&](auto tag) {
    typedef decltype(tag) T;
    long work = (long)s.N * s.H * s.W * (s.Ci / 8);
    hipLaunchKernelGGL((dwconv_dgrad_v8_kernel<T>), dim3(grid_for(work)), dim3(256), 0, st,
                       (const T*)dy, (const T*)wt, (const T*)z, (T*)dx, s, act);
  };
  if (f32) run(float{});
  else run(__bf16{});
}

void dwconv_wgrad(const void* dy, const void* x, const void* z, float* dw, float* dbias,
                  const GConvShape& s, int act, hipStream_t st, bool f32) {
  auto run = [&](auto tag) {
    typedef decltype(tag) T;
    const int cg = s.Co / 8, lanes = 256 / cg, taps = s.KH * s.KW;
    const long P = (long)s.N * s.Ho * s.Wo;
    const long R = (long)s.N * s.Ho;
    // ~2048 workgroups, each lane covering >= 32 output positions
    long splits = std::max<long>(1, 2048 / taps);
    splits = std::min<long>(splits, std::max<long>(1, P / ((long)lanes * 32)));
    splits = std::min<long>(splits, std::min<long>(R, 65535));
    const int rows_per = (int)((R + splits - 1) / splits);
    const int by = (int)((R + rows_per - 1) / rows_per);
    hipLaunchKernelGGL((dwconv_wgrad_v8_kernel<T>), dim3(1, by, taps), dim3(256), 0, st,
                       (const T*)dy, (const T*)x, (const T*)z, dw, dbias, s, act,
                       rows_per);
  };
  if (f32) run(float{});
  else run(__bf16{});
}

// ------------------------------------------------------------------------ BatchNorm, any C
// Block = 64 channels (one per lane) x 4 waves over rows; per-block partials reduced in LDS
// and added to the [C] outputs with one atomic per channel per block.
template <class T>
__global__ __launch_bounds__(256) void chan_stats_kernel(const T* __restrict__ y,
                                                         const float* __restrict__ shift, long M,
                                                         int C, float* __restrict__ psum,
                                                         float* __restrict__ psq) {
  __shared__ float sh_s[4][64], sh_q[4][64];
  const int c = blockIdx.x * 64 + threadIdx.x;
  const int ty = threadIdx.y;
  float s = 0.f, q = 0.f;
  if (c < C) {
    const float sf = shift[c];
    for (long r = (long)blockIdx.y * 4 + ty; r < M; r += (long)gridDim.y * 4) {
      float d = to_f32(y[r * C + c]) - sf;
      s += d;
      q += d * d;
    }
  }
  sh_s[ty][threadIdx.x] = s;
  sh_q[ty][threadIdx.x] = q;
  __syncthreads();
  if (ty == 0 && c < C) {
    s = sh_s[0][threadIdx.x] + sh_s[1][threadIdx.x] + sh_s[2][threadIdx.x] + sh_s[3][threadIdx.x];
    q = sh_q[0][threadIdx.x] + sh_q[1][threadIdx.x] + sh_q[2][threadIdx.x] + sh_q[3][threadIdx.x];
    atomicAdd(psum + c, s);
    atomicAdd(psq + c, q);
  }
}

template <class T>
__global__ __launch_bounds__(256) void affine_act_kernel(const T* __restrict__ y,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ bias,
                                                         T* __restrict__ z, long n, int C,
                                                         int act) {
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    z[t] = from_f32<T>(act_apply(to_f32(y[t]) * scale[c] + bias[c], act));
  }
}

// Σg and Σg·x̂ with g = dz·act'(z), x̂ = (y - mean)·invstd
template <class T>
__global__ __launch_bounds__(256) void bn_generic_bwd_reduce_kernel(
    const T* __restrict__ dz, const T* __restrict__ z, const T* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, long M, int C, int act,
    float* __restrict__ out_g, float* __restrict__ out_gx) {
  __shared__ float sh_g[4][64], sh_x[4][64];
  const int c = blockIdx.x * 64 + threadIdx.x;
  const int ty = threadIdx.y;
  float sg = 0.f, sgx = 0.f;
  if (c < C) {
    const float mu = mean[c], is = invstd[c];
    for (long r = (long)blockIdx.y * 4 + ty; r < M; r += (long)gridDim.y * 4) {
      const long i = r * C + c;
      float g = to_f32(dz[i]);
      if (act != 0 && !act_pass(to_f32(z[i]), act)) g = 0.f;
      sg += g;
      sgx += g * (to_f32(y[i]) - mu) * is;
    }
  }
  sh_g[ty][threadIdx.x] = sg;
  sh_x[ty][threadIdx.x] = sgx;
  __syncthreads();
  if (ty == 0 && c < C) {
    sg = sh_g[0][threadIdx.x] + sh_g[1][threadIdx.x] + sh_g[2][threadIdx.x] + sh_g[3][threadIdx.x];
    sgx = sh_x[0][threadIdx.x] + sh_x[1][threadIdx.x] + sh_x[2][threadIdx.x] + sh_x[3][threadIdx.x];
    atomicAdd(out_g + c, sg);
    atomicAdd(out_gx + c, sgx);
  }
}

// dy = γ·invstd·(g - Σg/count - x̂·Σg·x̂/count); sum_g == nullptr: eval-mode BN, dy = γ·invstd·g
template <class T>
__global__ __launch_bounds__(256) void bn_generic_bwd_apply_kernel(
    const T* __restrict__ dz, const T* __restrict__ z, const T* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ sum_g,
    const float* __restrict__ sum_gx, float inv_count, long n, int C, int act,
    T* __restrict__ dy) {
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    float g = to_f32(dz[t]);
    if (act != 0 && !act_pass(to_f32(z[t]), act)) g = 0.f;
    const float is = invstd[c];
    float v = g;
    if (sum_g != nullptr) {
      const float xh = (to_f32(y[t]) - mean[c]) * is;
      v = g - sum_g[c] * inv_count - xh * sum_gx[c] * inv_count;
    }
    dy[t] = from_f32<T>(gamma[c] * is * v);
  }
}

// ---- 16-byte vector variants (C % 8 == 0, C <= 2048): a thread owns one 8-channel group and
// strides over rows (tpr = C/8 threads per row, rpb = 256/tpr rows per block pass), so the
// per-channel coefficients stay in registers; reductions go through LDS (stride 9: conflict-free
// column reads), then one atomic per channel per block.
// out: [R][C] replica rows (R = kStatReplicas); this block adds into row blockIdx % R, which
// spreads the per-channel atomics of many blocks over R addresses (finalize sums the rows)
__device__ __forceinline__ void lds_reduce_atomic8(float* sh, const float* v, int tpr, int rpb,
                                                   float* out) {
  out += (long)(blockIdx.x % kStatReplicas) * (tpr * 8);
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 8; ++k) sh[t * 9 + k] = v[k];
  __syncthreads();
  if (t < tpr) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int g = 0; g < rpb; ++g)
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += sh[(g * tpr + t) * 9 + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) atomicAdd(out + t * 8 + k, s[k]);
  }
  __syncthreads();
}

// v8 ("any C % 8") BN kernels: the statistics / backward reductions keep kV8RowU rows of loads
// in flight per thread over up to 1024 blocks whose per-channel atomics go to kStatReplicas
// replica rows (one [C] row took every block's atomics: on DenseNet's concatenated inputs that
// serialised the reductions at ~2 TB/s, and more blocks made it slower); the apply passes walk
// contiguous tiles of kV8ApplyU rows per thread with the loads issued first (as bn.hip's)
constexpr int kV8RowU = 4;
constexpr int kV8ApplyU = 2;

template <class T>
__global__ __launch_bounds__(256) void chan_stats_v8_kernel(const T* __restrict__ y,
                                                            const float* __restrict__ shift,
                                                            long M, int C,
                                                            float* __restrict__ psum,
                                                            float* __restrict__ psq) {
  __shared__ float sh[256 * 9];
  const int tpr = C / 8, rpb = 256 / tpr;
  const int t = threadIdx.x, cg = t % tpr, rg = t / tpr;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (rg < rpb) {
    float sf[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) sf[k] = shift[cg * 8 + k];
    const long stride = (long)gridDim.x * rpb;
    for (long r0 = (long)blockIdx.x * rpb + rg; r0 < M; r0 += kV8RowU * stride) {
      Raw8<T> raw[kV8RowU];  // kV8RowU rows of loads in flight per thread
#pragma unroll
      for (int u = 0; u < kV8RowU; ++u) raw[u] = ld_raw8(y + min(r0 + u * stride, M - 1) * C + cg * 8);
#pragma unroll
      for (int u = 0; u < kV8RowU; ++u) {
        if (r0 + u * stride >= M) break;
        float v[8];
        unpack_raw(raw[u], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float d = v[k] - sf[k];
          s[k] += d;
          q[k] += d * d;
        }
      }
    }
  }
  lds_reduce_atomic8(sh, s, tpr, rpb, psum);
  lds_reduce_atomic8(sh, q, tpr, rpb, psq);
}

template <class T>
__global__ __launch_bounds__(256) void affine_act_v8_kernel(const T* __restrict__ y,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ bias,
                                                            T* __restrict__ z, long M, int C,
                                                            int act) {
  const int tpr = C / 8, rpb = 256 / tpr;
  const int t = threadIdx.x, cg = t % tpr, rg = t / tpr;
  if (rg >= rpb) return;
  float sc[8], bi[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = scale[cg * 8 + k];
    bi[k] = bias[cg * 8 + k];
  }
  for (long r0 = (long)blockIdx.x * rpb * kV8ApplyU + rg; r0 < M;
       r0 += (long)gridDim.x * rpb * kV8ApplyU) {
    Raw8<T> raw[kV8ApplyU];  // a contiguous tile of kV8ApplyU*rpb rows per block iteration
#pragma unroll
    for (int u = 0; u < kV8ApplyU; ++u) raw[u] = ld_raw8(y + min(r0 + u * rpb, M - 1) * C + cg * 8);
#pragma unroll
    for (int u = 0; u < kV8ApplyU; ++u) {
      const long r = r0 + u * rpb;
      if (r >= M) break;
      float v[8];
      unpack_raw(raw[u], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = act_apply(v[k] * sc[k] + bi[k], act);
      store8(z + r * C + cg * 8, v);
    }
  }
}

template <class T>
__global__ __launch_bounds__(256) void bn_generic_bwd_reduce_v8_kernel(
    const T* __restrict__ dz, const T* __restrict__ z, const T* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, long M, int C, int act,
    float* __restrict__ out_g, float* __restrict__ out_gx) {
  __shared__ float sh[256 * 9];
  const int tpr = C / 8, rpb = 256 / tpr;
  const int t = threadIdx.x, cg = t % tpr, rg = t / tpr;
  float sg[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float sx[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (rg < rpb) {
    float mu[8], is[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      mu[k] = mean[cg * 8 + k];
      is[k] = invstd[cg * 8 + k];
    }
    const long stride = (long)gridDim.x * rpb;
    for (long r0 = (long)blockIdx.x * rpb + rg; r0 < M; r0 += kV8RowU * stride) {
      Raw8<T> rgv[kV8RowU], rz[kV8RowU], ry[kV8RowU];  // all loads of kV8RowU rows in flight
#pragma unroll
      for (int u = 0; u < kV8RowU; ++u) {
        const long off = min(r0 + u * stride, M - 1) * C + cg * 8;
        rgv[u] = ld_raw8(dz + off);
        if (act != 0) rz[u] = ld_raw8(z + off);
        ry[u] = ld_raw8(y + off);
      }
#pragma unroll
      for (int u = 0; u < kV8RowU; ++u) {
        if (r0 + u * stride >= M) break;
        float g[8], v[8];
        unpack_raw(rgv[u], g);
        if (act != 0) {
          float zv[8];
          unpack_raw(rz[u], zv);
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (!act_pass(zv[k], act)) g[k] = 0.f;
        }
        unpack_raw(ry[u], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          sg[k] += g[k];
          sx[k] += g[k] * (v[k] - mu[k]) * is[k];
        }
      }
    }
  }
  lds_reduce_atomic8(sh, sg, tpr, rpb, out_g);
  lds_reduce_atomic8(sh, sx, tpr, rpb, out_gx);
}

// dy = A·g + B + Cc·(y - mean) with A = γ·invstd, B = -A·Σg/n, Cc = -A·invstd·Σg·x̂/n
template <class T>
__global__ __launch_bounds__(256) void bn_generic_bwd_apply_v8_kernel(
    const T* __restrict__ dz, const T* __restrict__ z, const T* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ sum_g,
    const float* __restrict__ sum_gx, float inv_count, long M, int C, int act,
    T* __restrict__ dy) {
  const int tpr = C / 8, rpb = 256 / tpr;
  const int t = threadIdx.x, cg = t % tpr, rg = t / tpr;
  if (rg >= rpb) return;
  float A[8], B[8], Cc[8], mu[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = cg * 8 + k;
    A[k] = gamma[c] * invstd[c];
    B[k] = sum_g ? -A[k] * sum_g[c] * inv_count : 0.f;
    Cc[k] = sum_g ? -A[k] * invstd[c] * sum_gx[c] * inv_count : 0.f;
    mu[k] = mean[c];
  }
  for (long r0 = (long)blockIdx.x * rpb * kV8ApplyU + rg; r0 < M;
       r0 += (long)gridDim.x * rpb * kV8ApplyU) {
    Raw8<T> rgv[kV8ApplyU], rz[kV8ApplyU], ry[kV8ApplyU];
#pragma unroll
    for (int u = 0; u < kV8ApplyU; ++u) {
      const long off = min(r0 + u * rpb, M - 1) * C + cg * 8;
      rgv[u] = ld_raw8(dz + off);
      if (act != 0) rz[u] = ld_raw8(z + off);
      ry[u] = ld_raw8(y + off);
    }
#pragma unroll
    for (int u = 0; u < kV8ApplyU; ++u) {
      const long r = r0 + u * rpb;
      if (r >= M) break;
      float g[8], v[8];
      unpack_raw(rgv[u], g);
      if (act != 0) {
        float zv[8];
        unpack_raw(rz[u], zv);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (!act_pass(zv[k], act)) g[k] = 0.f;
      }
      unpack_raw(ry[u], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = A[k] * g[k] + B[k] + Cc[k] * (v[k] - mu[k]);
      store8(dy + r * C + cg * 8, g);
    }
  }
}

static bool bn_v8(int C) { return C % 8 == 0 && C <= 2048; }

static int v8_grid(long M, int C, int cap) {
  const int rpb = 256 / (C / 8);
  long g = (M + rpb - 1) / rpb;
  return (int)std::max<long>(1, std::min<long>(g, cap));
}

// blocks for the apply passes: a block iteration covers kV8ApplyU * rpb rows
static int v8_tiles(long M, int C, int U, int cap) {
  const long rows = (long)(256 / (C / 8)) * U;
  return (int)std::max<long>(1, std::min<long>((M + rows - 1) / rows, cap));
}

static dim3 chan_grid(long M, int C) {
  const int bx = (C + 63) / 64;
  long by = std::max<long>(1, std::min<long>((M + 63) / 64, std::max(1, 2048 / bx)));
  return dim3(bx, (unsigned)by);
}

void chan_stats(const void* y, const float* shift, long M, int C, float* psum, float* psq,
                hipStream_t st, bool f32) {
  auto run = [&](auto tag) {
    typedef decltype(tag) T;
    if (bn_v8(C)) {
      hipLaunchKernelGGL((chan_stats_v8_kernel<T>), dim3(v8_grid(M, C, 1024)), dim3(256), 0, st,
                         (const T*)y, shift, M, C, psum, psq);
      return;
    }
    hipLaunchKernelGGL((chan_stats_kernel<T>), chan_grid(M, C), dim3(64, 4), 0, st, (const T*)y,
                       shift, M, C, psum, psq);
  };
  if (f32) run(float{});
  else run(__bf16{});
}

void affine_act(const void* y, const float* scale, const float* bias, void* z, long M, int C,
                int act, hipStream_t st, bool f32) {
  auto run = [&](auto tag) {
    typedef decltype(tag) T;
    if (bn_v8(C)) {
      hipLaunchKernelGGL((affine_act_v8_kernel<T>), dim3(v8_tiles(M, C, kV8ApplyU, 4096)), dim3(256), 0, st,
                         (const T*)y, scale, bias, (T*)z, M, C, act);
      return;
    }
    long n = M * C;
    hipLaunchKernelGGL((affine_act_kernel<T>), dim3(grid_for(n)), dim3(256), 0, st, (const T*)y,
                       scale, bias, (T*)z, n, C, act);
  };
  if (f32) run(float{});
  else run(__bf16{});
}

void bn_generic_bwd_reduce(const void* dz, const void* z, const void* y, const float* mean,
                           const float* invstd, long M, int C, int act, float* out_g,
                           float* out_gx, hipStream_t st, bool f32) {
  auto run = [&](auto tag) {
    typedef decltype(tag) T;
    if (bn_v8(C)) {
      hipLaunchKernelGGL((bn_generic_bwd_reduce_v8_kernel<T>), dim3(v8_grid(M, C, 1024)), dim3(256), 0,
                         st, (const T*)dz, (const T*)z, (const T*)y, mean, invstd, M,
                         C, act, out_g, out_gx);
      return;
    }
    hipLaunchKernelGGL((bn_generic_bwd_reduce_kernel<T>), chan_grid(M, C), dim3(64, 4), 0, st,
                       (const T*)dz, (const T*)z, (const T*)y, mean, invstd, M, C,
                       act, out_g, out_gx);
  };
  if (f32) run(float{});
  else run(__bf16{});
}

void bn_generic_bwd_apply(const void* dz, const void* z, const void* y, const float* mean,
                          const float* invstd, const float* gamma, const float* sum_g,
                          const float* sum_gx, long count, long M, int C, int act, void* dy,
                          hipStream_t st, bool f32) {
  auto run = [&](auto tag) {
    typedef decltype(tag) T;
    if (bn_v8(C)) {
      hipLaunchKernelGGL((bn_generic_bwd_apply_v8_kernel<T>), dim3(v8_tiles(M, C, kV8ApplyU, 4096)), dim3(256), 0,
                         st, (const T*)dz, (const T*)z, (const T*)y, mean, invstd,
                         gamma, sum_g, sum_gx, 1.f / (float)count, M, C, act, (T*)dy);
      return;
    }
    long n = M * C;
    hipLaunchKernelGGL((bn_generic_bwd_apply_kernel<T>), dim3(grid_for(n)), dim3(256), 0, st,
                       (const T*)dz, (const T*)z, (const T*)y, mean, invstd, gamma,
                       sum_g, sum_gx, 1.f / (float)count, n, C, act, (T*)dy);
  };
  if (f32) run(float{});
  else run(__bf16{});
}

// ------------------------------------------------------------------------ k x k average pool
// count_include_pad = True (torch's default, the only mode torchvision uses); any C.
template <class T>
__global__ __launch_bounds__(256) void avgpool2d_fwd_kernel(const T* __restrict__ x,
                                                            T* __restrict__ y, int N, int H,
                                                            int W, int C, int Ho, int Wo, int k,
                                                            int s, int p) {
  const long total = (long)N * Ho * Wo * C;
  const float inv = 1.f / (float)(k * k);
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    const long pix = t / C;
    const int wo = (int)(pix % Wo);
    const long r = pix / Wo;
    const int ho = (int)(r % Ho);
    const int n = (int)(r / Ho);
    float acc = 0.f;
    for (int kh = 0; kh < k; ++kh) {
      const int hi = ho * s - p + kh;
      if (hi < 0 || hi >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int wi = wo * s - p + kw;
        if (wi < 0 || wi >= W) continue;
        acc += to_f32(x[(((long)n * H + hi) * W + wi) * C + c]);
      }
    }
    y[t] = from_f32<T>(acc * inv);
  }
}

template <class T>
__global__ __launch_bounds__(256) void avgpool2d_bwd_kernel(const T* __restrict__ dy,
                                                            T* __restrict__ dx, int N, int H,
                                                            int W, int C, int Ho, int Wo, int k,
                                                            int s, int p) {
  const long total = (long)N * H * W * C;
  const float inv = 1.f / (float)(k * k);
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    const long pix = t / C;
    const int wi = (int)(pix % W);
    const long r = pix / W;
    const int hi = (int)(r % H);
    const int n = (int)(r / H);
    const int ho_lo = max(0, (hi + p - k + s) / s), ho_hi = min(Ho - 1, (hi + p) / s);
    const int wo_lo = max(0, (wi + p - k + s) / s), wo_hi = min(Wo - 1, (wi + p) / s);
    float acc = 0.f;
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      const int kh = hi - (ho * s - p);
      if (kh < 0 || kh >= k) continue;
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const int kw = wi - (wo * s - p);
        if (kw < 0 || kw >= k) continue;
        acc += to_f32(dy[(((long)n * Ho + ho) * Wo + wo) * C + c]);
      }
    }
    dx[t] = from_f32<T>(acc * inv);
  }
}

void avgpool2d_fwd(const void* x, void* y, int N, int H, int W, int C, int Ho, int Wo, int k,
                   int stride, int pad, hipStream_t st, bool f32) {
  auto run = [&](auto tag) {
    typedef decltype(tag) T;
    hipLaunchKernelGGL((avgpool2d_fwd_kernel<T>), dim3(grid_for((long)N * Ho * Wo * C)), dim3(256), 0,
                       st, (const T*)x, (T*)y, N, H, W, C, Ho, Wo, k, stride, pad);
  };
  if (f32) run(float{});
  else run(__bf16{});
}

void avgpool2d_bwd(const void* dy, void* dx, int N, int H, int W, int C, int Ho, int Wo, int k,
                   int stride, int pad, hipStream_t st, bool f32) {
  auto run = [&](auto tag) {
    typedef decltype(tag) T;
    hipLaunchKernelGGL((avgpool2d_bwd_kernel<T>), dim3(grid_for((long)N * H * W * C)), dim3(256), 0, st,
                       (const T*)dy, (T*)dx, N, H, W, C, Ho, Wo, k, stride, pad);
  };
  if (f32) run(float{});
  else run(__bf16{});
}

}  // namespace mipipe
