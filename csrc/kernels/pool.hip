// NHWC pooling: max-pool with 1-byte window-argmax (fwd/bwd) and global average pool.
// Backward max-pool is a gather over the windows covering each input pixel (deterministic,
// no atomics).  Each thread moves 8 channels (one 16-B bf16 vector or two fp32 vectors).
#include <stdexcept>

#include "common.hpp"
#include "launchers.hpp"

namespace mipipe {

template <class T>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const T* __restrict__ x,
                                                          T* __restrict__ y,
                                                          uint8_t* __restrict__ idx, int N, int H,
                                                          int W, int C, int Ho, int Wo, int k,
                                                          int s, int p) {
  const int cg = C / 8;
  long total = (long)N * Ho * Wo * cg;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    int c8 = (int)(t % cg);
    long pix = t / cg;
    int wo = (int)(pix % Wo);
    long r = pix / Wo;
    int ho = (int)(r % Ho);
    int n = (int)(r / Ho);
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      best[q] = -INFINITY;
      arg[q] = 0;
    }
    for (int kh = 0; kh < k; ++kh) {
      int hi = ho * s - p + kh;
      if (hi < 0 || hi >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        int wi = wo * s - p + kw;
        if (wi < 0 || wi >= W) continue;
        float v[8];
        load8(x + (((long)n * H + hi) * W + wi) * C + c8 * 8, v);
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (v[q] > best[q] || (v[q] != v[q])) {  // NaN propagates like torch
            best[q] = v[q];
            arg[q] = (uint8_t)(kh * k + kw);
          }
      }
    }
    long o = pix * C + c8 * 8;
    store8(y + o, best);
    uint2 a;
    a.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | ((uint32_t)arg[3] << 24);
    a.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | ((uint32_t)arg[7] << 24);
    *reinterpret_cast<uint2*>(idx + o) = a;
  }
}

template <class T>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const T* __restrict__ dy,
                                                          const uint8_t* __restrict__ idx,
                                                          T* __restrict__ dx, int N, int H,
                                                          int W, int C, int Ho, int Wo, int k,
                                                          int s, int p) {
  const int cg = C / 8;
  long total = (long)N * H * W * cg;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    int c8 = (int)(t % cg);
    long pix = t / cg;
    int wi = (int)(pix % W);
    long r = pix / W;
    int hi = (int)(r % H);
    int n = (int)(r / H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // output windows containing (hi, wi): ho*s - p <= hi <= ho*s - p + k - 1
    int ho_lo = max(0, (hi + p - k + s) / s);
    int ho_hi = min(Ho - 1, (hi + p) / s);
    int wo_lo = max(0, (wi + p - k + s) / s);
    int wo_hi = min(Wo - 1, (wi + p) / s);
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      int kh = hi - (ho * s - p);
      if (kh < 0 || kh >= k) continue;
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        int kw = wi - (wo * s - p);
        if (kw < 0 || kw >= k) continue;
        uint8_t want = (uint8_t)(kh * k + kw);
        long o = (((long)n * Ho + ho) * Wo + wo) * C + c8 * 8;
        uint2 a = *reinterpret_cast<const uint2*>(idx + o);
        float g[8];
        load8(dy + o, g);
        uint32_t w0 = a.x, w1 = a.y;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          uint32_t word = q < 4 ? w0 : w1;
          uint8_t ai = (uint8_t)(word >> ((q & 3) * 8));
          if (ai == want) acc[q] += g[q];
        }
      }
    }
    store8(dx + pix * C + c8 * 8, acc);
  }
}

// ---------------------------------------------------------------------------------------------
// Stem block fusion: BatchNorm-apply + ReLU + 3x3/2 max-pool in one pass over the conv output y
// (the normalised activation z = relu(y*scale + bias) is never stored: -411 MB written and read
// again per ResNet-50 b256 step), and its backward as two gathers over the pooling windows:
//   g(pixel) = sum of dp over the windows whose argmax is that pixel and whose output p > 0
//   (p > 0  <=>  the ReLU was active at the argmax: p is the max of relu(.)),
// reduce: Σg, Σg·x̂ -> replica slab (then bn_bwd_collect);  apply: dy = A·g + B·y + C.
// Each thread owns one 8-channel group: the host guarantees 256 % (C/8) == 0 and grid strides
// that are multiples of 256, so a thread's channel group is threadIdx.x % (C/8) throughout.
template <int KS, class T>  // KS > 0: compile-time window size (all KS*KS loads issued at once)
__global__ __launch_bounds__(256) void pool_bn_fwd_kernel(const T* __restrict__ y,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ bias,
                                                          T* __restrict__ out,
                                                          uint8_t* __restrict__ idx, int N, int H,
                                                          int W, int C, int Ho, int Wo, int k,
                                                          int s, int p) {
  const int cg = C / 8;
  const int c8 = threadIdx.x % cg;
  float sc[8], bi[8];
  ld_f32x8(scale + c8 * 8, sc);
  ld_f32x8(bias + c8 * 8, bi);
  const long total = (long)N * Ho * Wo * cg;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const long pix = t / cg;
    const int wo = (int)(pix % Wo);
    const long r = pix / Wo;
    const int ho = (int)(r % Ho);
    const int n = (int)(r / Ho);
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      best[q] = -INFINITY;
      arg[q] = 0;
    }
    auto visit = [&](const float* v, int tap) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float z = v[q] * sc[q] + bi[q];
        z = (z != z) ? z : fmaxf(z, 0.f);  // ReLU, NaN propagates like torch
        z = as_stored<T>(z);               // compare what the unfused path would have stored
        if (z > best[q] || (z != z)) {
          best[q] = z;
          arg[q] = (uint8_t)tap;
        }
      }
    };
    if constexpr (KS > 0) {
      Raw8<T> raw[KS * KS];
      bool ok[KS * KS];
#pragma unroll
      for (int kh = 0; kh < KS; ++kh)
#pragma unroll
        for (int kw = 0; kw < KS; ++kw) {
          const int hi = ho * s - p + kh, wi = wo * s - p + kw;
          ok[kh * KS + kw] = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
          const int hc = min(max(hi, 0), H - 1), wc = min(max(wi, 0), W - 1);
          raw[kh * KS + kw] = ld_raw8(y + (((long)n * H + hc) * W + wc) * C + c8 * 8);
        }
#pragma unroll
      for (int t2 = 0; t2 < KS * KS; ++t2) {
        if (!ok[t2]) continue;
        float v[8];
        unpack_raw(raw[t2], v);
        visit(v, t2);
      }
    } else {
      for (int kh = 0; kh < k; ++kh) {
        const int hi = ho * s - p + kh;
        if (hi < 0 || hi >= H) continue;
        for (int kw = 0; kw < k; ++kw) {
          const int wi = wo * s - p + kw;
          if (wi < 0 || wi >= W) continue;
          float v[8];
          load8(y + (((long)n * H + hi) * W + wi) * C + c8 * 8, v);
          visit(v, kh * k + kw);
        }
      }
    }
    const long o = pix * C + c8 * 8;
    store8(out + o, best);
    uint2 a;
    a.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | ((uint32_t)arg[3] << 24);
    a.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | ((uint32_t)arg[7] << 24);
    *reinterpret_cast<uint2*>(idx + o) = a;
  }
}

// g of 8 channels at pre-pool pixel (n, hi, wi): see above.
template <class T>
__device__ __forceinline__ void pool_grad8(const T* __restrict__ dp, const uint8_t* __restrict__ idx,
                                           const T* __restrict__ pout, int n, int hi, int wi,
                                           int c0, int C, int Ho, int Wo, int k, int s, int p,
                                           float* g) {
#pragma unroll
  for (int q = 0; q < 8; ++q) g[q] = 0.f;
  const int ho_lo = max(0, (hi + p - k + s) / s);
  const int ho_hi = min(Ho - 1, (hi + p) / s);
  const int wo_lo = max(0, (wi + p - k + s) / s);
  const int wo_hi = min(Wo - 1, (wi + p) / s);
  for (int ho = ho_lo; ho <= ho_hi; ++ho) {
    const int kh = hi - (ho * s - p);
    if (kh < 0 || kh >= k) continue;
    for (int wo = wo_lo; wo <= wo_hi; ++wo) {
      const int kw = wi - (wo * s - p);
      if (kw < 0 || kw >= k) continue;
      const uint8_t want = (uint8_t)(kh * k + kw);
      const long o = (((long)n * Ho + ho) * Wo + wo) * C + c0;
      const uint2 a = *reinterpret_cast<const uint2*>(idx + o);
      float d[8], pv[8];
      load8(dp + o, d);
      load8(pout + o, pv);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint32_t word = q < 4 ? a.x : a.y;
        const uint8_t ai = (uint8_t)(word >> ((q & 3) * 8));
        if (ai == want && pv[q] > 0.f) g[q] += d[q];
      }
    }
  }
}

// The ResNet stem's 3x3 / stride 2 / pad 1 pool, per 2x2 quad of pre-pool pixels (2a..2a+1,
// 2b..2b+1): all four are covered only by the windows (a, b), (a, b+1), (a+1, b), (a+1, b+1), so
// a thread loads those four windows once (dp, argmax, output) instead of 1 + 2 + 2 + 4 window
// visits, with no data-dependent loop.  Pixel (2a+i, 2b+j) is tap (1+i-2di)*3 + (1+j-2dj) of
// window (a+di, b+dj).  g[i*2+j][q]; windows outside the output grid contribute nothing.
// MASKED: the argmax already carries the ReLU mask (255 where the output is not > 0: the fused
// stem's stem_pool_kernel), so the pooled output is not read.
template <bool MASKED, class T>
__device__ __forceinline__ void pool_grad_quad(const T* __restrict__ dp,
                                               const uint8_t* __restrict__ idx,
                                               const T* __restrict__ pout, int n, int a, int b,
                                               int c0, int C, int Ho, int Wo, float (*g)[8]) {
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int q = 0; q < 8; ++q) g[u][q] = 0.f;
  float d[2][2][8], pv[2][2][8];
  uint2 ai[2][2];
#pragma unroll
  for (int di = 0; di < 2; ++di)
#pragma unroll
    for (int dj = 0; dj < 2; ++dj) {
      const bool ok = a + di < Ho && b + dj < Wo;
      const long o = (((long)n * Ho + min(a + di, Ho - 1)) * Wo + min(b + dj, Wo - 1)) * C + c0;
      load8(dp + o, d[di][dj]);
      if constexpr (!MASKED) load8(pout + o, pv[di][dj]);
      ai[di][dj] = *reinterpret_cast<const uint2*>(idx + o);
      if (!ok) ai[di][dj] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);  // no tap matches 255
    }
  // same window order as the generic gather (rows, then columns)
#pragma unroll
  for (int di = 0; di < 2; ++di)
#pragma unroll
    for (int dj = 0; dj < 2; ++dj)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (di > i || dj > j) continue;  // window (a+di, b+dj) covers pixel (2a+i, 2b+j)?
          const uint8_t tap = (uint8_t)((1 + i - 2 * di) * 3 + (1 + j - 2 * dj));
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const uint32_t word = q < 4 ? ai[di][dj].x : ai[di][dj].y;
            const uint8_t at = (uint8_t)(word >> ((q & 3) * 8));
            if (at == tap && (MASKED || pv[di][dj][q] > 0.f)) g[i * 2 + j][q] += d[di][dj][q];
          }
        }
}

template <bool QUAD, bool MASKED, class T>
__global__ __launch_bounds__(256) void pool_bn_bwd_reduce_kernel(
    const T* __restrict__ dp, const uint8_t* __restrict__ idx, const T* __restrict__ pout,
    const T* __restrict__ y, const float* __restrict__ mean, const float* __restrict__ invstd,
    int N, int H, int W, int C, int Ho, int Wo, int k, int s, int p, float* __restrict__ rep,
    int det_rows) {
  __shared__ float red[16][256];
  const int cg = C / 8;
  const int c8 = threadIdx.x % cg;
  float mu[8], is[8], sg[8], sx[8];
  ld_f32x8(mean + c8 * 8, mu);
  ld_f32x8(invstd + c8 * 8, is);
#pragma unroll
  for (int q = 0; q < 8; ++q) sg[q] = sx[q] = 0.f;
  auto acc = [&](const float* g8, long pix) {
    float yv[8];
    load8(y + pix * C + c8 * 8, yv);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float gq = as_stored<T>(g8[q]);  // statistics of the g the unfused path would store
      sg[q] += gq;
      sx[q] += gq * (yv[q] - mu[q]) * is[q];
    }
  };
  if constexpr (QUAD) {
    const int QH = (H + 1) / 2, QW = (W + 1) / 2;
    const long total = (long)N * QH * QW * cg;
    for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long)gridDim.x * blockDim.x) {
      const long qd = t / cg;
      const int b = (int)(qd % QW);
      const long r = qd / QW;
      const int a = (int)(r % QH);
      const int n = (int)(r / QH);
      float g[4][8], yv[4][8];
      bool in[4];
      pool_grad_quad<MASKED>(dp, idx, pout, n, a, b, c8 * 8, C, Ho, Wo, g);
      // the quad's y loads are issued unconditionally (clamped pixel; a pixel past an odd edge
      // adds nothing): behind the bounds branch each was closed with a full vmcnt drain
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          in[i * 2 + j] = 2 * a + i < H && 2 * b + j < W;
          const long pix = ((long)n * H + min(2 * a + i, H - 1)) * W + min(2 * b + j, W - 1);
          load8(y + pix * C + c8 * 8, yv[i * 2 + j]);
        }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float gq = in[u] ? as_stored<T>(g[u][q]) : 0.f;
          sg[q] += gq;
          sx[q] += gq * (yv[u][q] - mu[q]) * is[q];
        }
    }
  } else {
    const long total = (long)N * H * W * cg;
    for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long)gridDim.x * blockDim.x) {
      const long pix = t / cg;
      const int wi = (int)(pix % W);
      const long r = pix / W;
      const int hi = (int)(r % H);
      const int n = (int)(r / H);
      float g[8];
      pool_grad8(dp, idx, pout, n, hi, wi, c8 * 8, C, Ho, Wo, k, s, p, g);
      acc(g, pix);
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    red[q][threadIdx.x] = sg[q];
    red[8 + q][threadIdx.x] = sx[q];
  }
  __syncthreads();
  const long rs = (long)(det_rows > 0 ? det_rows : kStatReplicas) * C;
  for (int j = threadIdx.x; j < 2 * C; j += blockDim.x) {
    const int arr = j / C, c = j % C, grp = c >> 3, q = c & 7;
    float a = 0.f;
    for (int t = grp; t < (int)blockDim.x; t += cg) a += red[arr * 8 + q][t];
    if (det_rows > 0) rep[arr * rs + (long)blockIdx.x * C + c] = a;
    else atomicAdd(rep + arr * rs + (long)(blockIdx.x % kStatReplicas) * C + c, a);
  }
}

template <bool QUAD, class T>
__global__ __launch_bounds__(256) void pool_bn_bwd_apply_kernel(
    const T* __restrict__ dp, const uint8_t* __restrict__ idx, const T* __restrict__ pout,
    const T* __restrict__ y, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ sum_g,
    const float* __restrict__ sum_gx, float inv_n, T* __restrict__ dy, int N, int H, int W, int C,
    int Ho, int Wo, int k, int s, int p) {
  const int cg = C / 8;
  const int c8 = threadIdx.x % cg;
  // dy = A*g + B*y + Cc   with A = γ·is, B = -A·is·k2, Cc = -A·k1 + A·is·k2·μ (bn.hip)
  float A[8], Bc[8], Cc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int c = c8 * 8 + q;
    const float is = invstd[c], a = gamma[c] * is;
    const float k1 = sum_g[c] * inv_n, k2 = sum_gx[c] * inv_n;
    A[q] = a;
    Bc[q] = -a * is * k2;
    Cc[q] = -a * k1 + a * is * k2 * mean[c];
  }
  auto emit = [&](const float* g8, long pix) {
    float yv[8], o[8];
    load8(y + pix * C + c8 * 8, yv);
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = A[q] * as_stored<T>(g8[q]) + Bc[q] * yv[q] + Cc[q];
    store8(dy + pix * C + c8 * 8, o);
  };
  if constexpr (QUAD) {
    const int QH = (H + 1) / 2, QW = (W + 1) / 2;
    const long total = (long)N * QH * QW * cg;
    for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long)gridDim.x * blockDim.x) {
      const long qd = t / cg;
      const int b = (int)(qd % QW);
      const long r = qd / QW;
      const int a = (int)(r % QH);
      const int n = (int)(r / QH);
      float g[4][8], yv[4][8];
      pool_grad_quad<false>(dp, idx, pout, n, a, b, c8 * 8, C, Ho, Wo, g);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {  // unconditional y loads, as in the reduction
          const long pix = ((long)n * H + min(2 * a + i, H - 1)) * W + min(2 * b + j, W - 1);
          load8(y + pix * C + c8 * 8, yv[i * 2 + j]);
        }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (2 * a + i < H && 2 * b + j < W) {
            const long pix = ((long)n * H + 2 * a + i) * W + 2 * b + j;
            float o[8];
#pragma unroll
            for (int q = 0; q < 8; ++q)
              o[q] = A[q] * as_stored<T>(g[i * 2 + j][q]) + Bc[q] * yv[i * 2 + j][q] + Cc[q];
            store8(dy + pix * C + c8 * 8, o);
          }
    }
  } else {
    const long total = (long)N * H * W * cg;
    for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long)gridDim.x * blockDim.x) {
      const long pix = t / cg;
      const int wi = (int)(pix % W);
      const long r = pix / W;
      const int hi = (int)(r % H);
      const int n = (int)(r / H);
      float g[8];
      pool_grad8(dp, idx, pout, n, hi, wi, c8 * 8, C, Ho, Wo, k, s, p, g);
      emit(g, pix);
    }
  }
}

static int ew_grid(long work) {
  long g = (work + 255) / 256;
  return (int)std::max<long>(1, std::min<long>(g, 4096));
}

void maxpool_fwd(const void* x, void* y, uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo,
                 int k, int stride, int pad, hipStream_t st, bool f32) {
  long work = (long)N * Ho * Wo * (C / 8);
  if (f32)
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, dim3(ew_grid(work)), dim3(256), 0, st,
                       (const float*)x, (float*)y, idx, N, H, W, C, Ho, Wo, k, stride, pad);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<__bf16>, dim3(ew_grid(work)), dim3(256), 0, st,
                       (const __bf16*)x, (__bf16*)y, idx, N, H, W, C, Ho, Wo, k, stride, pad);
}

void maxpool_bwd(const void* dy, const uint8_t* idx, void* dx, int N, int H, int W, int C, int Ho,
                 int Wo, int k, int stride, int pad, hipStream_t st, bool f32) {
  long work = (long)N * H * W * (C / 8);
  if (f32)
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, dim3(ew_grid(work)), dim3(256), 0, st,
                       (const float*)dy, idx, (float*)dx, N, H, W, C, Ho, Wo, k, stride, pad);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<__bf16>, dim3(ew_grid(work)), dim3(256), 0, st,
                       (const __bf16*)dy, idx, (__bf16*)dx, N, H, W, C, Ho, Wo, k, stride, pad);
}

void pool_bn_fwd(const void* y, const float* scale, const float* bias, void* out, uint8_t* idx,
                 int N, int H, int W, int C, int Ho, int Wo, int k, int stride, int pad,
                 hipStream_t st, bool f32) {
  long work = (long)N * Ho * Wo * (C / 8);
  auto launch = [&](auto tag, auto ks) {
    typedef decltype(tag) T;
    hipLaunchKernelGGL((pool_bn_fwd_kernel<decltype(ks)::value, T>), dim3(ew_grid(work)), dim3(256),
                       0, st, (const T*)y, scale, bias, (T*)out, idx, N, H, W, C, Ho, Wo, k, stride,
                       pad);
  };
  typedef std::integral_constant<int, 3> K3;
  typedef std::integral_constant<int, 0> KAny;
  if (f32) {
    if (k == 3) launch(float{}, K3{});
    else launch(float{}, KAny{});
  } else {
    if (k == 3) launch(__bf16{}, K3{});
    else launch(__bf16{}, KAny{});
  }
}

// 3x3 / stride 2 / pad 1 with the floor output size: the 2x2-quad gather applies
static bool pool_quad_ok(int H, int W, int Ho, int Wo, int k, int s, int p) {
  return k == 3 && s == 2 && p == 1 && Ho == (H - 1) / 2 + 1 && Wo == (W - 1) / 2 + 1;
}

int pool_bn_bwd_reduce_blocks(long pixels, int C) {
  long g = (pixels * (C / 8) + 256 * 16 - 1) / (256 * 16);  // >= 16 pixels per thread
  return (int)std::max<long>(1, std::min<long>(g, 1024));
}

void pool_bn_bwd_reduce(const void* dp, const uint8_t* idx, const void* pout, const void* y,
                        const float* mean, const float* invstd, int N, int H, int W, int C,
                        int Ho, int Wo, int k, int stride, int pad, float* rep, int det_rows,
                        hipStream_t st, bool f32) {
  const int G = det_rows > 0 ? det_rows : pool_bn_bwd_reduce_blocks((long)N * H * W, C);
  auto launch = [&](auto tag, auto quad) {
    typedef decltype(tag) T;
    hipLaunchKernelGGL((pool_bn_bwd_reduce_kernel<decltype(quad)::value, false, T>), dim3(G),
                       dim3(256), 0, st, (const T*)dp, idx, (const T*)pout, (const T*)y, mean,
                       invstd, N, H, W, C, Ho, Wo, k, stride, pad, rep, det_rows);
  };
  const bool quad = pool_quad_ok(H, W, Ho, Wo, k, stride, pad);
  if (pout == nullptr) {  // argmax carries the ReLU mask (fused stem): quad gather, bf16 only
    if (f32 || !quad) throw std::invalid_argument("pool_bn_bwd_reduce: masked argmax needs the bf16 quad path");
    hipLaunchKernelGGL((pool_bn_bwd_reduce_kernel<true, true, __bf16>), dim3(G), dim3(256), 0, st,
                       (const __bf16*)dp, idx, (const __bf16*)nullptr, (const __bf16*)y, mean,
                       invstd, N, H, W, C, Ho, Wo, k, stride, pad, rep, det_rows);
    return;
  }
  if (f32) {
    if (quad) launch(float{}, std::true_type{});
    else launch(float{}, std::false_type{});
  } else {
    if (quad) launch(__bf16{}, std::true_type{});
    else launch(__bf16{}, std::false_type{});
  }
}

void pool_bn_bwd_apply(const void* dp, const uint8_t* idx, const void* pout, const void* y,
                       const float* mean, const float* invstd, const float* gamma,
                       const float* sum_g, const float* sum_gx, long count, void* dy, int N, int H,
                       int W, int C, int Ho, int Wo, int k, int stride, int pad, hipStream_t st,
                       bool f32) {
  const bool quad = pool_quad_ok(H, W, Ho, Wo, k, stride, pad);
  const long work = (quad ? (long)N * ((H + 1) / 2) * ((W + 1) / 2) : (long)N * H * W) * (C / 8);
  const float inv_n = 1.f / (float)count;
  auto launch = [&](auto tag, auto q) {
    typedef decltype(tag) T;
    hipLaunchKernelGGL((pool_bn_bwd_apply_kernel<decltype(q)::value, T>), dim3(ew_grid(work)),
                       dim3(256), 0, st, (const T*)dp, idx, (const T*)pout, (const T*)y, mean,
                       invstd, gamma, sum_g, sum_gx, inv_n, (T*)dy, N, H, W, C, Ho, Wo, k, stride,
                       pad);
  };
  if (f32) {
    if (quad) launch(float{}, std::true_type{});
    else launch(float{}, std::false_type{});
  } else {
    if (quad) launch(__bf16{}, std::true_type{});
    else launch(__bf16{}, std::false_type{});
  }
}

// Global average pool: y[n][c] = mean_hw x[n][hw][c]
template <class T>
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const T* __restrict__ x,
                                                          T* __restrict__ y, int N, int HW,
                                                          int C) {
  const int cg = C / 8;
  long total = (long)N * cg;
  float inv = 1.f / (float)HW;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    int c8 = (int)(t % cg);
    long n = t / cg;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const T* base = x + n * HW * C + c8 * 8;
    for (int i = 0; i < HW; ++i) {
      float v[8];
      load8(base + (long)i * C, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += v[q];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] *= inv;
    store8(y + n * C + c8 * 8, acc);
  }
}

template <class T>
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const T* __restrict__ dy,
                                                          T* __restrict__ dx, int N, int HW,
                                                          int C) {
  const int cg = C / 8;
  long total = (long)N * HW * cg;
  float inv = 1.f / (float)HW;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    int c8 = (int)(t % cg);
    long pix = t / cg;
    long n = pix / HW;
    float v[8];
    load8(dy + n * C + c8 * 8, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] *= inv;
    store8(dx + pix * C + c8 * 8, v);
  }
}

void avgpool_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t st, bool f32) {
  dim3 g(ew_grid((long)N * (C / 8)));
  if (f32)
    hipLaunchKernelGGL(avgpool_fwd_kernel<float>, g, dim3(256), 0, st, (const float*)x, (float*)y, N, HW, C);
  else
    hipLaunchKernelGGL(avgpool_fwd_kernel<__bf16>, g, dim3(256), 0, st, (const __bf16*)x, (__bf16*)y, N, HW, C);
}

void avgpool_bwd(const void* dy, void* dx, int N, int HW, int C, hipStream_t st, bool f32) {
  dim3 g(ew_grid((long)N * HW * (C / 8)));
  if (f32)
    hipLaunchKernelGGL(avgpool_bwd_kernel<float>, g, dim3(256), 0, st, (const float*)dy, (float*)dx, N, HW, C);
  else
    hipLaunchKernelGGL(avgpool_bwd_kernel<__bf16>, g, dim3(256), 0, st, (const __bf16*)dy, (__bf16*)dx, N, HW, C);
}

}  // namespace mipipe
