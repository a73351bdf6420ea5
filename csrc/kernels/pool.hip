// NHWC pooling: max-pool with 1-byte window-argmax (fwd/bwd) and global average pool.
// Backward max-pool is a gather over the windows covering each input pixel (deterministic,
// no atomics).  Each thread moves 8 channels (one 16-B bf16 vector or two fp32 vectors).
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
