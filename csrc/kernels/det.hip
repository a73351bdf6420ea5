// Deterministic reductions (the reference's cudnn.deterministic = True, task.py:25-26).
//
// In deterministic mode no kernel accumulates a floating-point value with atomics: producers
// write per-block partial rows, and these kernels sum the rows in a FIXED order (fixed thread ->
// row assignment, fixed LDS tree), so two identical runs produce bit-identical results.
#include "common.hpp"
#include "launchers.hpp"

namespace mipipe {

int g_deterministic = 0;

// out[c] (+)= sum_p in[p * stride][c] for up to three row arrays (blockIdx.y).  Block: 64 channels x 16 row
// groups; group g sums rows g, g+16, ... in order, then the 16 group sums are added in index order.
__global__ __launch_bounds__(1024) void det_sum_rows_kernel(const float* __restrict__ in0,
                                                            const float* __restrict__ in1,
                                                            const float* __restrict__ in2, int P,
                                                            int C, float* __restrict__ out0,
                                                            float* __restrict__ out1,
                                                            float* __restrict__ out2,
                                                            bool accumulate, int stride) {
  __shared__ float part[16][65];
  const int lc = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lc;
  const float* in = blockIdx.y == 0 ? in0 : blockIdx.y == 1 ? in1 : in2;
  float* out = blockIdx.y == 0 ? out0 : blockIdx.y == 1 ? out1 : out2;
  const long rs = (long)stride * C;
  float a = 0.f;
  if (c < C) {
    // 8 rows of loads in flight, then added in row order (same order as a plain loop: the
    // result is bit-identical, the latency is paid once per 8 rows instead of per row)
    int p = g;
    for (; p + 7 * 16 < P; p += 8 * 16) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = in[(long)(p + u * 16) * rs + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) a += v[u];
    }
    for (; p < P; p += 16) a += in[(long)p * rs + c];
  }
  part[g][lc] = a;
  __syncthreads();
  if (g == 0 && c < C) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += part[k][lc];
    out[c] = accumulate ? out[c] + s : s;
  }
}

// First level of a long column sum (P partial rows, e.g. one per M-tile of a conv: 6272 for
// ResNet-50's layer 1): block (x, k, array) sums rows [k*R, k*R + R) of its 64 channels in a
// fixed order and writes the chunk sum over the chunk's FIRST row (the partial rows are scratch;
// only this block reads its chunk).  The one-level kernel ran such a sum on C/64 blocks — two
// CUs for C = 64 — and cost ~11 us per call, 1.2 ms per deterministic ResNet-50 step.
__global__ __launch_bounds__(256) void det_chunk_sum_kernel(float* __restrict__ in0,
                                                            float* __restrict__ in1,
                                                            float* __restrict__ in2, int P,
                                                            int C) {
  __shared__ float part[4][65];
  const int lc = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lc;
  float* in = blockIdx.z == 0 ? in0 : blockIdx.z == 1 ? in1 : in2;
  const int r0 = blockIdx.y * kDetChunkRows;
  const int r1 = min(P, r0 + kDetChunkRows);
  float a = 0.f;
  if (c < C) {
    float v[kDetChunkRows / 4];
#pragma unroll
    for (int u = 0; u < kDetChunkRows / 4; ++u) {
      const int p = r0 + g + 4 * u;
      v[u] = p < r1 ? in[(long)min(p, P - 1) * C + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kDetChunkRows / 4; ++u) a += v[u];
  }
  part[g][lc] = a;
  __syncthreads();  // every row of the chunk has been read before its first row is overwritten
  if (g == 0 && c < C) in[(long)r0 * C + c] = ((part[0][lc] + part[1][lc]) + part[2][lc]) + part[3][lc];
}

int det_chunk_sums(float* in0, float* in1, float* in2, int P, int C, hipStream_t st) {
  const int arrays = in1 == nullptr ? 1 : in2 == nullptr ? 2 : 3;
  const int nch = (P + kDetChunkRows - 1) / kDetChunkRows;
  hipLaunchKernelGGL(det_chunk_sum_kernel, dim3((C + 63) / 64, nch, arrays), dim3(256), 0, st,
                     in0, in1, in2, P, C);
  return nch;
}

void det_sum_rows(float* in0, float* in1, int P, int C, float* out0, float* out1,
                  bool accumulate, hipStream_t st, float* in2, float* out2) {
  // arrays are taken in order: in2 only together with in1
  const int arrays = in1 == nullptr ? 1 : in2 == nullptr ? 2 : 3;
  int stride = 1;
  if (P > 4 * kDetChunkRows) {  // two levels: chunk sums in place, then the chunk sums
    const int nch = (P + kDetChunkRows - 1) / kDetChunkRows;
    hipLaunchKernelGGL(det_chunk_sum_kernel, dim3((C + 63) / 64, nch, arrays), dim3(256), 0, st,
                       in0, in1, in2, P, C);
    P = nch;
    stride = kDetChunkRows;
  }
  dim3 grid((C + 63) / 64, arrays);
  hipLaunchKernelGGL(det_sum_rows_kernel, grid, dim3(1024), 0, st, in0, in1, in2, P, C, out0,
                     out1, out2, accumulate, stride);
}

// out[i] += sum_s ws[s][i], s in order (split-K partial tiles of a weight gradient).
__global__ __launch_bounds__(256) void splitk_sum_kernel(const float* __restrict__ ws, int splits,
                                                         long n4, float* __restrict__ out) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    float4 a = reinterpret_cast<const float4*>(ws)[i];
    for (int s = 1; s < splits; ++s) {
      const float4 b = reinterpret_cast<const float4*>(ws + (long)s * n4 * 4)[i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    float4 o = reinterpret_cast<float4*>(out)[i];
    o.x += a.x; o.y += a.y; o.z += a.z; o.w += a.w;
    reinterpret_cast<float4*>(out)[i] = o;
  }
}

// Same sum with the split count a template constant: every slice load of an element is issued
// before the first add (one memory latency per element instead of `splits` dependent ones).
template <int S>
__global__ __launch_bounds__(256) void splitk_sum_fixed_kernel(const float* __restrict__ ws, long n4,
                                                               float* __restrict__ out) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    float4 v[S];
#pragma unroll
    for (int s = 0; s < S; ++s) v[s] = reinterpret_cast<const float4*>(ws + (long)s * n4 * 4)[i];
    float4 o = reinterpret_cast<float4*>(out)[i];
    float4 a = v[0];
#pragma unroll
    for (int s = 1; s < S; ++s) {
      a.x += v[s].x; a.y += v[s].y; a.z += v[s].z; a.w += v[s].w;
    }
    o.x += a.x; o.y += a.y; o.z += a.z; o.w += a.w;
    reinterpret_cast<float4*>(out)[i] = o;
  }
}

__global__ void splitk_sum_tail_kernel(const float* __restrict__ ws, int splits, long n0, long n,
                                       float* __restrict__ out) {
  const long i = n0 + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float a = 0.f;
  for (int s = 0; s < splits; ++s) a += ws[(long)s * n + i];
  out[i] += a;
}

// Many splits over a small output (the patch-resident 3x3 weight-grad: 256 slices of a 36 K-float
// tile): one thread per float4 column would serialise 256 dependent loads.  P threads per column
// each sum a fixed strided subset of the slices, then the P partials are added in a fixed order
// through LDS — deterministic for a given (splits, P).
template <int P>
__global__ __launch_bounds__(256) void splitk_sum_wide_kernel(const float* __restrict__ ws,
                                                              int splits, long n4,
                                                              float* __restrict__ out) {
  constexpr int C = 256 / P;  // float4 columns per block
  __shared__ float4 part[P][C];
  const int c = threadIdx.x % C, w = threadIdx.x / C;
  const long col = (long)blockIdx.x * C + c;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < n4) {
    for (int s = w; s < splits; s += P) {
      const float4 b = reinterpret_cast<const float4*>(ws + (long)s * n4 * 4)[col];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
  }
  part[w][c] = a;
  __syncthreads();
  if (w == 0 && col < n4) {
    float4 t = part[0][c];
#pragma unroll
    for (int q = 1; q < P; ++q) {
      const float4 b = part[q][c];
      t.x += b.x; t.y += b.y; t.z += b.z; t.w += b.w;
    }
    float4 o = reinterpret_cast<float4*>(out)[col];
    o.x += t.x; o.y += t.y; o.z += t.z; o.w += t.w;
    reinterpret_cast<float4*>(out)[col] = o;
  }
}

// out[m][n] = T(sum_s ws[s][m][n] + bias[n] + addend[m][n]), s in order: the finishing pass of
// a split-K GEMM with an activation-dtype output (M x N, N % 8 == 0; ws slices are [M][N]
// contiguous; addend: the data-grad's second gradient, [M][N] in T, as the GEMM epilogue adds it).
// T = bf16, or fp32 on the reference-precision path (the fc layer of ResNet-18 at 32x32: 64-128
// output tiles of 128x64 for 256 CUs).
template <class T>
__global__ __launch_bounds__(256) void splitk_sum_out_kernel(const float* __restrict__ ws,
                                                             int splits, long M, int N,
                                                             const float* __restrict__ bias,
                                                             const T* __restrict__ addend,
                                                             T* __restrict__ out, long ldc) {
  const long n8 = (long)N / 8;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // one 8-column chunk
  if (i >= M * n8) return;
  const long m = i / n8, c = (i % n8) * 8;
  const float* src = ws + m * N + c;
  float f[8];
  ld_f32x8(src, f);
  for (int s = 1; s < splits; ++s) {
    float g[8];
    ld_f32x8(src + (long)s * M * N, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] += g[e];
  }
  if (bias != nullptr) {
    float b[8];
    ld_f32x8(bias + c, b);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] += b[e];
  }
  if (addend != nullptr) {  // the GEMM epilogue's order: T(acc + float(addend))
    float a[8];
    load8(addend + m * (long)N + c, a);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] += a[e];
  }
  store8(out + m * ldc + c, f);
}

void splitk_sum_bf16(const float* ws, int splits, long M, int N, const float* bias, void* out,
                     long ldc, hipStream_t st, const void* addend) {
  const long chunks = M * (N / 8);
  hipLaunchKernelGGL(splitk_sum_out_kernel<__bf16>, dim3((unsigned)((chunks + 255) / 256)),
                     dim3(256), 0, st, ws, splits, M, N, bias, (const __bf16*)addend,
                     (__bf16*)out, ldc);
}

void splitk_sum_f32out(const float* ws, int splits, long M, int N, const float* bias, float* out,
                       long ldc, hipStream_t st, const float* addend) {
  const long chunks = M * (N / 8);
  hipLaunchKernelGGL(splitk_sum_out_kernel<float>, dim3((unsigned)((chunks + 255) / 256)),
                     dim3(256), 0, st, ws, splits, M, N, bias, addend, out, ldc);
}

void splitk_sum(const float* ws, int splits, long n, float* out, hipStream_t st) {
  // the vector path needs n % 4 == 0 and 16-B aligned rows of ws / out
  const bool vec = (n % 4) == 0 && (reinterpret_cast<uintptr_t>(out) % 16) == 0;
  if (vec && splits >= 32) {
    const long n4 = n / 4;
    hipLaunchKernelGGL(splitk_sum_wide_kernel<16>, dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0,
                       st, ws, splits, n4, out);
  } else if (vec && splits >= 8) {
    const long n4 = n / 4;
    hipLaunchKernelGGL(splitk_sum_wide_kernel<4>, dim3((unsigned)((n4 + 63) / 64)), dim3(256), 0,
                       st, ws, splits, n4, out);
  } else if (vec && splits >= 2 && splits <= 7) {
    const long n4 = n / 4;
    const dim3 grid((unsigned)std::max<long>(1, std::min<long>(4096, (n4 + 255) / 256)));
    switch (splits) {
      case 2: hipLaunchKernelGGL(splitk_sum_fixed_kernel<2>, grid, dim3(256), 0, st, ws, n4, out); break;
      case 3: hipLaunchKernelGGL(splitk_sum_fixed_kernel<3>, grid, dim3(256), 0, st, ws, n4, out); break;
      case 4: hipLaunchKernelGGL(splitk_sum_fixed_kernel<4>, grid, dim3(256), 0, st, ws, n4, out); break;
      case 5: hipLaunchKernelGGL(splitk_sum_fixed_kernel<5>, grid, dim3(256), 0, st, ws, n4, out); break;
      case 6: hipLaunchKernelGGL(splitk_sum_fixed_kernel<6>, grid, dim3(256), 0, st, ws, n4, out); break;
      default: hipLaunchKernelGGL(splitk_sum_fixed_kernel<7>, grid, dim3(256), 0, st, ws, n4, out); break;
    }
  } else if (vec) {
    const long n4 = n / 4;
    const long g = std::min<long>(4096, (n4 + 255) / 256);
    hipLaunchKernelGGL(splitk_sum_kernel, dim3((unsigned)std::max<long>(1, g)), dim3(256), 0, st,
                       ws, splits, n4, out);
  } else {
    hipLaunchKernelGGL(splitk_sum_tail_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       st, ws, splits, 0l, n, out);
  }
}

}  // namespace mipipe
