// BatchNorm (training) kernels on NHWC bf16, fused with ReLU and the ResNet residual add.
//
// Forward: statistics come from the conv epilogue as a [P][C] slab of shifted partial sums;
//   bn_finalize reduces it (two deterministic stages, no atomics) into mean / invstd / scale /
//   bias and updates running stats (unbiased variance, momentum) — torch BatchNorm2d semantics.
//   bn_act_fwd then applies  z = relu(y*scale + bias [+ r | + r*rscale + rbias])  in ONE pass.
// Backward: bn_act_bwd_reduce computes Σg, Σg·x̂ (and Σg·x̂₂ for the downsample branch that
//   shares the add/ReLU) with g = dz·[z>0]; bn_act_bwd_apply produces dy (and d(residual) or
//   dy₂) in ONE pass:  dy = γ·invstd·(g − Σg/n − x̂·Σg·x̂/n).
// Elementwise mapping: a thread owns a fixed 8-channel group (16-B vectors) and strides over
// rows, so per-channel coefficients are loaded once per thread.
#include "common.hpp"
#include "launchers.hpp"

namespace mipipe {

namespace {

constexpr int kT = 256;

struct RowMap {
  int tpr;   // threads per row (C/8), capped at 256 per pass
  int rpb;   // rows per block-iteration
  int passes;  // channel passes when C/8 > 256
};

__host__ __device__ inline RowMap row_map(int C) {
  RowMap m;
  int chunks = C / 8;
  if (chunks <= kT) {
    m.tpr = chunks;
    m.rpb = kT / chunks;
    m.passes = 1;
  } else {
    m.tpr = kT;
    m.rpb = 1;
    m.passes = (chunks + kT - 1) / kT;
  }
  return m;
}

inline int grid_for_rows(long M, int rpb, int cap = 2048) {
  long g = (M + rpb - 1) / rpb;
  return (int)std::max<long>(1, std::min<long>(g, cap));
}

}  // namespace

// Per-channel final reduction of an [S][C] slab (S small) + BN statistics.
__global__ void bn_finalize_kernel(const float* __restrict__ s1, const float* __restrict__ s2,
                                   int S, int C, float inv_count, float unbias, const float* shift,
                                   const float* gamma, const float* beta, float* run_mean,
                                   float* run_var, float momentum, float eps, float* mean,
                                   float* invstd, float* scale, float* bias) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float a = 0.f, b = 0.f;
  for (int s = 0; s < S; ++s) {
    a += s1[(long)s * C + c];
    b += s2[(long)s * C + c];
  }
  float ms = a * inv_count;
  float var = fmaxf(b * inv_count - ms * ms, 0.f);
  float mu = ms + shift[c];
  float is = rsqrtf(var + eps);
  float sc = gamma[c] * is;
  mean[c] = mu;
  invstd[c] = is;
  scale[c] = sc;
  bias[c] = beta[c] - mu * sc;
  if (run_mean != nullptr) {
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mu;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * var * unbias;
  }
}

// Two-column-array colsum stage (sum and sq) without pointer arrays.
__global__ __launch_bounds__(256) void colsum2_kernel(const float* __restrict__ a_in,
                                                      const float* __restrict__ b_in,
                                                      const float* __restrict__ c_in,
                                                      float* a_out, float* b_out, float* c_out,
                                                      int P, int C, int chunk) {
  __shared__ float red[3][4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rp = threadIdx.x >> 6;
  const int p0 = blockIdx.y * chunk, p1 = min(P, p0 + chunk);
  float x = 0.f, y = 0.f, z = 0.f;
  if (col < C) {
    for (int p = p0 + rp; p < p1; p += 4) {
      long o = (long)p * C + col;
      x += a_in[o];
      y += b_in[o];
      if (c_in != nullptr) z += c_in[o];
    }
  }
  red[0][rp][threadIdx.x & 63] = x;
  red[1][rp][threadIdx.x & 63] = y;
  red[2][rp][threadIdx.x & 63] = z;
  __syncthreads();
  if (rp == 0 && col < C) {
    int t = threadIdx.x;
    long o = (long)blockIdx.y * C + col;
    a_out[o] = red[0][0][t] + red[0][1][t] + red[0][2][t] + red[0][3][t];
    b_out[o] = red[1][0][t] + red[1][1][t] + red[1][2][t] + red[1][3][t];
    if (c_out != nullptr) c_out[o] = red[2][0][t] + red[2][1][t] + red[2][2][t] + red[2][3][t];
  }
}

// Reduce up to three [P][C] slabs to [S][C] with S <= 32 rows.  Returns S; outputs in work.
static int stage_reduce(const float* a, const float* b, const float* c, int P, int C, float* work,
                        const float** ra, const float** rb, const float** rc, hipStream_t st) {
  if (P <= 32) {
    *ra = a; *rb = b; *rc = c;
    return P;
  }
  int S = std::min(32, (P + 15) / 16);
  int chunk = (P + S - 1) / S;
  S = (P + chunk - 1) / chunk;
  float* wa = work;
  float* wb = work + (long)S * C;
  float* wc = c ? work + 2L * S * C : nullptr;
  dim3 grid((C + 63) / 64, S);
  hipLaunchKernelGGL(colsum2_kernel, grid, dim3(256), 0, st, a, b, c, wa, wb, wc, P, C, chunk);
  *ra = wa; *rb = wb; *rc = wc;
  return S;
}

void bn_finalize(const float* psum, const float* psq, int P, int C, long count, const float* shift,
                 const float* gamma, const float* beta, float* run_mean, float* run_var,
                 float momentum, float eps, float* mean, float* invstd, float* scale, float* bias,
                 float* work, hipStream_t st) {
  const float *ra, *rb, *rc;
  int S = stage_reduce(psum, psq, nullptr, P, C, work, &ra, &rb, &rc, st);
  float unbias = count > 1 ? (float)count / (float)(count - 1) : 1.f;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, ra, rb, S, C,
                     1.f / (float)count, unbias, shift, gamma, beta, run_mean, run_var, momentum,
                     eps, mean, invstd, scale, bias);
}

// ----------------------------------------------------------------------------- forward apply
template <int RES>  // 0 none, 1 raw residual, 2 BN'd residual
__global__ __launch_bounds__(256) void bn_act_fwd_kernel(const __bf16* __restrict__ y,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ bias,
                                                         const __bf16* __restrict__ r,
                                                         const float* __restrict__ rscale,
                                                         const float* __restrict__ rbias,
                                                         __bf16* __restrict__ z, long M, int C,
                                                         bool relu) {
  const RowMap mp = row_map(C);
  const int t = threadIdx.x;
  const int rg = t / mp.tpr;
  if (rg >= mp.rpb) return;
  for (int pass = 0; pass < mp.passes; ++pass) {
    const int cg = pass * mp.tpr + (t % mp.tpr);
    if (cg * 8 >= C) continue;
    const int c0 = cg * 8;
    float sc[8], bi[8], rs[8], rb[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      sc[q] = scale[c0 + q];
      bi[q] = bias[c0 + q];
      if (RES == 2) {
        rs[q] = rscale[c0 + q];
        rb[q] = rbias[c0 + q];
      }
    }
    for (long row = (long)blockIdx.x * mp.rpb + rg; row < M; row += (long)gridDim.x * mp.rpb) {
      long off = row * C + c0;
      uint4 yv = *reinterpret_cast<const uint4*>(y + off);
      float v[8];
      unpack8(yv, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = v[q] * sc[q] + bi[q];
      if (RES != 0) {
        uint4 rv = *reinterpret_cast<const uint4*>(r + off);
        float w[8];
        unpack8(rv, w);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] += (RES == 2) ? (w[q] * rs[q] + rb[q]) : w[q];
      }
      if (relu) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
      }
      *reinterpret_cast<uint4*>(z + off) = pack8(v);
    }
  }
}

void bn_act_fwd(const void* y, const float* scale, const float* bias, const void* r,
                const float* rscale, const float* rbias, void* z, long M, int C, bool relu,
                hipStream_t st) {
  RowMap mp = row_map(C);
  int grid = grid_for_rows(M, mp.rpb);
  const __bf16* yp = (const __bf16*)y;
  const __bf16* rp = (const __bf16*)r;
  __bf16* zp = (__bf16*)z;
  if (r == nullptr)
    hipLaunchKernelGGL(bn_act_fwd_kernel<0>, dim3(grid), dim3(256), 0, st, yp, scale, bias, rp, rscale, rbias, zp, M, C, relu);
  else if (rscale == nullptr)
    hipLaunchKernelGGL(bn_act_fwd_kernel<1>, dim3(grid), dim3(256), 0, st, yp, scale, bias, rp, rscale, rbias, zp, M, C, relu);
  else
    hipLaunchKernelGGL(bn_act_fwd_kernel<2>, dim3(grid), dim3(256), 0, st, yp, scale, bias, rp, rscale, rbias, zp, M, C, relu);
}

// ----------------------------------------------------------------------------- backward
int bn_bwd_partials(long M, int C) {
  RowMap mp = row_map(C);
  return grid_for_rows(M, mp.rpb, 1024);
}

template <bool TWO>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const __bf16* __restrict__ dz, const __bf16* __restrict__ z, const __bf16* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const __bf16* __restrict__ y2, const float* __restrict__ mean2,
    const float* __restrict__ invstd2, bool relu, long M, int C, float* __restrict__ pg,
    float* __restrict__ pgx, float* __restrict__ pgx2) {
  __shared__ float red[3][kT][8];
  const RowMap mp = row_map(C);
  const int t = threadIdx.x;
  const int rg = t / mp.tpr;
  const bool active = rg < mp.rpb;
  for (int pass = 0; pass < mp.passes; ++pass) {
    const int cg = pass * mp.tpr + (t % mp.tpr);
    const int c0 = cg * 8;
    float sg[8], sx[8], sx2[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) sg[q] = sx[q] = sx2[q] = 0.f;
    if (active && c0 < C) {
      float mu[8], is[8], mu2[8], is2[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        mu[q] = mean[c0 + q];
        is[q] = invstd[c0 + q];
        if (TWO) {
          mu2[q] = mean2[c0 + q];
          is2[q] = invstd2[c0 + q];
        }
      }
      for (long row = (long)blockIdx.x * mp.rpb + rg; row < M; row += (long)gridDim.x * mp.rpb) {
        long off = row * C + c0;
        float g[8], yv[8];
        unpack8(*reinterpret_cast<const uint4*>(dz + off), g);
        if (relu) {
          float zv[8];
          unpack8(*reinterpret_cast<const uint4*>(z + off), zv);
#pragma unroll
          for (int q = 0; q < 8; ++q) g[q] = zv[q] > 0.f ? g[q] : 0.f;
        }
        unpack8(*reinterpret_cast<const uint4*>(y + off), yv);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          sg[q] += g[q];
          sx[q] += g[q] * (yv[q] - mu[q]) * is[q];
        }
        if (TWO) {
          float y2v[8];
          unpack8(*reinterpret_cast<const uint4*>(y2 + off), y2v);
#pragma unroll
          for (int q = 0; q < 8; ++q) sx2[q] += g[q] * (y2v[q] - mu2[q]) * is2[q];
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      red[0][t][q] = sg[q];
      red[1][t][q] = sx[q];
      red[2][t][q] = sx2[q];
    }
    __syncthreads();
    if (active && rg == 0 && c0 < C) {
      for (int k = 1; k < mp.rpb; ++k) {
        int src = k * mp.tpr + (t % mp.tpr);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          sg[q] += red[0][src][q];
          sx[q] += red[1][src][q];
          sx2[q] += red[2][src][q];
        }
      }
      long o = (long)blockIdx.x * C + c0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        pg[o + q] = sg[q];
        pgx[o + q] = sx[q];
        if (TWO) pgx2[o + q] = sx2[q];
      }
    }
    __syncthreads();
  }
}

__global__ void sum_rows3_kernel(const float* a, const float* b, const float* c, int S, int C,
                                 float* oa, float* ob, float* oc) {
  int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= C) return;
  float x = 0.f, y = 0.f, z = 0.f;
  for (int s = 0; s < S; ++s) {
    x += a[(long)s * C + col];
    y += b[(long)s * C + col];
    if (c) z += c[(long)s * C + col];
  }
  oa[col] = x;
  ob[col] = y;
  if (oc) oc[col] = z;
}

void bn_act_bwd_reduce(const void* dz, const void* z, const void* y, const float* mean,
                       const float* invstd, const void* y2, const float* mean2,
                       const float* invstd2, bool relu, long M, int C, float* out_g,
                       float* out_gx, float* out_gx2, float* work, hipStream_t st) {
  RowMap mp = row_map(C);
  int G = grid_for_rows(M, mp.rpb, 1024);
  float* pg = work;
  float* pgx = work + (long)G * C;
  float* pgx2 = work + 2L * G * C;
  float* rest = work + 3L * G * C;
  const __bf16 *dzp = (const __bf16*)dz, *zp = (const __bf16*)z, *yp = (const __bf16*)y,
               *y2p = (const __bf16*)y2;
  if (y2 == nullptr)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<false>, dim3(G), dim3(256), 0, st, dzp, zp, yp, mean, invstd, y2p, mean2, invstd2, relu, M, C, pg, pgx, pgx2);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<true>, dim3(G), dim3(256), 0, st, dzp, zp, yp, mean, invstd, y2p, mean2, invstd2, relu, M, C, pg, pgx, pgx2);
  const float *ra, *rb, *rc;
  int S = stage_reduce(pg, pgx, y2 ? pgx2 : nullptr, G, C, rest, &ra, &rb, &rc, st);
  hipLaunchKernelGGL(sum_rows3_kernel, dim3((C + 255) / 256), dim3(256), 0, st, ra, rb,
                     y2 ? rc : nullptr, S, C, out_g, out_gx, y2 ? out_gx2 : nullptr);
}

template <int MODE>  // 0: dy only, 1: dy + dres (=g), 2: dy + dy2 (second BN branch)
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const __bf16* __restrict__ dz, const __bf16* __restrict__ z, const __bf16* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ sum_g,
    const float* __restrict__ sum_gx, const __bf16* __restrict__ y2,
    const float* __restrict__ mean2, const float* __restrict__ invstd2,
    const float* __restrict__ gamma2, const float* __restrict__ sum_gx2, float inv_n, bool relu,
    __bf16* __restrict__ dy, __bf16* __restrict__ dother, long M, int C) {
  const RowMap mp = row_map(C);
  const int t = threadIdx.x;
  const int rg = t / mp.tpr;
  if (rg >= mp.rpb) return;
  for (int pass = 0; pass < mp.passes; ++pass) {
    const int cg = pass * mp.tpr + (t % mp.tpr);
    const int c0 = cg * 8;
    if (c0 >= C) continue;
    // dy = A*g + B*y + Cc   with A = γ·is, B = -A·is·k2, Cc = -A·k1 + A·is·k2·μ
    float A[8], Bc[8], Cc[8], A2[8], B2[8], C2[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      int c = c0 + q;
      float is = invstd[c], a = gamma[c] * is;
      float k1 = sum_g[c] * inv_n, k2 = sum_gx[c] * inv_n;
      A[q] = a;
      Bc[q] = -a * is * k2;
      Cc[q] = -a * k1 + a * is * k2 * mean[c];
      if (MODE == 2) {
        float is2 = invstd2[c], a2 = gamma2[c] * is2, k22 = sum_gx2[c] * inv_n;
        A2[q] = a2;
        B2[q] = -a2 * is2 * k22;
        C2[q] = -a2 * k1 + a2 * is2 * k22 * mean2[c];
      }
    }
    for (long row = (long)blockIdx.x * mp.rpb + rg; row < M; row += (long)gridDim.x * mp.rpb) {
      long off = row * C + c0;
      float g[8], yv[8], o[8];
      unpack8(*reinterpret_cast<const uint4*>(dz + off), g);
      if (relu) {
        float zv[8];
        unpack8(*reinterpret_cast<const uint4*>(z + off), zv);
#pragma unroll
        for (int q = 0; q < 8; ++q) g[q] = zv[q] > 0.f ? g[q] : 0.f;
      }
      unpack8(*reinterpret_cast<const uint4*>(y + off), yv);
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = A[q] * g[q] + Bc[q] * yv[q] + Cc[q];
      *reinterpret_cast<uint4*>(dy + off) = pack8(o);
      if (MODE == 1) {
        *reinterpret_cast<uint4*>(dother + off) = pack8(g);
      } else if (MODE == 2) {
        float y2v[8];
        unpack8(*reinterpret_cast<const uint4*>(y2 + off), y2v);
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = A2[q] * g[q] + B2[q] * y2v[q] + C2[q];
        *reinterpret_cast<uint4*>(dother + off) = pack8(o);
      }
    }
  }
}

void bn_act_bwd_apply(const void* dz, const void* z, const void* y, const float* mean,
                      const float* invstd, const float* gamma, const float* sum_g,
                      const float* sum_gx, const void* y2, const float* mean2,
                      const float* invstd2, const float* gamma2, const float* sum_gx2, long count,
                      bool relu, bool want_dres, void* dy, void* dother, long M, int C,
                      hipStream_t st) {
  RowMap mp = row_map(C);
  int grid = grid_for_rows(M, mp.rpb);
  float inv_n = 1.f / (float)count;
  const __bf16 *dzp = (const __bf16*)dz, *zp = (const __bf16*)z, *yp = (const __bf16*)y,
               *y2p = (const __bf16*)y2;
  __bf16 *dyp = (__bf16*)dy, *dop = (__bf16*)dother;
  if (y2 != nullptr)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<2>, dim3(grid), dim3(256), 0, st, dzp, zp, yp, mean, invstd, gamma, sum_g, sum_gx, y2p, mean2, invstd2, gamma2, sum_gx2, inv_n, relu, dyp, dop, M, C);
  else if (want_dres)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<1>, dim3(grid), dim3(256), 0, st, dzp, zp, yp, mean, invstd, gamma, sum_g, sum_gx, y2p, mean2, invstd2, gamma2, sum_gx2, inv_n, relu, dyp, dop, M, C);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<0>, dim3(grid), dim3(256), 0, st, dzp, zp, yp, mean, invstd, gamma, sum_g, sum_gx, y2p, mean2, invstd2, gamma2, sum_gx2, inv_n, relu, dyp, dop, M, C);
}

}  // namespace mipipe
