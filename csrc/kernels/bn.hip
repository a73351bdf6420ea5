// BatchNorm (training) kernels on NHWC bf16 / fp32 (element type T), fused with ReLU and the ResNet residual add.
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
constexpr int kRowU = 4;  // rows per thread-iteration of bn_bwd_reduce (loads in flight)

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

}  // namespace

// Per-channel final reduction of a [P][C] slab pair (P = replica rows) + BN statistics.
// With zero_after the slab is cleared for reuse (replica slabs are persistent and zeroed).
// All P loads are issued before any store (one memory latency, not P), and the
// num_batches_tracked increment rides along (no separate launch).
template <int P>
__global__ void bn_finalize_kernel(float* __restrict__ s1, float* __restrict__ s2, int Pdyn, int C,
                                   float inv_count, float unbias, const float* shift,
                                   const float* gamma, const float* beta, float* run_mean,
                                   float* run_var, float momentum, float eps, float* mean,
                                   float* invstd, float* scale, float* bias, bool zero_after,
                                   long long* nbt) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (nbt != nullptr && c == 0) *nbt += 1;
  if (c >= C) return;
  float a = 0.f, b = 0.f;
  if (P > 0) {
    float va[P > 0 ? P : 1], vb[P > 0 ? P : 1];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      va[p] = s1[(long)p * C + c];
      vb[p] = s2[(long)p * C + c];
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
      a += va[p];
      b += vb[p];
    }
    if (zero_after) {
#pragma unroll
      for (int p = 0; p < P; ++p) {
        s1[(long)p * C + c] = 0.f;
        s2[(long)p * C + c] = 0.f;
      }
    }
  } else {
    for (int p = 0; p < Pdyn; ++p) {
      a += s1[(long)p * C + c];
      b += s2[(long)p * C + c];
    }
    if (zero_after)
      for (int p = 0; p < Pdyn; ++p) {
        s1[(long)p * C + c] = 0.f;
        s2[(long)p * C + c] = 0.f;
      }
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

// Sum of P rows (row p at in[k][p * rs + c]) in det_sum_rows' fixed order: 16 row groups per
// channel (group g: rows g, g+16, ... with 8 rows of loads in flight, added in row order), the
// caller then adds the 16 group sums in index order.  One memory latency per 8 rows instead of
// one per row: a one-thread-per-channel loop over 128 rows cost 34-36 us per call.
template <int NA>
__device__ __forceinline__ void rows_sum16(float* const (&in)[NA], int P, long rs, int c, int g,
                                           float (&a)[NA]) {
#pragma unroll
  for (int k = 0; k < NA; ++k) a[k] = 0.f;
  int p = g;
  for (; p + 7 * 16 < P; p += 8 * 16) {
    float v[NA][8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int k = 0; k < NA; ++k) v[k][u] = in[k][(long)(p + u * 16) * rs + c];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int k = 0; k < NA; ++k) a[k] += v[k][u];
  }
  for (; p < P; p += 16)
#pragma unroll
    for (int k = 0; k < NA; ++k) a[k] += in[k][(long)p * rs + c];
}

// bn_finalize of P partial rows that are NOT a replica slab (the deterministic mode's one row
// per M-tile of the producing conv): 64 channels x 16 row groups per 1024-thread block, the
// rows summed in det_sum_rows' order — the same bits as det_sum_rows into a zeroed replica slab
// followed by the replica finalize, in one launch.  stride: rows are every stride-th row of the
// [rows][C] array (the chunk sums det_chunk_sums leaves in place for P > 256).
__global__ __launch_bounds__(1024) void bn_finalize_rows_kernel(
    float* __restrict__ s1, float* __restrict__ s2, int P, int C, int stride, float inv_count,
    float unbias, const float* shift, const float* gamma, const float* beta, float* run_mean,
    float* run_var, float momentum, float eps, float* mean, float* invstd, float* scale,
    float* bias, bool zero_after, long long* nbt) {
  __shared__ float part[2][16][65];
  const int lc = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lc;
  if (nbt != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;
  float a[2] = {0.f, 0.f};
  const long rs = (long)stride * C;
  if (c < C) {
    float* const in[2] = {s1, s2};
    rows_sum16<2>(in, P, rs, c, g, a);
    if (zero_after)  // (every row this thread read; its own loads retired above)
      for (int p = g; p < P; p += 16) {
        s1[(long)p * rs + c] = 0.f;
        s2[(long)p * rs + c] = 0.f;
      }
  }
  part[0][g][lc] = a[0];
  part[1][g][lc] = a[1];
  __syncthreads();
  if (g != 0 || c >= C) return;
  float sa = 0.f, sb = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    sa += part[0][k][lc];
    sb += part[1][k][lc];
  }
  float ms = sa * inv_count;
  float var = fmaxf(sb * inv_count - ms * ms, 0.f);
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

void bn_finalize(float* psum, float* psq, int P, int C, long count, const float* shift,
                 const float* gamma, const float* beta, float* run_mean, float* run_var,
                 float momentum, float eps, float* mean, float* invstd, float* scale, float* bias,
                 bool zero_after, long long* nbt, hipStream_t st) {
  float unbias = count > 1 ? (float)count / (float)(count - 1) : 1.f;
  if (P == kStatReplicas) {
    dim3 grid((C + 255) / 256);
    hipLaunchKernelGGL(bn_finalize_kernel<kStatReplicas>, grid, dim3(256), 0, st, psum, psq, P, C,
                       1.f / (float)count, unbias, shift, gamma, beta, run_mean, run_var, momentum,
                       eps, mean, invstd, scale, bias, zero_after, nbt);
    return;
  }
  // partial rows (deterministic mode): long columns are chunk-summed in place first, exactly as
  // det_sum_rows does (so the result is det_sum_rows' bits)
  int stride = 1;
  if (P > 4 * kDetChunkRows) {
    P = det_chunk_sums(psum, psq, nullptr, P, C, st);
    stride = kDetChunkRows;
    zero_after = false;  // scratch rows, now partly overwritten by the chunk sums
  }
  hipLaunchKernelGGL(bn_finalize_rows_kernel, dim3((C + 63) / 64), dim3(1024), 0, st, psum, psq,
                     P, C, stride, 1.f / (float)count, unbias, shift, gamma, beta, run_mean,
                     run_var, momentum, eps, mean, invstd, scale, bias, zero_after, nbt);
}

// ----------------------------------------------------------------------------- forward apply
// Each block owns a contiguous tile of kApplyU * rpb rows; a thread issues the loads of its
// kApplyU rows before any arithmetic (two 16-B loads per stream in flight instead of one).
// tools/r2/bnlab.hip at ResNet-50 b256 shapes: 5.3 -> 5.7-6.1 TB/s vs the grid-stride loop with
// one row in flight (4-8 rows per thread measured no better, grid-strided rows worse).
constexpr int kApplyU = 2;

template <int RES, class T, int U = kApplyU>  // RES: 0 none, 1 raw residual, 2 BN'd residual
__global__ __launch_bounds__(256) void bn_act_fwd_kernel(const T* __restrict__ y,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ bias,
                                                         const T* __restrict__ r,
                                                         const float* __restrict__ rscale,
                                                         const float* __restrict__ rbias,
                                                         T* __restrict__ z, long M, int C,
                                                         bool relu,
                                                         uint8_t* __restrict__ mask, bool nt,
                                                         bool ntl) {
  const RowMap mp = row_map(C);
  const int t = threadIdx.x;
  const int rg = t / mp.tpr;
  if (rg >= mp.rpb) return;
  const long row0 = (long)blockIdx.x * mp.rpb * U + rg;
  for (int pass = 0; pass < mp.passes; ++pass) {
    const int cg = pass * mp.tpr + (t % mp.tpr);
    if (cg * 8 >= C) continue;
    const int c0 = cg * 8;
    Raw8<T> ry[U], rr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long off = min(row0 + (long)u * mp.rpb, M - 1) * C + c0;
      ry[u] = ld_raw8(y + off, ntl);
      if (RES != 0) rr[u] = ld_raw8(r + off, ntl);
    }
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
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long row = row0 + (long)u * mp.rpb;
      if (row >= M) break;
      const long off = row * C + c0;
      float v[8];
      unpack_raw(ry[u], v);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = v[q] * sc[q] + bi[q];
      if (RES != 0) {
        float w[8];
        unpack_raw(rr[u], w);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] += (RES == 2) ? (w[q] * rs[q] + rb[q]) : w[q];
      }
      if (relu) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
      }
      if (mask != nullptr) {  // 1 bit per element of the STORED z: the backward's ReLU mask
        uint32_t bits = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) bits |= (as_stored<T>(v[q]) > 0.f ? 1u : 0u) << q;
        mask[row * (C / 8) + cg] = (uint8_t)bits;
      }
      store8(z + off, v, nt);
    }
  }
}

inline int grid_for_tiles(long M, int rpb, int u = kApplyU) {
  return (int)std::max<long>(1, (M + (long)rpb * u - 1) / ((long)rpb * u));
}
// rows in flight per thread of the BN apply passes (MIPIPE_BN_U = 2 or 4; A/B knob)
static int bn_u() {
  static const int u = [] {
    const char* v = getenv("MIPIPE_BN_U");
    return v != nullptr && atoi(v) == 4 ? 4 : 2;
  }();
  return u;
}

template <class T>
static void bn_act_fwd_t(const void* y, const float* scale, const float* bias, const void* r,
                         const float* rscale, const float* rbias, void* z, long M, int C,
                         bool relu, hipStream_t st, uint8_t* mask) {
  RowMap mp = row_map(C);
  const int u = bn_u();
  int grid = grid_for_tiles(M, mp.rpb, u);
  const bool nt = (g_nt_store & 4) != 0;  // BN forward apply
  const bool ntl = (g_nt_store & 32) != 0;  // its loads streaming
  const T* yp = (const T*)y;
  const T* rp = (const T*)r;
  T* zp = (T*)z;
  if (r == nullptr)
    {
      if (u == 4) hipLaunchKernelGGL((bn_act_fwd_kernel<0, T, 4>), dim3(grid), dim3(256), 0, st, yp, scale, bias, rp, rscale, rbias, zp, M, C, relu, mask, nt, ntl);
      else hipLaunchKernelGGL((bn_act_fwd_kernel<0, T>), dim3(grid), dim3(256), 0, st, yp, scale, bias, rp, rscale, rbias, zp, M, C, relu, mask, nt, ntl);
    }
  else if (rscale == nullptr)
    {
      if (u == 4) hipLaunchKernelGGL((bn_act_fwd_kernel<1, T, 4>), dim3(grid), dim3(256), 0, st, yp, scale, bias, rp, rscale, rbias, zp, M, C, relu, mask, nt, ntl);
      else hipLaunchKernelGGL((bn_act_fwd_kernel<1, T>), dim3(grid), dim3(256), 0, st, yp, scale, bias, rp, rscale, rbias, zp, M, C, relu, mask, nt, ntl);
    }
  else
    {
      if (u == 4) hipLaunchKernelGGL((bn_act_fwd_kernel<2, T, 4>), dim3(grid), dim3(256), 0, st, yp, scale, bias, rp, rscale, rbias, zp, M, C, relu, mask, nt, ntl);
      else hipLaunchKernelGGL((bn_act_fwd_kernel<2, T>), dim3(grid), dim3(256), 0, st, yp, scale, bias, rp, rscale, rbias, zp, M, C, relu, mask, nt, ntl);
    }
}

void bn_act_fwd(const void* y, const float* scale, const float* bias, const void* r,
                const float* rscale, const float* rbias, void* z, long M, int C, bool relu,
                hipStream_t st, bool f32, uint8_t* mask) {
  if (f32) bn_act_fwd_t<float>(y, scale, bias, r, rscale, rbias, z, M, C, relu, st, mask);
  else bn_act_fwd_t<__bf16>(y, scale, bias, r, rscale, rbias, z, M, C, relu, st, mask);
}

// ----------------------------------------------------------------------------- backward
template <bool TWO, class T>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const T* __restrict__ dz, const T* __restrict__ z, const T* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const T* __restrict__ y2, const float* __restrict__ mean2,
    const float* __restrict__ invstd2, bool relu, long M, int C, float* __restrict__ rep,
    int det_rows) {
  __shared__ float red[3][kT][8];
  const RowMap mp = row_map(C);
  const int t = threadIdx.x;
  const int rg = t / mp.tpr;
  const bool active = rg < mp.rpb;
  // atomic mode: replica row blockIdx % R of [3][R][C]; deterministic: row blockIdx of
  // [3][det_rows][C], written (one writer per element)
  float* rrow = rep + (long)(det_rows > 0 ? blockIdx.x : blockIdx.x % kStatReplicas) * C;
  const long rstride = (long)(det_rows > 0 ? det_rows : kStatReplicas) * C;
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
        is[q] = invstd != nullptr ? invstd[c0 + q] : 1.f;
        if (TWO) {
          mu2[q] = mean2[c0 + q];
          is2[q] = invstd2[c0 + q];
        }
      }
      const long stride = (long)gridDim.x * mp.rpb;
      for (long row0 = (long)blockIdx.x * mp.rpb + rg; row0 < M; row0 += kRowU * stride) {
        Raw8<T> rg_[kRowU], rz[kRowU], ry[kRowU], ry2[kRowU];
#pragma unroll
        for (int u = 0; u < kRowU; ++u) {
          const long off = min(row0 + u * stride, M - 1) * C + c0;
          rg_[u] = ld_raw8(dz + off);
          if (relu) rz[u] = ld_raw8(z + off);
          ry[u] = ld_raw8(y + off);
          if (TWO) ry2[u] = ld_raw8(y2 + off);
        }
#pragma unroll
        for (int u = 0; u < kRowU; ++u) {
          if (row0 + u * stride >= M) break;
          float g[8], yv[8];
          unpack_raw(rg_[u], g);
          if (relu) {
            float zv[8];
            unpack_raw(rz[u], zv);
#pragma unroll
            for (int q = 0; q < 8; ++q) g[q] = zv[q] > 0.f ? g[q] : 0.f;
          }
          unpack_raw(ry[u], yv);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            sg[q] += g[q];
            sx[q] += g[q] * (yv[q] - mu[q]) * is[q];
          }
          if (TWO) {
            float y2v[8];
            unpack_raw(ry2[u], y2v);
#pragma unroll
            for (int q = 0; q < 8; ++q) sx2[q] += g[q] * (y2v[q] - mu2[q]) * is2[q];
          }
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
    // transpose through LDS so each atomic wave-instruction covers 64 consecutive channels
    const int cpass = min(C - pass * mp.tpr * 8, mp.tpr * 8);
    for (int c = t; c < cpass; c += kT) {
      const int owner = c >> 3, q = c & 7;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f;
      for (int k = 0; k < mp.rpb; ++k) {
        a0 += red[0][k * mp.tpr + owner][q];
        a1 += red[1][k * mp.tpr + owner][q];
        if (TWO) a2 += red[2][k * mp.tpr + owner][q];
      }
      const int cc = pass * mp.tpr * 8 + c;
      if (det_rows > 0) {
        rrow[cc] = a0;
        rrow[rstride + cc] = a1;
        if (TWO) rrow[2 * rstride + cc] = a2;
      } else {
        atomicAdd(rrow + cc, a0);
        atomicAdd(rrow + rstride + cc, a1);
        if (TWO) atomicAdd(rrow + 2 * rstride + cc, a2);
      }
    }
    __syncthreads();
  }
}

// Sum the replica rows into the outputs and zero the replicas for reuse.  Optionally also
// ACCUMULATE the parameter gradients (dβ = Σg, dγ = Σg·x̂; dβ₂ = Σg, dγ₂ = Σg·x̂₂) straight into
// the flat gradient buffer, replacing autograd's AccumulateGrad kernels.
__global__ void bn_bwd_collect_kernel(float* __restrict__ rep, int C, float* og, float* ogx,
                                      float* ogx2, float* dgamma, float* dbeta, float* dgamma2,
                                      float* dbeta2, const float* gx_div) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const long rs = (long)kStatReplicas * C;
  float va[kStatReplicas], vb[kStatReplicas], vd[kStatReplicas];
#pragma unroll
  for (int r = 0; r < kStatReplicas; ++r) {  // all loads first: one memory latency
    long o = (long)r * C + c;
    va[r] = rep[o];
    vb[r] = rep[rs + o];
    vd[r] = rep[2 * rs + o];
  }
  float a = 0.f, b = 0.f, d = 0.f;
#pragma unroll
  for (int r = 0; r < kStatReplicas; ++r) {
    long o = (long)r * C + c;
    a += va[r];
    b += vb[r];
    d += vd[r];
    rep[o] = 0.f;
    rep[rs + o] = 0.f;
    rep[2 * rs + o] = 0.f;
  }
  if (gx_div != nullptr) {  // Σg·(z-β) -> Σg·x̂ = Σg·(z-β)/γ (x̂ recovered from the BN output)
    const float gd = gx_div[c];
    b = fabsf(gd) > 1e-30f ? b / gd : 0.f;
  }
  og[c] = a;
  ogx[c] = b;
  if (ogx2 != nullptr) ogx2[c] = d;
  if (dgamma != nullptr) {
    dgamma[c] += b;
    dbeta[c] += a;
  }
  if (dgamma2 != nullptr) {
    dgamma2[c] += d;
    dbeta2[c] += a;
  }
}

// bn_bwd_collect of P partial rows ([2|3][P][C], the deterministic mode's one row per block of
// the producing reduction) instead of a replica slab: rows summed in det_sum_rows' order
// (rows_sum16, chunk sums in place first for P > 256) — the bits of det_sum_rows into a zeroed
// slab followed by bn_bwd_collect_kernel, without the extra launches.
__global__ __launch_bounds__(1024) void bn_bwd_collect_rows_kernel(
    float* __restrict__ in, int P, int C, int stride, long as, bool two, float* og, float* ogx,
    float* ogx2, float* dgamma, float* dbeta, float* dgamma2, float* dbeta2, const float* gx_div) {
  __shared__ float part[3][16][65];
  const int lc = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lc;
  float a[3] = {0.f, 0.f, 0.f};
  const long rs = (long)stride * C;
  if (c < C) {
    if (two) {
      float* const src[3] = {in, in + as, in + 2 * as};
      rows_sum16<3>(src, P, rs, c, g, a);
    } else {
      float* const src[2] = {in, in + as};
      float a2[2];
      rows_sum16<2>(src, P, rs, c, g, a2);
      a[0] = a2[0];
      a[1] = a2[1];
    }
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) part[k][g][lc] = a[k];
  __syncthreads();
  if (g != 0 || c >= C) return;
  float sa = 0.f, sb = 0.f, sd = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    sa += part[0][k][lc];
    sb += part[1][k][lc];
    sd += part[2][k][lc];
  }
  if (gx_div != nullptr) {  // Σg·(z-β) -> Σg·x̂ = Σg·(z-β)/γ (as bn_bwd_collect_kernel)
    const float gd = gx_div[c];
    sb = fabsf(gd) > 1e-30f ? sb / gd : 0.f;
  }
  og[c] = sa;
  ogx[c] = sb;
  if (ogx2 != nullptr) ogx2[c] = sd;
  if (dgamma != nullptr) {
    dgamma[c] += sb;
    dbeta[c] += sa;
  }
  if (dgamma2 != nullptr) {
    dgamma2[c] += sd;
    dbeta2[c] += sa;
  }
}

void bn_bwd_collect_rows(float* rows, int P, int C, bool two, float* out_g, float* out_gx,
                         float* out_gx2, float* dgamma, float* dbeta, float* dgamma2,
                         float* dbeta2, const float* gx_div, hipStream_t st) {
  const long as = (long)P * C;  // array stride of the [2|3][P][C] rows
  int stride = 1;
  if (P > 4 * kDetChunkRows) {
    const int n = det_chunk_sums(rows, rows + as, two ? rows + 2 * as : nullptr, P, C, st);
    P = n;
    stride = kDetChunkRows;
  }
  hipLaunchKernelGGL(bn_bwd_collect_rows_kernel, dim3((C + 63) / 64), dim3(1024), 0, st, rows, P,
                     C, stride, as, two, out_g, out_gx, out_gx2, dgamma, dbeta, dgamma2, dbeta2,
                     gx_div);
}

int bn_bwd_reduce_blocks(long M, int C) {
  RowMap mp = row_map(C);
  // >= 16 row-iterations per thread, and at most ~1M atomic adds in total
  long cap = std::max<long>(64, (1l << 20) / (3l * C));
  return (int)std::max<long>(1, std::min<long>(std::min<long>(1024, cap),
                                               (M + mp.rpb * 16 - 1) / (mp.rpb * 16)));
}

void bn_act_bwd_reduce(const void* dz, const void* z, const void* y, const float* mean,
                       const float* invstd, const void* y2, const float* mean2,
                       const float* invstd2, bool relu, long M, int C, float* out_g,
                       float* out_gx, float* out_gx2, float* rep, float* dgamma, float* dbeta,
                       float* dgamma2, float* dbeta2, hipStream_t st, bool f32, float* det_ws,
                       const float* gx_div) {
  const int G = bn_bwd_reduce_blocks(M, C);
  const int det_rows = det_ws != nullptr ? G : 0;
  float* part = det_ws != nullptr ? det_ws : rep;
  auto launch = [&](auto tag) {
    typedef decltype(tag) T;
      const T *dzp = (const T*)dz, *zp = (const T*)z, *yp = (const T*)y, *y2p = (const T*)y2;
    if (y2 == nullptr)
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<false, T>), dim3(G), dim3(256), 0, st, dzp, zp, yp, mean, invstd, y2p, mean2, invstd2, relu, M, C, part, det_rows);
    else
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<true, T>), dim3(G), dim3(256), 0, st, dzp, zp, yp, mean, invstd, y2p, mean2, invstd2, relu, M, C, part, det_rows);
  };
  if (f32) launch(float{});
  else launch(__bf16{});
  if (det_ws != nullptr) {
    // the G per-block rows collected in det_sum_rows' fixed order by one launch (the replica
    // slab is not touched)
    bn_bwd_collect_rows(det_ws, G, C, y2 != nullptr, out_g, out_gx, y2 ? out_gx2 : nullptr,
                        dgamma, dbeta, y2 ? dgamma2 : nullptr, y2 ? dbeta2 : nullptr, gx_div, st);
    return;
  }
  hipLaunchKernelGGL(bn_bwd_collect_kernel, dim3((C + 255) / 256), dim3(256), 0, st, rep, C, out_g,
                     out_gx, y2 ? out_gx2 : nullptr, dgamma, dbeta, y2 ? dgamma2 : nullptr,
                     y2 ? dbeta2 : nullptr, gx_div);
}

template <int MODE, class T, int U = kApplyU>  // MODE 0: dy only, 1: dy + dres (=g), 2: dy + dy2 (second branch)
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const T* __restrict__ dz, const T* __restrict__ z, const T* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ sum_g,
    const float* __restrict__ sum_gx, const T* __restrict__ y2,
    const float* __restrict__ mean2, const float* __restrict__ invstd2,
    const float* __restrict__ gamma2, const float* __restrict__ sum_gx2, float inv_n, bool relu,
    T* __restrict__ dy, T* __restrict__ dother, long M, int C, bool nt, bool ntl) {
  const RowMap mp = row_map(C);
  const int t = threadIdx.x;
  const int rg = t / mp.tpr;
  if (rg >= mp.rpb) return;
  const long row0 = (long)blockIdx.x * mp.rpb * U + rg;
  for (int pass = 0; pass < mp.passes; ++pass) {
    const int cg = pass * mp.tpr + (t % mp.tpr);
    const int c0 = cg * 8;
    if (c0 >= C) continue;
    Raw8<T> rgv[U], rz[U], ry[U], ry2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long off = min(row0 + (long)u * mp.rpb, M - 1) * C + c0;
      rgv[u] = ld_raw8(dz + off, ntl);
      if (relu) rz[u] = ld_raw8(z + off, ntl);
      ry[u] = ld_raw8(y + off, ntl);
      if (MODE == 2) ry2[u] = ld_raw8(y2 + off, ntl);
    }
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
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long row = row0 + (long)u * mp.rpb;
      if (row >= M) break;
      const long off = row * C + c0;
      float g[8], yv[8], o[8];
      unpack_raw(rgv[u], g);
      if (relu) {
        float zv[8];
        unpack_raw(rz[u], zv);
#pragma unroll
        for (int q = 0; q < 8; ++q) g[q] = zv[q] > 0.f ? g[q] : 0.f;
      }
      unpack_raw(ry[u], yv);
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = A[q] * g[q] + Bc[q] * yv[q] + Cc[q];
      store8(dy + off, o, nt);
      if (MODE == 1) {
        store8(dother + off, g, nt);
      } else if (MODE == 2) {
        float y2v[8];
        unpack_raw(ry2[u], y2v);
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = A2[q] * g[q] + B2[q] * y2v[q] + C2[q];
        store8(dother + off, o, nt);
      }
    }
  }
}

void bn_act_bwd_apply(const void* dz, const void* z, const void* y, const float* mean,
                      const float* invstd, const float* gamma, const float* sum_g,
                      const float* sum_gx, const void* y2, const float* mean2,
                      const float* invstd2, const float* gamma2, const float* sum_gx2, long count,
                      bool relu, bool want_dres, void* dy, void* dother, long M, int C,
                      hipStream_t st, bool f32) {
  RowMap mp = row_map(C);
  const bool nt = (g_nt_store & 8) != 0;  // BN backward apply
  const bool ntl = (g_nt_store & 64) != 0;  // its loads streaming
  const int u = bn_u();
  int grid = grid_for_tiles(M, mp.rpb, u);
  float inv_n = 1.f / (float)count;
  auto launch = [&](auto tag) {
    typedef decltype(tag) T;
      const T *dzp = (const T*)dz, *zp = (const T*)z, *yp = (const T*)y, *y2p = (const T*)y2;
    T *dyp = (T*)dy, *dop = (T*)dother;
    if (y2 != nullptr)
      {
        if (u == 4) hipLaunchKernelGGL((bn_bwd_apply_kernel<2, T, 4>), dim3(grid), dim3(256), 0, st, dzp, zp, yp, mean, invstd, gamma, sum_g, sum_gx, y2p, mean2, invstd2, gamma2, sum_gx2, inv_n, relu, dyp, dop, M, C, nt, ntl);
        else hipLaunchKernelGGL((bn_bwd_apply_kernel<2, T>), dim3(grid), dim3(256), 0, st, dzp, zp, yp, mean, invstd, gamma, sum_g, sum_gx, y2p, mean2, invstd2, gamma2, sum_gx2, inv_n, relu, dyp, dop, M, C, nt, ntl);
      }
    else if (want_dres)
      {
        if (u == 4) hipLaunchKernelGGL((bn_bwd_apply_kernel<1, T, 4>), dim3(grid), dim3(256), 0, st, dzp, zp, yp, mean, invstd, gamma, sum_g, sum_gx, y2p, mean2, invstd2, gamma2, sum_gx2, inv_n, relu, dyp, dop, M, C, nt, ntl);
        else hipLaunchKernelGGL((bn_bwd_apply_kernel<1, T>), dim3(grid), dim3(256), 0, st, dzp, zp, yp, mean, invstd, gamma, sum_g, sum_gx, y2p, mean2, invstd2, gamma2, sum_gx2, inv_n, relu, dyp, dop, M, C, nt, ntl);
      }
    else
      {
        if (u == 4) hipLaunchKernelGGL((bn_bwd_apply_kernel<0, T, 4>), dim3(grid), dim3(256), 0, st, dzp, zp, yp, mean, invstd, gamma, sum_g, sum_gx, y2p, mean2, invstd2, gamma2, sum_gx2, inv_n, relu, dyp, dop, M, C, nt, ntl);
        else hipLaunchKernelGGL((bn_bwd_apply_kernel<0, T>), dim3(grid), dim3(256), 0, st, dzp, zp, yp, mean, invstd, gamma, sum_g, sum_gx, y2p, mean2, invstd2, gamma2, sum_gx2, inv_n, relu, dyp, dop, M, C, nt, ntl);
      }
  };
  if (f32) launch(float{});
  else launch(__bf16{});
}

void bn_bwd_collect(float* rep, int C, float* out_g, float* out_gx, float* dgamma, float* dbeta,
                    hipStream_t st) {
  hipLaunchKernelGGL(bn_bwd_collect_kernel, dim3((C + 255) / 256), dim3(256), 0, st, rep, C, out_g,
                     out_gx, nullptr, dgamma, dbeta, nullptr, nullptr, nullptr);
}

}  // namespace mipipe
