// Memory-bound kernels of the training step: fused cross-entropy (fwd+bwd in one pass over
// the logits), flat-buffer SGD-momentum / AdamW (one launch for the whole model, also emitting
// the bf16 weight shadow), NCHW->NHWC input conversion, on-device synthetic data, GELU,
// LayerNorm, embedding-grad scatter and column sums.  16-B vector accesses throughout
// (cdna_hip_programming.md Guideline 13).
#include "common.hpp"
#include "launchers.hpp"

namespace mipipe {

static int grid1d(long work, int per_thread = 1, int cap = 8192) {
  long g = (work / per_thread + 255) / 256;
  return (int)std::max<long>(1, std::min<long>(g, cap));
}

// ------------------------------------------------------------------------------ cross-entropy
__global__ void ce_count_kernel(const int64_t* __restrict__ labels, int R, int64_t ignore,
                                int* __restrict__ out) {
  __shared__ int red[256];
  int c = 0;
  for (int i = threadIdx.x; i < R; i += 256) c += labels[i] != ignore;
  red[threadIdx.x] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

__device__ __forceinline__ float block_reduce(float v, float* sh, bool is_max) {
  v = is_max ? wave_max(v) : wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float r = sh[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = is_max ? fmaxf(r, sh[i]) : r + sh[i];
  return r;
}

// one block per row; logits T (bf16 / fp32) [R][V] of which the first Vv columns are classes
// (the rest: tile padding of the vocabulary, excluded from the softmax, gradient 0)
template <class T>
__global__ __launch_bounds__(256) void ce_kernel(const T* __restrict__ logits,
                                                 const int64_t* __restrict__ labels,
                                                 float* __restrict__ loss, T* __restrict__ grad,
                                                 int V, int Vv, float eps, int64_t ignore,
                                                 const int* __restrict__ nvalid,
                                                 float* __restrict__ rowloss) {
  __shared__ float sh[8];
  const long row = blockIdx.x;
  const T* x = logits + row * V;
  T* g = grad + row * V;
  const int64_t lab = labels[row];
  const bool valid = lab != ignore;
  const bool vec = (V % 8) == 0;
  float mx = -INFINITY, sx = 0.f;
  if (vec) {
    for (int c = threadIdx.x; c < V / 8; c += 256) {
      float v[8];
      load8(x + c * 8, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (c * 8 + q < Vv) {
          mx = fmaxf(mx, v[q]);
          sx += v[q];
        }
      }
    }
  } else {
    for (int c = threadIdx.x; c < Vv; c += 256) {
      float v = (float)x[c];
      mx = fmaxf(mx, v);
      sx += v;
    }
  }
  mx = block_reduce(mx, sh, true);
  sx = block_reduce(sx, sh, false);
  float se = 0.f;
  if (vec) {
    for (int c = threadIdx.x; c < V / 8; c += 256) {
      float v[8];
      load8(x + c * 8, v);
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (c * 8 + q < Vv) se += __expf(v[q] - mx);
    }
  } else {
    for (int c = threadIdx.x; c < Vv; c += 256) se += __expf((float)x[c] - mx);
  }
  se = block_reduce(se, sh, false);
  const float lse = mx + __logf(se);
  const float inv_n = 1.f / (float)max(1, nvalid[0]);
  if (threadIdx.x == 0) {  // summed in a fixed order by ce_sum_kernel (no float atomics)
    float l = 0.f;
    if (valid) {
      float xl = (float)x[lab];
      l = (1.f - eps) * (lse - xl) + eps * (lse - sx / (float)Vv);
    }
    rowloss[row] = l * inv_n;
  }
  const float scale = valid ? inv_n : 0.f;
  const float inv_se = 1.f / se;
  const float base_t = eps / (float)Vv;
  if (vec) {
    for (int c = threadIdx.x; c < V / 8; c += 256) {
      float v[8];
      load8(x + c * 8, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        int col = c * 8 + q;
        float t = base_t + (col == lab ? 1.f - eps : 0.f);
        v[q] = col < Vv ? (__expf(v[q] - mx) * inv_se - t) * scale : 0.f;
      }
      store8(g + c * 8, v);
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) {
      float t = base_t + (c == lab ? 1.f - eps : 0.f);
      g[c] = (T)(c < Vv ? (__expf((float)x[c] - mx) * inv_se - t) * scale : 0.f);
    }
  }
}

// loss = sum of the per-row losses in a fixed order (thread t: rows t, t+256, ...; then a tree)
__global__ __launch_bounds__(256) void ce_sum_kernel(const float* __restrict__ rowloss, int R,
                                                     float* __restrict__ loss) {
  __shared__ float red[256];
  float a = 0.f;
  for (int i = threadIdx.x; i < R; i += 256) a += rowloss[i];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = red[0];
}

void cross_entropy_fwd_bwd(const void* logits, const int64_t* labels, float* loss, void* grad,
                           int R, int V, float smoothing, int64_t ignore_index, int* work,
                           hipStream_t st, bool f32, int Vv) {
  if (Vv <= 0 || Vv > V) Vv = V;
  float* rowloss = reinterpret_cast<float*>(work + 4);
  hipLaunchKernelGGL(ce_count_kernel, dim3(1), dim3(256), 0, st, labels, R, ignore_index, work);
  if (f32)
    hipLaunchKernelGGL(ce_kernel<float>, dim3(R), dim3(256), 0, st, (const float*)logits, labels,
                       loss, (float*)grad, V, Vv, smoothing, ignore_index, (const int*)work, rowloss);
  else
    hipLaunchKernelGGL(ce_kernel<__bf16>, dim3(R), dim3(256), 0, st, (const __bf16*)logits, labels,
                       loss, (__bf16*)grad, V, Vv, smoothing, ignore_index, (const int*)work, rowloss);
  hipLaunchKernelGGL(ce_sum_kernel, dim3(1), dim3(256), 0, st, rowloss, R, loss);
}

// Split form for the training step: the forward keeps only the per-row log-sum-exp (one pass
// over the logits: running max and rescaled exp-sum per thread, merged per wave and block), the
// backward writes grad = (softmax - target) * g / n straight from the logits with the upstream
// gradient g read on the device — so no [R][V] gradient is written in the forward and then
// rescaled by a separate elementwise pass (BERT-base MLM: 640 x 30528 logits).
__device__ __forceinline__ void lse_merge(float& m, float& s, float mo, float so) {
  const float mn = fmaxf(m, mo);
  if (mn == -INFINITY) return;  // both empty
  s = s * __expf(m - mn) + so * __expf(mo - mn);
  m = mn;
}

template <class T>
__global__ __launch_bounds__(256) void ce_fwd_kernel(const T* __restrict__ logits,
                                                     const int64_t* __restrict__ labels, int V,
                                                     int Vv, float eps, int64_t ignore,
                                                     const int* __restrict__ nvalid,
                                                     float* __restrict__ rowloss,
                                                     float* __restrict__ lse_out) {
  __shared__ float sh[3][4];
  const long row = blockIdx.x;
  const T* x = logits + row * V;
  float m = -INFINITY, s = 0.f, sx = 0.f;
  if ((V % 8) == 0) {
    for (int c = threadIdx.x; c < V / 8; c += 256) {
      float v[8];
      load8(x + c * 8, v);
      float m8 = -INFINITY;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (c * 8 + q < Vv) {
          m8 = fmaxf(m8, v[q]);
          sx += v[q];
        }
      const float mn = fmaxf(m, m8);
      if (mn == -INFINITY) continue;
      float e = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (c * 8 + q < Vv) e += __expf(v[q] - mn);
      s = s * __expf(m - mn) + e;
      m = mn;
    }
  } else {
    for (int c = threadIdx.x; c < Vv; c += 256) {
      const float v = (float)x[c];
      sx += v;
      lse_merge(m, s, v, 1.f);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float mo = __shfl_xor(m, o), so = __shfl_xor(s, o);
    lse_merge(m, s, mo, so);
    sx += __shfl_xor(sx, o);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[0][w] = m;
    sh[1][w] = s;
    sh[2][w] = sx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sh[0][0], S = sh[1][0], SX = sh[2][0];
    for (int i = 1; i < 4; ++i) {
      lse_merge(M, S, sh[0][i], sh[1][i]);
      SX += sh[2][i];
    }
    const float lse = M + __logf(S);
    const int64_t lab = labels[row];
    float l = 0.f;
    if (lab != ignore)
      l = (1.f - eps) * (lse - (float)x[lab]) + eps * (lse - SX / (float)Vv);
    rowloss[row] = l / (float)max(1, nvalid[0]);
    lse_out[row] = lse;
  }
}

// grid (column blocks, rows): 8 columns per thread (V % 8 == 0) or 1
template <class T, bool VEC>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const T* __restrict__ logits,
                                                     const int64_t* __restrict__ labels,
                                                     const float* __restrict__ lse,
                                                     const int* __restrict__ nvalid,
                                                     const float* __restrict__ gout,
                                                     T* __restrict__ grad, int R, int V, int Vv,
                                                     float eps, int64_t ignore) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= (VEC ? V / 8 : V)) return;
  const float gs = gout[0] / (float)max(1, nvalid[0]), base_t = eps / (float)Vv;
  for (long row = blockIdx.y; row < R; row += gridDim.y) {  // (grid.y is capped at 65535)
  const int64_t lab = labels[row];
  const float scale = lab != ignore ? gs : 0.f;
  const float l = lse[row];
  if constexpr (VEC) {
    float v[8];
    load8(logits + row * V + c * 8, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int col = c * 8 + q;
      const float t = base_t + (col == lab ? 1.f - eps : 0.f);
      v[q] = col < Vv ? (__expf(v[q] - l) - t) * scale : 0.f;
    }
    store8(grad + row * V + c * 8, v);
  } else {
    const float t = base_t + (c == lab ? 1.f - eps : 0.f);
    grad[row * V + c] = (T)(c < Vv ? (__expf((float)logits[row * V + c] - l) - t) * scale : 0.f);
  }
  }
}

void cross_entropy_fwd(const void* logits, const int64_t* labels, float* loss, int R, int V,
                       float smoothing, int64_t ignore_index, int* work, hipStream_t st, bool f32,
                       int Vv) {
  if (Vv <= 0 || Vv > V) Vv = V;
  float* rowloss = reinterpret_cast<float*>(work + 4);
  float* lse = rowloss + R;
  hipLaunchKernelGGL(ce_count_kernel, dim3(1), dim3(256), 0, st, labels, R, ignore_index, work);
  if (f32)
    hipLaunchKernelGGL(ce_fwd_kernel<float>, dim3(R), dim3(256), 0, st, (const float*)logits,
                       labels, V, Vv, smoothing, ignore_index, (const int*)work, rowloss, lse);
  else
    hipLaunchKernelGGL(ce_fwd_kernel<__bf16>, dim3(R), dim3(256), 0, st, (const __bf16*)logits,
                       labels, V, Vv, smoothing, ignore_index, (const int*)work, rowloss, lse);
  hipLaunchKernelGGL(ce_sum_kernel, dim3(1), dim3(256), 0, st, rowloss, R, loss);
}

void cross_entropy_bwd(const void* logits, const int64_t* labels, const int* work,
                       const float* gout, void* grad, int R, int V, float smoothing,
                       int64_t ignore_index, hipStream_t st, bool f32, int Vv) {
  if (Vv <= 0 || Vv > V) Vv = V;
  const float* lse = reinterpret_cast<const float*>(work + 4) + R;
  const bool vec = V % 8 == 0;
  const dim3 g((unsigned)(((vec ? V / 8 : V) + 255) / 256), (unsigned)std::min(R, 65535));
  auto go = [&](auto t, auto vec_c) {
    using T = decltype(t);
    hipLaunchKernelGGL((ce_bwd_kernel<T, decltype(vec_c)::value>), g, dim3(256), 0, st,
                       (const T*)logits, labels, lse, work, gout, (T*)grad, R, V, Vv,
                       smoothing, ignore_index);
  };
  if (f32) {
    if (vec) go(float(), std::true_type());
    else go(float(), std::false_type());
  } else {
    if (vec) go(__bf16(), std::true_type());
    else go(__bf16(), std::false_type());
  }
}

// ------------------------------------------------------------------------------ cache warming
// One 4-B load per 64-B line of up to kTouchRanges byte ranges: brings a GEMM operand that was
// last read milliseconds ago (a weight, a saved activation) into the memory-side cache before
// its GEMM runs (mipipe/ops/prefetch.py launches it on a side stream beside the previous GEMM).
// Nothing is written: the loads feed a sum that is stored only if it equals a constant AND sink
// is non-null (never, sink is null) — which keeps the compiler from dropping them.
__global__ __launch_bounds__(256) void touch_kernel(TouchRanges r, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < kTouchRanges; ++k) {
    if (k < r.count) {
      const long lines = r.bytes[k] >> 6;
      for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < lines; i += (long)gridDim.x * 256)
        acc += *reinterpret_cast<const uint32_t*>(r.ptr[k] + (i << 6));
    }
  }
  if (acc == 0x2545F491u && sink != nullptr) sink[threadIdx.x] = acc;
}

void touch(const TouchRanges& r, hipStream_t st) {
  long lines = 0;
  for (int k = 0; k < r.count; ++k) lines = std::max(lines, r.bytes[k] >> 6);
  if (lines == 0) return;
  hipLaunchKernelGGL(touch_kernel, dim3(grid1d(lines, 1, 512)), dim3(256), 0, st, r, nullptr);
}

// ------------------------------------------------------------------------------ evaluation
// Top-1 correct count (the reference's eval loop: argmax over classes == label, summed): one
// wave per row, first maximal index wins (torch.argmax's tie rule), NaN counts as maximal; the
// per-block count is one integer atomic into *correct (order-independent, so deterministic).
template <class T>
__global__ __launch_bounds__(256) void top1_correct_kernel(const T* __restrict__ logits,
                                                           const int64_t* __restrict__ labels,
                                                           int R, int V, int* __restrict__ correct) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave;
  int hit = 0;
  if (row < R) {
    const T* x = logits + (long)row * V;
    float best = -INFINITY;
    int arg = 0x7fffffff;
    for (int c = lane; c < V; c += 64) {
      const float v = (float)x[c];
      if (v > best || (v != v && best == best)) {  // strictly greater keeps the first index
        best = v;
        arg = c;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o);
      const int oa = __shfl_xor(arg, o);
      const bool onan = ob != ob, mnan = best != best;
      if ((onan && !mnan) || (onan == mnan && (ob > best || (ob == best && oa < arg)))) {
        best = ob;
        arg = oa;
      }
    }
    hit = (lane == 0 && (int64_t)arg == labels[row]) ? 1 : 0;
  }
  __shared__ int cnt;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  if (hit) atomicAdd(&cnt, 1);
  __syncthreads();
  if (threadIdx.x == 0 && cnt) atomicAdd(correct, cnt);
}

void top1_correct(const void* logits, const int64_t* labels, int R, int V, int* correct,
                  hipStream_t st, bool f32) {
  dim3 g((R + 3) / 4);
  if (f32)
    hipLaunchKernelGGL(top1_correct_kernel<float>, g, dim3(256), 0, st, (const float*)logits, labels, R, V, correct);
  else
    hipLaunchKernelGGL(top1_correct_kernel<__bf16>, g, dim3(256), 0, st, (const __bf16*)logits, labels, R, V, correct);
}

// ------------------------------------------------------------------------------ optimizers
// SGD ([torch] optim/sgd.py:354-380): g += wd*p; m = momentum*m + (1-damp)*g (m = g first);
// p -= lr * (nesterov ? g + momentum*m : m).  Flat fp32 buffers, n % 4 == 0.
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ m, __bf16* __restrict__ sh,
                                                  long n4, float lr, float mom, float damp, float wd,
                                                  bool nesterov, bool first, float gs) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    float4 gv = reinterpret_cast<const float4*>(g)[i];
    float pa[4] = {pv.x, pv.y, pv.z, pv.w};
    float ga[4] = {gv.x * gs, gv.y * gs, gv.z * gs, gv.w * gs};
    if (mom != 0.f) {
      float4 mv = reinterpret_cast<float4*>(m)[i];
      float ma[4] = {mv.x, mv.y, mv.z, mv.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float d = ga[q] + wd * pa[q];
        ma[q] = first ? d : mom * ma[q] + (1.f - damp) * d;
        float upd = nesterov ? d + mom * ma[q] : ma[q];
        pa[q] -= lr * upd;
      }
      reinterpret_cast<float4*>(m)[i] = make_float4(ma[0], ma[1], ma[2], ma[3]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) pa[q] -= lr * (ga[q] + wd * pa[q]);
    }
    reinterpret_cast<float4*>(p)[i] = make_float4(pa[0], pa[1], pa[2], pa[3]);
    if (sh != nullptr)
      reinterpret_cast<uint2*>(sh)[i] = make_uint2(pack2(pa[0], pa[1]), pack2(pa[2], pa[3]));
  }
}

void sgd_step(float* p, const float* g, float* m, void* shadow, long n, float lr, float momentum,
              float dampening, float wd, bool nesterov, bool first, float grad_scale,
              hipStream_t st) {
  long n4 = n / 4;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid1d(n4, 4)), dim3(256), 0, st, p, g, m, (__bf16*)shadow,
                     n4, lr, momentum, dampening, wd, nesterov, first, grad_scale);
}

// ------------------------------------------------------------------------------ DDP wire format
// bf16 gradient wire (DistributedDataParallel(comm_dtype=bf16)): one pass turns a
// bucket of the flat fp32 gradient into bf16 already multiplied by 1/world, so RCCL's SUM is the
// average (no post-divide pass); one pass widens the reduced bucket back into the fp32 gradient.
// Buckets are 64-element aligned slices of the flat buffer: n % 8 == 0, 16-B aligned.
__global__ __launch_bounds__(256) void grad_pack_bf16_kernel(const float* __restrict__ g,
                                                             uint4* __restrict__ w, long n8,
                                                             float scale) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (long)gridDim.x * blockDim.x) {
    float f[8];
    load8(g + i * 8, f);
#pragma unroll
    for (int q = 0; q < 8; ++q) f[q] *= scale;
    w[i] = pack8(f);
  }
}

__global__ __launch_bounds__(256) void grad_unpack_bf16_kernel(const uint4* __restrict__ w,
                                                               float* __restrict__ g, long n8) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (long)gridDim.x * blockDim.x) {
    float f[8];
    unpack8(w[i], f);
    float4* o = reinterpret_cast<float4*>(g + i * 8);
    o[0] = make_float4(f[0], f[1], f[2], f[3]);
    o[1] = make_float4(f[4], f[5], f[6], f[7]);
  }
}

void grad_pack_bf16(const float* g, void* wire, long n, float scale, hipStream_t st) {
  const long n8 = n / 8;
  if (n8 == 0) return;
  hipLaunchKernelGGL(grad_pack_bf16_kernel, dim3(grid1d(n8, 4)), dim3(256), 0, st, g,
                     (uint4*)wire, n8, scale);
}

void grad_unpack_bf16(const void* wire, float* g, long n, hipStream_t st) {
  const long n8 = n / 8;
  if (n8 == 0) return;
  hipLaunchKernelGGL(grad_unpack_bf16_kernel, dim3(grid1d(n8, 4)), dim3(256), 0, st,
                     (const uint4*)wire, g, n8);
}

// NT: streaming (non-temporal) loads / stores of the fp32 state (p, g, m, v: 16 B per parameter
// each, touched once per step); the bf16 shadow the next forward reads stays cached
template <bool NT>
__device__ __forceinline__ float4 ldf4(const float* p, long i) {
  if constexpr (NT) {
    typedef __attribute__((ext_vector_type(4))) float f4;
    const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p) + i);
    return make_float4(v.x, v.y, v.z, v.w);
  } else {
    return reinterpret_cast<const float4*>(p)[i];
  }
}
template <bool NT>
__device__ __forceinline__ void stf4(float* p, long i, float a, float b, float c, float d) {
  if constexpr (NT) {
    typedef __attribute__((ext_vector_type(4))) float f4;
    __builtin_nontemporal_store(f4{a, b, c, d}, reinterpret_cast<f4*>(p) + i);
  } else {
    reinterpret_cast<float4*>(p)[i] = make_float4(a, b, c, d);
  }
}

// U float4 items per thread per iteration (items i, i + stride, ...): every item's four loads
// are issued before any is used — U x 64 B of each thread in flight
template <bool NT, int U>
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    __bf16* __restrict__ sh, long n4, float lr,
                                                    float b1, float b2, float eps, float wd,
                                                    float bc1, float bc2, float gs,
                                                    const int* __restrict__ t_dev) {
  if (t_dev != nullptr) {  // step count on the device: graph-replayable bias correction
    const float t = (float)__hip_atomic_load(t_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bc1 = 1.f - exp2f(t * log2f(b1));
    bc2 = 1.f - exp2f(t * log2f(b2));
  }
  const float rbc2 = rsqrtf(bc2);
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x; i0 < n4; i0 += stride * U) {
    float4 pv[U], gv[U], mv[U], vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      if (u == 0 || i < n4) {
        pv[u] = ldf4<NT>(p, i);
        gv[u] = ldf4<NT>(g, i);
        mv[u] = ldf4<NT>(m, i);
        vv[u] = ldf4<NT>(v, i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      if (u > 0 && i >= n4) break;
      float pa[4] = {pv[u].x, pv[u].y, pv[u].z, pv[u].w}, ga[4] = {gv[u].x, gv[u].y, gv[u].z, gv[u].w};
      float ma[4] = {mv[u].x, mv[u].y, mv[u].z, mv[u].w}, va[4] = {vv[u].x, vv[u].y, vv[u].z, vv[u].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float gq = ga[q] * gs;
        pa[q] *= 1.f - lr * wd;
        ma[q] = b1 * ma[q] + (1.f - b1) * gq;
        va[q] = b2 * va[q] + (1.f - b2) * gq * gq;
        float denom = sqrtf(va[q]) * rbc2 + eps;
        pa[q] -= (lr / bc1) * ma[q] / denom;
      }
      stf4<NT>(p, i, pa[0], pa[1], pa[2], pa[3]);
      stf4<NT>(m, i, ma[0], ma[1], ma[2], ma[3]);
      stf4<NT>(v, i, va[0], va[1], va[2], va[3]);
      if (sh != nullptr)
        reinterpret_cast<uint2*>(sh)[i] = make_uint2(pack2(pa[0], pa[1]), pack2(pa[2], pa[3]));
    }
  }
}

void adamw_step(float* p, const float* g, float* m, float* v, void* shadow, long n, float lr,
                float b1, float b2, float eps, float wd, float bc1, float bc2, float grad_scale,
                hipStream_t st, const int* t_dev) {
  long n4 = n / 4;
  // 32768 blocks: 5.10 TB/s at BERT-base size vs 4.63 with the default 8192 cap (more waves in
  // flight per SIMD; tools/r3/adamw_lab.hip, profiles/r3_bert_gemm_splitk_adamw.txt)
  static const int cap = [] {
    const char* e = getenv("MIPIPE_ADAMW_BLOCKS");
    return e == nullptr ? 32768 : atoi(e);
  }();
  // MIPIPE_ADAMW_UNROLL: float4 items in flight per thread (1, 2 or 4); 2 measured +0.7 % on
  // BERT-base over 1 (profiles/r6_adamw_unroll.txt)
  static const int unroll = [] {
    const char* e = getenv("MIPIPE_ADAMW_UNROLL");
    const int u = e != nullptr ? atoi(e) : 2;
    return u == 4 ? 4 : u == 1 ? 1 : 2;
  }();
  auto go = [&](auto nt_c, auto u_c) {
    constexpr bool NT = decltype(nt_c)::value;
    constexpr int U = decltype(u_c)::value;
    hipLaunchKernelGGL((adamw_kernel<NT, U>), dim3(grid1d(n4, U, cap)), dim3(256), 0, st, p, g,
                       m, v, (__bf16*)shadow, n4, lr, b1, b2, eps, wd, bc1, bc2, grad_scale, t_dev);
  };
  const bool nt = (g_nt_store & 1024) != 0;
  if (unroll == 4) {
    if (nt) go(std::true_type(), std::integral_constant<int, 4>());
    else go(std::false_type(), std::integral_constant<int, 4>());
  } else if (unroll == 2) {
    if (nt) go(std::true_type(), std::integral_constant<int, 2>());
    else go(std::false_type(), std::integral_constant<int, 2>());
  } else {
    if (nt) go(std::true_type(), std::integral_constant<int, 1>());
    else go(std::false_type(), std::integral_constant<int, 1>());
  }
}

// ------------------------------------------------------------------------------ layout / data
// x [N][C][H][W] (fp32 or bf16) -> y [N][H][W][Cp] T (channels >= C zero)
template <bool BF16IN, class T>
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const void* __restrict__ xin,
                                                           T* __restrict__ y, int N, int C,
                                                           int H, int W, int Cp) {
  long total = (long)N * H * W;
  long hw = (long)H * W;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    long n = t / hw, pix = t % hw;
    for (int c0 = 0; c0 < Cp; c0 += 8) {
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {  // unconditional loads (clamped channel), padding selected
        const int c = c0 + q;
        const long src = (n * C + (c < C ? c : C - 1)) * hw + pix;
        const float x = BF16IN ? (float)reinterpret_cast<const __bf16*>(xin)[src]
                               : reinterpret_cast<const float*>(xin)[src];
        v[q] = c < C ? x : 0.f;
      }
      store8(y + t * Cp + c0, v);
    }
  }
}

void nchw_to_nhwc(const void* x, bool x_is_bf16, void* y, int N, int C, int H, int W, int Cp,
                  hipStream_t st, bool y_f32) {
  long total = (long)N * H * W;
  dim3 g(grid1d(total));
  if (y_f32) {
    if (x_is_bf16) hipLaunchKernelGGL((nchw_to_nhwc_kernel<true, float>), g, dim3(256), 0, st, x, (float*)y, N, C, H, W, Cp);
    else hipLaunchKernelGGL((nchw_to_nhwc_kernel<false, float>), g, dim3(256), 0, st, x, (float*)y, N, C, H, W, Cp);
  } else {
    if (x_is_bf16) hipLaunchKernelGGL((nchw_to_nhwc_kernel<true, __bf16>), g, dim3(256), 0, st, x, (__bf16*)y, N, C, H, W, Cp);
    else hipLaunchKernelGGL((nchw_to_nhwc_kernel<false, __bf16>), g, dim3(256), 0, st, x, (__bf16*)y, N, C, H, W, Cp);
  }
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA77u;
  x ^= x >> 13;
  x *= 0xC2B2AE3Du;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ float u01(uint32_t h) { return ((float)(h >> 8) + 0.5f) * (1.f / 16777216.f); }

// Same hash / Box-Muller as mipipe.data.synthetic.synthetic_batch (CPU reference).
__global__ __launch_bounds__(256) void synthetic_kernel(const int64_t* __restrict__ idx, int n,
                                                        int P, int classes, int seed,
                                                        void* __restrict__ x, bool bf16_out,
                                                        int64_t* __restrict__ labels) {
  long total = (long)n * P;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    int i = (int)(t / P);
    uint32_t pos = (uint32_t)(t % P);
    uint32_t id = (uint32_t)idx[i];
    uint32_t lab = mix32(id * 0x9E3779B1u + (uint32_t)seed * 7919u + 17u) % (uint32_t)classes;
    if (pos == 0) labels[i] = lab;
    uint32_t tk = mix32(lab * 0x27D4EB2Fu + pos * 0x9E3779B1u + (uint32_t)seed * 31u + 1u);
    float t1 = u01(tk), t2 = u01(mix32(tk + 0x165667B1u));
    float templ = sqrtf(-2.f * logf(t1)) * cosf(6.283185307179586f * t2);
    uint32_t nk = mix32(id * 0x632BE5ABu + pos * 0x85EBCA77u + (uint32_t)seed * 131u + 7u);
    float u1 = u01(nk), u2 = u01(mix32(nk + 0x27D4EB2Fu));
    float noise = sqrtf(-2.f * logf(u1)) * cosf(6.283185307179586f * u2);
    float v = 0.5f * templ + noise;
    if (bf16_out) reinterpret_cast<__bf16*>(x)[t] = (__bf16)v;
    else reinterpret_cast<float*>(x)[t] = v;
  }
}

void synthetic_batch(const int64_t* idx, int n, int C, int H, int W, int classes, int seed,
                     void* x, bool bf16_out, int64_t* labels, hipStream_t st) {
  int P = C * H * W;
  hipLaunchKernelGGL(synthetic_kernel, dim3(grid1d((long)n * P)), dim3(256), 0, st, idx, n, P,
                     classes, seed, x, bf16_out, labels);
}

// ------------------------------------------------------------------------------ GELU (erf)
__global__ __launch_bounds__(256) void gelu_fwd_kernel(const __bf16* __restrict__ x,
                                                       __bf16* __restrict__ y, long n8) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (long)gridDim.x * blockDim.x) {
    float v[8];
    unpack8(reinterpret_cast<const uint4*>(x)[i], v);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = gelu_erf(v[q]);
    reinterpret_cast<uint4*>(y)[i] = pack8(v);
  }
}

// gelu'(v) = Φ(v) + v·φ(v).  Φ through erfc(|v|/√2) = poly(t)·exp(-v²/2), t = 1/(1 + p|v|/√2)
// (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7) sharing φ's exponential: one exp and one
// reciprocal per element instead of libm's erff, so the backward pass stays HBM-bound.
__device__ __forceinline__ float gelu_grad(float v) {
  const float e = __expf(-0.5f * v * v);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, fabsf(v), 1.f));
  const float poly =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f),
                       -0.284496736f), 0.254829592f);
  const float half_erfc = 0.5f * poly * e;  // Φ(-|v|)
  const float cdf = v >= 0.f ? 1.f - half_erfc : half_erfc;
  return cdf + v * (0.3989422804014327f * e);
}

__global__ __launch_bounds__(256) void gelu_bwd_kernel(const __bf16* __restrict__ dy,
                                                       const __bf16* __restrict__ x,
                                                       __bf16* __restrict__ dx, long n8) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (long)gridDim.x * blockDim.x) {
    float g[8], v[8];
    unpack8(reinterpret_cast<const uint4*>(dy)[i], g);
    unpack8(reinterpret_cast<const uint4*>(x)[i], v);
#pragma unroll
    for (int q = 0; q < 8; ++q) g[q] *= gelu_grad(v[q]);
    reinterpret_cast<uint4*>(dx)[i] = pack8(g);
  }
}

void gelu_fwd(const void* x, void* y, long n, hipStream_t st) {
  long n8 = n / 8;
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(grid1d(n8)), dim3(256), 0, st, (const __bf16*)x,
                     (__bf16*)y, n8);
}

void gelu_bwd(const void* dy, const void* x, void* dx, long n, hipStream_t st) {
  long n8 = n / 8;
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(grid1d(n8)), dim3(256), 0, st, (const __bf16*)dy,
                     (const __bf16*)x, (__bf16*)dx, n8);
}

// ------------------------------------------------------------------------------ column sums
// out[c] += sum_r x[r][c]  (bias gradients; out may be a view of the flat gradient buffer).
// Grid (column chunks of 512, row blocks): each lane owns 8 consecutive columns (one 16-B bf16
// / two 16-B fp32 loads per row), the block's 4 waves take interleaved rows with 4 rows of loads
// in flight per lane, then the 4 wave partials are summed through LDS and added with one fp32
// atomic per column per block (deterministic mode: written as a partial row instead).
constexpr int kColsumChunk = 512;

template <class T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* __restrict__ x,
                                                     float* __restrict__ out, long rows, int cols,
                                                     long rows_per_block,
                                                     float* __restrict__ part) {
  __shared__ float red[4][kColsumChunk + 4];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int c0 = blockIdx.x * kColsumChunk + l * 8;
  const long r0 = (long)blockIdx.y * rows_per_block;
  const long r1 = min(rows, r0 + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < cols) {
    const T* p = x + c0;
    long r = r0 + w;
    for (; r + 12 < r1; r += 16) {
      float v[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) load8(p + (r + 4 * u) * cols, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += v[u][q];
    }
    for (; r < r1; r += 4) {
      float v[8];
      load8(p + r * cols, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += v[q];
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) red[w][l * 8 + q] = acc[q];
  __syncthreads();
  for (int c = threadIdx.x; c < kColsumChunk; c += 256) {
    const int col = blockIdx.x * kColsumChunk + c;
    if (col >= cols) break;
    const float s = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    if (part != nullptr) part[(long)blockIdx.y * cols + col] = s;
    else atomicAdd(out + col, s);
  }
}

// dx = gelu'(x) * dy AND Σ_rows dx (the bias gradient of the GELU Linear, summed from the
// stored bf16 dx) in one pass over the [rows, cols] tensors.  Grid (column chunk, row block):
// each wave loads 4 rows of dy and x (8 16-B loads per lane in flight) before the math —
// the pass is HBM-bound only with ~1.5k blocks resident (the colsum grid, sized for a pure read
// pass, left it latency-bound at half the bandwidth).
constexpr int kGeluColsumRowsPerBlock = 16;

__global__ __launch_bounds__(256) void gelu_bwd_colsum_kernel(const __bf16* __restrict__ dy,
                                                              const __bf16* __restrict__ x,
                                                              __bf16* __restrict__ dx,
                                                              float* __restrict__ out, long rows,
                                                              int cols, long rows_per_block,
                                                              float* __restrict__ part) {
  __shared__ float red[4][kColsumChunk + 4];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int c0 = blockIdx.x * kColsumChunk + l * 8;
  const long r0 = (long)blockIdx.y * rows_per_block;
  const long r1 = min(rows, r0 + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto row_op = [&](uint4 gv, uint4 xv, long r) {
    float g[8], v[8];
    unpack8(gv, g);
    unpack8(xv, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) g[q] *= gelu_grad(v[q]);
    const uint4 ob = pack8(g);
    *reinterpret_cast<uint4*>(dx + r * cols + c0) = ob;
    unpack8(ob, g);
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += g[q];
  };
  if (c0 < cols) {
    long r = r0 + w;
    for (; r + 12 < r1; r += 16) {
      uint4 gv[4], xv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        gv[u] = *reinterpret_cast<const uint4*>(dy + (r + 4 * u) * cols + c0);
        xv[u] = *reinterpret_cast<const uint4*>(x + (r + 4 * u) * cols + c0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) row_op(gv[u], xv[u], r + 4 * u);
    }
    for (; r < r1; r += 4)
      row_op(*reinterpret_cast<const uint4*>(dy + r * cols + c0),
             *reinterpret_cast<const uint4*>(x + r * cols + c0), r);
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) red[w][l * 8 + q] = acc[q];
  __syncthreads();
  for (int c = threadIdx.x; c < kColsumChunk; c += 256) {
    const int col = blockIdx.x * kColsumChunk + c;
    if (col >= cols) break;
    const float sm = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    if (part != nullptr) part[(long)blockIdx.y * cols + col] = sm;
    else atomicAdd(out + col, sm);
  }
}

static void gelu_colsum_grid(long rows, int cols, long& G, long& rpb) {
  const long chunks = (cols + kColsumChunk - 1) / kColsumChunk;
  G = std::max<long>(1, std::min<long>((rows + kGeluColsumRowsPerBlock - 1) / kGeluColsumRowsPerBlock,
                                       std::max<long>(1, 1536 / chunks)));
  rpb = (rows + G - 1) / G;
  G = (rows + rpb - 1) / rpb;
}

int gelu_bwd_colsum_blocks(long rows, int cols) {
  long G, rpb;
  gelu_colsum_grid(rows, cols, G, rpb);
  return (int)G;
}

int g_colsum_row_blocks = 0;  // > 0: fixed row-block count (tuning experiments)

static void colsum_grid(long rows, int cols, long& G, long& rpb) {
  const long chunks = (cols + kColsumChunk - 1) / kColsumChunk;
  // measured (tools/r2/colsum_sweep.py): ~64-128 rows per block, <= ~1024 blocks
  G = g_colsum_row_blocks > 0 ? g_colsum_row_blocks
                              : std::min<long>((rows + 95) / 96, std::max<long>(1, 1024 / chunks));
  G = std::max<long>(1, std::min<long>(G, (rows + 15) / 16));
  rpb = (rows + G - 1) / G;
  G = (rows + rpb - 1) / rpb;
}

int colsum_blocks(long rows, int cols) {
  long G, rpb;
  colsum_grid(rows, cols, G, rpb);
  return (int)G;
}

void gelu_bwd_colsum(const void* dy, const void* x, void* dx, float* out, long rows, int cols,
                     float* work, hipStream_t st) {
  long G, rpb;
  gelu_colsum_grid(rows, cols, G, rpb);
  dim3 grid((cols + kColsumChunk - 1) / kColsumChunk, (unsigned)G);
  hipLaunchKernelGGL(gelu_bwd_colsum_kernel, grid, dim3(256), 0, st, (const __bf16*)dy,
                     (const __bf16*)x, (__bf16*)dx, out, rows, cols, rpb, work);
  if (work != nullptr) det_sum_rows(work, nullptr, (int)G, cols, out, nullptr, true, st);
}

void colsum_f32(const void* x, bool bf16, float* out, long rows, int cols, float* work,
                hipStream_t st) {
  long G, rpb;
  colsum_grid(rows, cols, G, rpb);
  dim3 grid((cols + kColsumChunk - 1) / kColsumChunk, (unsigned)G);
  // work != null (deterministic mode): per-row-block partial rows, then a fixed-order sum
  if (bf16)
    hipLaunchKernelGGL(colsum_kernel<__bf16>, grid, dim3(256), 0, st, (const __bf16*)x, out, rows,
                       cols, rpb, work);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, st, (const float*)x, out, rows,
                       cols, rpb, work);
  if (work != nullptr) det_sum_rows(work, nullptr, (int)G, cols, out, nullptr, true, st);
}

// ------------------------------------------------------------------------------ embedding grad
// out[idx[r]][:] += dy[r][:] (out fp32, zeroed or the flat gradient view).  Large tables: one
// fp32 atomic per element (rows rarely collide).  Small tables (token types, <= 8 rows): every
// token hits the same few rows, so each block first reduces its tokens into an LDS copy of the
// table (LDS atomics) and adds it to out once — thousands-way global contention otherwise.
__global__ __launch_bounds__(256) void embedding_bwd_kernel(const __bf16* __restrict__ dy,
                                                            const int64_t* __restrict__ idx,
                                                            float* __restrict__ out, long n, int H) {
  long total = n * H;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    long r = t / H;
    int c = (int)(t % H);
    atomicAdd(out + idx[r] * H + c, (float)dy[t]);
  }
}

constexpr int kEmbSmallRows = 8;

// (Column c of the LDS table is only ever touched by thread c % 256, in token order, so the
// block's table is deterministic; with `partial` set each block WRITES its table to row
// blockIdx.x of a [blocks][rows*H] slab — summed in block order by det_sum_rows — instead of
// adding it to out with float atomics.)
__global__ __launch_bounds__(256) void embedding_bwd_small_kernel(
    const __bf16* __restrict__ dy, const int64_t* __restrict__ idx, float* __restrict__ out,
    long n, int H, int rows, long tok_per_block, float* __restrict__ partial) {
  extern __shared__ float tab[];  // [rows][H]
  for (int i = threadIdx.x; i < rows * H; i += 256) tab[i] = 0.f;
  __syncthreads();
  const long t0 = (long)blockIdx.x * tok_per_block, t1 = min(n, t0 + tok_per_block);
  for (long t = t0; t < t1; ++t) {
    const long r = idx[t];
    for (int c = threadIdx.x; c < H; c += 256) atomicAdd(&tab[r * H + c], (float)dy[t * H + c]);
  }
  __syncthreads();
  if (partial != nullptr) {
    float* dst = partial + (long)blockIdx.x * rows * H;
    for (int i = threadIdx.x; i < rows * H; i += 256) dst[i] = tab[i];
  } else {
    for (int i = threadIdx.x; i < rows * H; i += 256) atomicAdd(out + i, tab[i]);
  }
}

// Deterministic scatter-add over tokens SORTED by row id (stable sort: position order inside a
// run of equal ids), in fixed-size CHUNKS of kEmbChunk sorted entries — one wave per chunk — so
// a long run of one id (the [PAD] token of a padded batch: thousands of rows) is summed by many
// waves in parallel instead of serially by one:
//   pass 1: each wave sums the runs of its chunk in position order (8 bf16 columns per 16-B
//           chunk, NC chunks per lane, four rows of loads in flight).  A run that lies wholly
//           inside the chunk is added (x scale) to its output row — its only writer.  A run
//           that enters from the previous chunk leaves its partial in ws[chunk][0] (head), one
//           that continues into the next chunk in ws[chunk][1] (tail); a chunk covered by one
//           run that does both uses the head slot.
//   pass 2: the wave of the chunk where a crossing run STARTS adds its tail partial and the
//           head partials of the following chunks, in chunk order, and writes the row.
// Every output row has exactly one writer and a fixed summation order: bit-identical run to run
// and on every rank that scatters the same tokens.  Negative ids (padding of a fixed-capacity
// exchange, parallel/ddp.py) sort first and are skipped.
constexpr int kEmbChunk = 64;

template <int NC>
__device__ __forceinline__ void emb_add_row(float* __restrict__ o, const float (&acc)[NC][8],
                                            int lane, int nch, float scale) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      float* q = o + ch * 8;
      const float4 a = reinterpret_cast<float4*>(q)[0], b = reinterpret_cast<float4*>(q)[1];
      reinterpret_cast<float4*>(q)[0] = make_float4(a.x + scale * acc[c][0], a.y + scale * acc[c][1],
                                                    a.z + scale * acc[c][2], a.w + scale * acc[c][3]);
      reinterpret_cast<float4*>(q)[1] = make_float4(b.x + scale * acc[c][4], b.y + scale * acc[c][5],
                                                    b.z + scale * acc[c][6], b.w + scale * acc[c][7]);
    }
  }
}

template <int NC>
__device__ __forceinline__ void emb_store_row(float* __restrict__ o, const float (&acc)[NC][8],
                                              int lane, int nch) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      reinterpret_cast<float4*>(o + ch * 8)[0] =
          make_float4(acc[c][0], acc[c][1], acc[c][2], acc[c][3]);
      reinterpret_cast<float4*>(o + ch * 8)[1] =
          make_float4(acc[c][4], acc[c][5], acc[c][6], acc[c][7]);
    }
  }
}

template <int NC>
__global__ __launch_bounds__(256) void embedding_bwd_sorted_kernel(
    const __bf16* __restrict__ dy, const int64_t* __restrict__ sid,
    const int64_t* __restrict__ perm, float* __restrict__ out, float* __restrict__ ws, long n,
    int H, float scale) {
  const long chunk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const long c0 = chunk * kEmbChunk;
  if (c0 >= n) return;
  const long c1 = min(n, c0 + kEmbChunk);
  const int nch = H / 8;
  long i = c0;
  while (i < c1) {
    const int64_t id = sid[i];
    long e = i + 1;
    while (e < c1 && sid[e] == id) ++e;
    if (id >= 0) {
      float acc[NC][8];
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[c][q] = 0.f;
      for (long j = i; j < e; j += 4) {
        long p[4];
        const int cnt = (int)min<long>(4, e - j);
#pragma unroll
        for (int u = 0; u < 4; ++u) p[u] = perm[u < cnt ? j + u : j];
        uint4 v[4][NC];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            const int ch = lane + 64 * c;
            v[u][c] = ch < nch ? *reinterpret_cast<const uint4*>(dy + p[u] * H + ch * 8)
                               : make_uint4(0, 0, 0, 0);
          }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (u < cnt) {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
              float f[8];
              unpack8(v[u][c], f);
#pragma unroll
              for (int q = 0; q < 8; ++q) acc[c][q] += f[q];
            }
          }
        }
      }
      const bool head = i == c0 && c0 > 0 && sid[c0 - 1] == id;
      const bool tail = e == c1 && c1 < n && sid[c1] == id;
      if (!head && !tail) emb_add_row<NC>(out + id * H, acc, lane, nch, scale);
      else emb_store_row<NC>(ws + (chunk * 2 + (head ? 0 : 1)) * H, acc, lane, nch);
    }
    i = e;
  }
}

template <int NC>
__global__ __launch_bounds__(256) void embedding_bwd_sorted_fix_kernel(
    const int64_t* __restrict__ sid, const float* __restrict__ ws, float* __restrict__ out,
    long n, int H, float scale) {
  const long chunk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const long c0 = chunk * kEmbChunk;
  if (c0 >= n) return;
  const long c1 = min(n, c0 + kEmbChunk);
  if (c1 >= n) return;
  const int64_t id = sid[c1 - 1];
  if (id < 0 || sid[c1] != id) return;                   // the chunk's last run ends inside it
  if (c0 > 0 && sid[c0] == id && sid[c0 - 1] == id) return;  // started before: not its owner
  const int nch = H / 8;
  float acc[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[c][q] = 0.f;
  auto add = [&](const float* src) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < nch) {
        const float4 a = reinterpret_cast<const float4*>(src + ch * 8)[0];
        const float4 b = reinterpret_cast<const float4*>(src + ch * 8)[1];
        acc[c][0] += a.x; acc[c][1] += a.y; acc[c][2] += a.z; acc[c][3] += a.w;
        acc[c][4] += b.x; acc[c][5] += b.y; acc[c][6] += b.z; acc[c][7] += b.w;
      }
    }
  };
  add(ws + (chunk * 2 + 1) * H);                          // this chunk's tail partial
  for (long k = chunk + 1;; ++k) {                         // following chunks' head partials
    add(ws + (k * 2) * H);
    const long k1 = min(n, (k + 1) * kEmbChunk);
    if (k1 >= n || sid[k1] != id) break;                   // the run ends inside chunk k
  }
  emb_add_row<NC>(out + id * H, acc, lane, nch, scale);
}

// Tables of <= kEmbSmallRows rows (BERT's token types: 2) with H % 8 == 0: each thread owns one
// 8-column chunk of every table row in registers and walks its token stream (tokens t0 + s,
// t0 + s + S, ...: 256 / (H/8) streams per block) with 16-B loads — no LDS atomics — then the
// streams are added into the block's table in stream order (deterministic) and written out as
// in embedding_bwd_small_kernel.  BERT-base 4096 x 768: 36.4 us (LDS atomics) -> 14.7 us with
// 128 blocks (profiles/r6_bert_emb_tiny.txt).
__global__ __launch_bounds__(256) void embedding_bwd_tiny_kernel(
    const __bf16* __restrict__ dy, const int64_t* __restrict__ idx, float* __restrict__ out,
    long n, int H, int rows, long tok_per_block, float* __restrict__ partial) {
  extern __shared__ float tab[];  // [rows][H]
  const int nc8 = H / 8, S = 256 / nc8;
  const int s = threadIdx.x / nc8, c8 = threadIdx.x - s * nc8;
  const bool act = s < S;
  float acc[kEmbSmallRows][8];
#pragma unroll
  for (int r = 0; r < kEmbSmallRows; ++r)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[r][q] = 0.f;
  const long t0 = (long)blockIdx.x * tok_per_block, t1 = min(n, t0 + tok_per_block);
  if (act) {
    long t = t0 + s;
    for (; t + S < t1; t += 2 * S) {  // two tokens' loads in flight
      const long r0 = idx[t], r1 = idx[t + S];
      const uint4 u0 = *reinterpret_cast<const uint4*>(dy + t * H + c8 * 8);
      const uint4 u1 = *reinterpret_cast<const uint4*>(dy + (t + S) * H + c8 * 8);
      float v0[8], v1[8];
      unpack8(u0, v0);
      unpack8(u1, v1);
#pragma unroll
      for (int rr = 0; rr < kEmbSmallRows; ++rr)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          acc[rr][q] += r0 == rr ? v0[q] : 0.f;
          acc[rr][q] += r1 == rr ? v1[q] : 0.f;
        }
    }
    if (t < t1) {
      const long r = idx[t];
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(dy + t * H + c8 * 8), v);
#pragma unroll
      for (int rr = 0; rr < kEmbSmallRows; ++rr)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[rr][q] += r == rr ? v[q] : 0.f;
    }
  }
  for (int i = threadIdx.x; i < rows * H; i += 256) tab[i] = 0.f;
  __syncthreads();
  for (int ss = 0; ss < S; ++ss) {  // streams added in order
    if (act && s == ss) {
#pragma unroll
      for (int rr = 0; rr < kEmbSmallRows; ++rr)
        if (rr < rows)
#pragma unroll
          for (int q = 0; q < 8; ++q) tab[rr * H + c8 * 8 + q] += acc[rr][q];
    }
    __syncthreads();
  }
  if (partial != nullptr) {
    float* dst = partial + (long)blockIdx.x * rows * H;
    for (int i = threadIdx.x; i < rows * H; i += 256) dst[i] = tab[i];
  } else {
    for (int i = threadIdx.x; i < rows * H; i += 256) atomicAdd(out + i, tab[i]);
  }
}

int embedding_bwd_small_blocks(long n) {
  const long G = std::max<long>(1, std::min<long>(256, (n + 15) / 16));
  const long per = (n + G - 1) / G;
  return (int)((n + per - 1) / per);
}

void embedding_bwd(const void* dy, const int64_t* idx, float* out, long n, int H, int rows,
                   hipStream_t st, float* partial) {
  if (rows > 0 && rows <= kEmbSmallRows) {
    const int G = embedding_bwd_small_blocks(n);
    const long per = (n + G - 1) / G;
    if (H % 8 == 0 && H / 8 <= 256)
      hipLaunchKernelGGL(embedding_bwd_tiny_kernel, dim3((unsigned)G), dim3(256),
                         (size_t)rows * H * 4, st, (const __bf16*)dy, idx, out, n, H, rows, per,
                         partial);
    else
      hipLaunchKernelGGL(embedding_bwd_small_kernel, dim3((unsigned)G), dim3(256),
                         (size_t)rows * H * 4, st, (const __bf16*)dy, idx, out, n, H, rows, per,
                         partial);
    if (partial != nullptr) det_sum_rows(partial, nullptr, G, rows * H, out, nullptr, true, st);
    return;
  }
  hipLaunchKernelGGL(embedding_bwd_kernel, dim3(grid1d(n * H)), dim3(256), 0, st,
                     (const __bf16*)dy, idx, out, n, H);
}

long embedding_bwd_sorted_ws_floats(long n, int H) {
  return ((n + kEmbChunk - 1) / kEmbChunk) * 2 * (long)H;
}

void embedding_bwd_sorted(const void* dy, const int64_t* sorted_ids, const int64_t* perm,
                          float* out, float* ws, long n, int H, float scale, hipStream_t st) {
  const long chunks = (n + kEmbChunk - 1) / kEmbChunk;
  const unsigned g = (unsigned)((chunks + 3) / 4);
  const int nc = (H / 8 + 63) / 64;
  auto go = [&](auto tag) {
    constexpr int NC = decltype(tag)::value;
    hipLaunchKernelGGL(embedding_bwd_sorted_kernel<NC>, dim3(g), dim3(256), 0, st,
                       (const __bf16*)dy, sorted_ids, perm, out, ws, n, H, scale);
    if (chunks > 1)
      hipLaunchKernelGGL(embedding_bwd_sorted_fix_kernel<NC>, dim3(g), dim3(256), 0, st,
                         sorted_ids, (const float*)ws, out, n, H, scale);
  };
  if (nc <= 1) go(std::integral_constant<int, 1>());
  else if (nc == 2) go(std::integral_constant<int, 2>());
  else go(std::integral_constant<int, 4>());
}

// ------------------------------------------------------------------------------ dropout hash
// keep(element i) = hash(seed, i) >= p * 2^32; the per-step part of a device seed (graph replay)
// is mixed in from seed_dev.  Shared by the standalone dropout kernel and the LayerNorm kernels
// that fuse the residual branch's dropout (identical masks: same element index, same hash).
__device__ __forceinline__ uint32_t drop_mix(uint32_t x) {
  x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t drop_base(uint32_t seed, const uint32_t* seed_dev) {
  if (seed_dev != nullptr) {  // L2-served agent-scope load (see attention.hip eff_seed)
    const uint32_t c = __hip_atomic_load(seed_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    seed = drop_mix(seed ^ (c * 0x9e3779b1u + 0x632be5abu));
  }
  return drop_mix(seed * 0x9e3779b1u + 0x7f4a7c15u);
}

__device__ __forceinline__ bool drop_keep(uint32_t base, long idx, uint32_t thr) {
  return drop_mix(base ^ (uint32_t)idx * 0x85ebca77u) >= thr;
}

struct DropArgs {  // by value into the kernels; thr == 0 and scale == 1 when p == 0
  float scale;
  uint32_t thr, seed;
  const uint32_t* seed_dev;
};

static DropArgs drop_args(const DropSpec* d) {
  DropArgs a{1.f, 0u, 0u, nullptr};
  if (d != nullptr && d->p > 0.f) {
    const double t = (double)d->p * 4294967296.0;
    a.thr = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
    a.scale = 1.f / (1.f - d->p);
    a.seed = d->seed;
    a.seed_dev = d->seed_dev;
  }
  return a;
}

// ------------------------------------------------------------------------------ LayerNorm
// One wave per row, up to 4 x 8 elements per lane (H <= 2048), H % 8 == 0.
// DROP: y = LN(dropout(x) + res) — the post-LN residual branch's dropout applied on the load of x
// (the dropped tensor is never stored; the stored sum is what the backward normalises).
constexpr int LN_MAXC = 4;

template <bool DROP>
__global__ __launch_bounds__(256) void layernorm_fwd_kernel(const __bf16* __restrict__ x,
                                                            const __bf16* __restrict__ res,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta,
                                                            __bf16* __restrict__ y,
                                                            __bf16* __restrict__ xsum,
                                                            float* __restrict__ mean,
                                                            float* __restrict__ rstd, long rows,
                                                            int H, float eps, DropArgs dr) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nc = H / 8;
  const uint32_t dbase = DROP ? drop_base(dr.seed, dr.seed_dev) : 0u;
  float v[LN_MAXC][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < LN_MAXC; ++k) {
    int c = lane + k * 64;
    if (c < nc) {
      unpack8(*reinterpret_cast<const uint4*>(x + row * H + c * 8), v[k]);
      if constexpr (DROP) {
        // the standalone kernel rounds the dropped value to bf16: same here, same sums
        float t[8];
#pragma unroll
        for (int q = 0; q < 8; ++q)
          t[q] = drop_keep(dbase, row * H + c * 8 + q, dr.thr) ? v[k][q] * dr.scale : 0.f;
        unpack8(pack8(t), v[k]);
      }
      if (res != nullptr) {
        float r[8];
        unpack8(*reinterpret_cast<const uint4*>(res + row * H + c * 8), r);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[k][q] += r[q];
        *reinterpret_cast<uint4*>(xsum + row * H + c * 8) = pack8(v[k]);
        unpack8(pack8(v[k]), v[k]);  // normalise the bf16-rounded sum that backward will see
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) s += v[k][q];
    }
  }
  const float mu = wave_sum(s) / (float)H;
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < LN_MAXC; ++k) {
    int c = lane + k * 64;
    if (c < nc) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float d = v[k][q] - mu;
        ss += d * d;
      }
    }
  }
  const float rs = rsqrtf(wave_sum(ss) / (float)H + eps);
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
#pragma unroll
  for (int k = 0; k < LN_MAXC; ++k) {
    int c = lane + k * 64;
    if (c < nc) {
      float o[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = (v[k][q] - mu) * rs * gamma[c * 8 + q] + beta[c * 8 + q];
      *reinterpret_cast<uint4*>(y + row * H + c * 8) = pack8(o);
    }
  }
}

// Exact-width LayerNorm: H = NC * 64 * VEC, every lane holds NC whole chunks of VEC elements
// (BERT-base H = 768: 3 chunks of 4 per lane, where the 16-B kernel above leaves half the wave
// idle on its second chunk behind a divergent branch), all loads issued before the first use
// and the two row sums done with DPP instead of ds_bpermute shuffles.
template <int VEC>
using LnVec = std::conditional_t<VEC == 8, uint4, uint2>;

int g_ln_mode = [] {
  const char* v = getenv("MIPIPE_LN_MODE");
  return v != nullptr ? atoi(v) : 8;
}();
void set_layernorm_mode(int mode) { g_ln_mode = mode; }
int get_layernorm_mode() { return g_ln_mode; }

// (VEC, chunks per lane) of the exact kernels for H, or VEC = 0 where they do not apply
static void ln_exact_shape(int H, int& vec, int& nc) {
  vec = nc = 0;
  if (g_ln_mode == 0 || H > 1024) return;
  if (H % 512 == 0) { vec = 8; nc = H / 512; }        // 512, 1024
  else if (H % 256 == 0) { vec = 4; nc = H / 256; }   // 256, 768
}

template <bool DROP, int VEC, int NC>
__global__ __launch_bounds__(256) void layernorm_fwd_exact_kernel(
    const __bf16* __restrict__ x, const __bf16* __restrict__ res, const float* __restrict__ gamma,
    const float* __restrict__ beta, __bf16* __restrict__ y, __bf16* __restrict__ xsum,
    float* __restrict__ mean, float* __restrict__ rstd, long rows, float eps, DropArgs dr) {
  using VT = LnVec<VEC>;
  constexpr int H = NC * 64 * VEC;
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const __bf16* xr = x + row * H;
  VT ux[NC], ur[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) ux[k] = reinterpret_cast<const VT*>(xr)[lane + k * 64];
  if (res != nullptr) {
#pragma unroll
    for (int k = 0; k < NC; ++k) ur[k] = reinterpret_cast<const VT*>(res + row * H)[lane + k * 64];
  }
  const uint32_t dbase = DROP ? drop_base(dr.seed, dr.seed_dev) : 0u;
  float v[NC][VEC];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = lane + k * 64;
    unpackv(ux[k], v[k]);
    if constexpr (DROP) {
      float t[VEC];  // the standalone kernel rounds the dropped value to bf16: same here
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        t[q] = drop_keep(dbase, row * H + c * VEC + q, dr.thr) ? v[k][q] * dr.scale : 0.f;
      unpackv(packv<VT>(t), v[k]);
    }
    if (res != nullptr) {
      float r[VEC];
      unpackv(ur[k], r);
#pragma unroll
      for (int q = 0; q < VEC; ++q) v[k][q] += r[q];
      const VT sb = packv<VT>(v[k]);
      reinterpret_cast<VT*>(xsum + row * H)[c] = sb;
      unpackv(sb, v[k]);  // normalise the bf16-rounded sum that backward will see
    }
#pragma unroll
    for (int q = 0; q < VEC; ++q) s += v[k][q];
  }
  const float mu = wave_sum_dpp(s) * (1.f / (float)H);
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < NC; ++k)
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      const float d = v[k][q] - mu;
      ss += d * d;
    }
  const float rs = rsqrtf(wave_sum_dpp(ss) * (1.f / (float)H) + eps);
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = lane + k * 64;
    float o[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) o[q] = (v[k][q] - mu) * rs * gamma[c * VEC + q] + beta[c * VEC + q];
    reinterpret_cast<VT*>(y + row * H)[c] = packv<VT>(o);
  }
}

void layernorm_fwd(const void* x, const void* res, const float* gamma, const float* beta, void* y,
                   void* xsum, float* mean, float* rstd, long rows, int H, float eps,
                   hipStream_t st, const DropSpec* drop) {
  const DropArgs dr = drop_args(drop);
  int vec, nc;
  ln_exact_shape(H, vec, nc);
  // forward: the 8-wide exact kernel measured slower than the generic one at H = 1024 (9.5 vs
  // 8.0 us, 4096 rows, profiles/r6_layernorm_modes.txt); the 4-wide one is faster at H = 768
  if (vec == 4) {
    auto go = [&](auto drop_c, auto vec_c, auto nc_c) {
      constexpr bool DROP = decltype(drop_c)::value;
      constexpr int VEC = decltype(vec_c)::value, NC = decltype(nc_c)::value;
      hipLaunchKernelGGL((layernorm_fwd_exact_kernel<DROP, VEC, NC>), dim3((rows + 3) / 4),
                         dim3(256), 0, st, (const __bf16*)x, (const __bf16*)res, gamma, beta,
                         (__bf16*)y, (__bf16*)xsum, mean, rstd, rows, eps, dr);
    };
    auto go_v = [&](auto drop_c) {  // (4, 1) H = 256, (4, 3) H = 768
      if (nc == 1) go(drop_c, std::integral_constant<int, 4>(), std::integral_constant<int, 1>());
      else go(drop_c, std::integral_constant<int, 4>(), std::integral_constant<int, 3>());
    };
    if (dr.thr != 0u) go_v(std::true_type());
    else go_v(std::false_type());
    return;
  }
  if (dr.thr != 0u)
    hipLaunchKernelGGL(layernorm_fwd_kernel<true>, dim3((rows + 3) / 4), dim3(256), 0, st,
                       (const __bf16*)x, (const __bf16*)res, gamma, beta, (__bf16*)y,
                       (__bf16*)xsum, mean, rstd, rows, H, eps, dr);
  else
    hipLaunchKernelGGL(layernorm_fwd_kernel<false>, dim3((rows + 3) / 4), dim3(256), 0, st,
                       (const __bf16*)x, (const __bf16*)res, gamma, beta, (__bf16*)y,
                       (__bf16*)xsum, mean, rstd, rows, H, eps, dr);
}

// dx = rstd*(g*γ - mean(g*γ) - x̂*mean(g*γ*x̂)); per-block partials of Σg·x̂ and Σg for dγ, dβ.
// Each wave walks rows w, w+4, ... of its block with the NEXT row's dy / x loads in flight while
// it reduces the current one (the kernel is latency-bound otherwise: two dependent wave sums
// per row); γ is held in registers for the whole block.
// DROP: also dxd = dropout'(dx) — the gradient of the dropped branch (the residual keeps dx).
// BSUM: also per-block partials of Σ_rows of the branch gradient (dxd, else dx; bf16-rounded as
// stored) — the bias gradient of the Linear that produced the LayerNorm's input.
template <int NCH, bool DROP, bool BSUM>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const __bf16* __restrict__ dy,
                                                            const __bf16* __restrict__ x,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            const float* __restrict__ gamma,
                                                            __bf16* __restrict__ dx,
                                                            float* __restrict__ pg,
                                                            float* __restrict__ pb, long rows,
                                                            int H, int rows_per_block,
                                                            __bf16* __restrict__ dxd, DropArgs dr,
                                                            float* __restrict__ pd) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t dbase = DROP ? drop_base(dr.seed, dr.seed_dev) : 0u;
  const int nc = H / 8;
  float accg[NCH][8], accb[NCH][8], accd[NCH][8], gam[NCH][8];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = lane + k * 64;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      accg[k][q] = accb[k][q] = accd[k][q] = 0.f;
      gam[k][q] = c < nc ? gamma[c * 8 + q] : 0.f;
    }
  }
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = min(rows, r0 + rows_per_block);
  uint4 ng[NCH], nx[NCH];
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](long row) {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = lane + k * 64;
      if (c < nc) {
        ng[k] = *reinterpret_cast<const uint4*>(dy + row * H + c * 8);
        nx[k] = *reinterpret_cast<const uint4*>(x + row * H + c * 8);
      }
    }
    nmu = mean[row];
    nrs = rstd[row];
  };
  if (r0 + w < r1) fetch(r0 + w);
  for (long row = r0 + w; row < r1; row += 4) {
    const float mu = nmu, rs = nrs;
    float g[NCH][8], xh[NCH][8];
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      if (lane + k * 64 < nc) {
        unpack8(ng[k], g[k]);
        unpack8(nx[k], xh[k]);
      }
    }
    if (row + 4 < r1) fetch(row + 4);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      if (lane + k * 64 < nc) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          xh[k][q] = (xh[k][q] - mu) * rs;
          accg[k][q] += g[k][q] * xh[k][q];
          accb[k][q] += g[k][q];
          const float gg = g[k][q] * gam[k][q];
          s1 += gg;
          s2 += gg * xh[k][q];
        }
      }
    }
    s1 = wave_sum(s1) / (float)H;
    s2 = wave_sum(s2) / (float)H;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = lane + k * 64;
      if (c < nc) {
        float o[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = rs * (g[k][q] * gam[k][q] - s1 - xh[k][q] * s2);
        const uint4 ob = pack8(o);
        *reinterpret_cast<uint4*>(dx + row * H + c * 8) = ob;
        if constexpr (DROP) {  // from the bf16-rounded dx, as the standalone kernel would see it
          float od[8];
          unpack8(ob, od);
#pragma unroll
          for (int q = 0; q < 8; ++q)
            od[q] = drop_keep(dbase, row * H + c * 8 + q, dr.thr) ? od[q] * dr.scale : 0.f;
          const uint4 odb = pack8(od);
          *reinterpret_cast<uint4*>(dxd + row * H + c * 8) = odb;
          if constexpr (BSUM) {
            unpack8(odb, od);
#pragma unroll
            for (int q = 0; q < 8; ++q) accd[k][q] += od[q];
          }
        } else if constexpr (BSUM) {
          unpack8(ob, o);
#pragma unroll
          for (int q = 0; q < 8; ++q) accd[k][q] += o[q];
        }
      }
    }
  }
  // block partials of dγ/dβ: the 4 waves reduce through LDS into this block's partial rows
  // (pg / pb: [gridDim.x][H]); summed in a fixed order by det_sum_rows (no atomics: every
  // block would otherwise contend on the same 2H addresses)
  __shared__ float red[4][NCH * 64 * 8];
  for (int arr = 0; arr < (BSUM ? 3 : 2); ++arr) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      int c = lane + k * 64;
      if (c < nc)
#pragma unroll
        for (int q = 0; q < 8; ++q)
          red[w][c * 8 + q] = arr == 0 ? accg[k][q] : arr == 1 ? accb[k][q] : accd[k][q];
    }
    __syncthreads();
    float* dst = (arr == 0 ? pg : arr == 1 ? pb : pd) + (long)blockIdx.x * H;
    for (int c = threadIdx.x; c < H; c += 256)
      dst[c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
  }
}

// Exact-width backward (H = NC * 64 * VEC, as layernorm_fwd_exact_kernel) with W waves per block:
// the same <= 256 blocks (one fixed-order summing pass over their partial rows) but W = 8 puts
// 8 waves on each CU instead of 4, so the rows' loads overlap across waves rather than only
// through the one-row prefetch.  Partials: LDS, summed over the waves in a fixed pairwise order.
// BERT-base 4096 x 768 with dropout + bias sum: 14.6 -> 11.3 us incl. the partial-row sum
// (W = 16: 11.5, and 23.6 at H = 1024; profiles/r6_layernorm_modes.txt).
template <int VEC, int NC, int W, bool DROP, bool BSUM>
__global__ __launch_bounds__(W * 64) void layernorm_bwd_exact_kernel(
    const __bf16* __restrict__ dy, const __bf16* __restrict__ x, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ gamma, __bf16* __restrict__ dx,
    float* __restrict__ pg, float* __restrict__ pb, long rows, int rows_per_block,
    __bf16* __restrict__ dxd, DropArgs dr, float* __restrict__ pd) {
  using VT = LnVec<VEC>;
  constexpr int H = NC * 64 * VEC;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t dbase = DROP ? drop_base(dr.seed, dr.seed_dev) : 0u;
  float accg[NC][VEC], accb[NC][VEC], accd[NC][VEC], gam[NC][VEC];
#pragma unroll
  for (int k = 0; k < NC; ++k)
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      accg[k][q] = accb[k][q] = accd[k][q] = 0.f;
      gam[k][q] = gamma[(lane + k * 64) * VEC + q];
    }
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = min(rows, r0 + rows_per_block);
  VT ng[NC], nx[NC];
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](long row) {
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      ng[k] = reinterpret_cast<const VT*>(dy + row * H)[lane + k * 64];
      nx[k] = reinterpret_cast<const VT*>(x + row * H)[lane + k * 64];
    }
    nmu = mean[row];
    nrs = rstd[row];
  };
  if (r0 + w < r1) fetch(r0 + w);
  for (long row = r0 + w; row < r1; row += W) {
    const float mu = nmu, rs = nrs;
    float g[NC][VEC], xh[NC][VEC];
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      unpackv(ng[k], g[k]);
      unpackv(nx[k], xh[k]);
    }
    if (row + W < r1) fetch(row + W);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k)
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        xh[k][q] = (xh[k][q] - mu) * rs;
        accg[k][q] += g[k][q] * xh[k][q];
        accb[k][q] += g[k][q];
        const float gg = g[k][q] * gam[k][q];
        s1 += gg;
        s2 += gg * xh[k][q];
      }
    s1 = wave_sum_dpp(s1) * (1.f / (float)H);
    s2 = wave_sum_dpp(s2) * (1.f / (float)H);
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c = lane + k * 64;
      float o[VEC];
#pragma unroll
      for (int q = 0; q < VEC; ++q) o[q] = rs * (g[k][q] * gam[k][q] - s1 - xh[k][q] * s2);
      const VT ob = packv<VT>(o);
      reinterpret_cast<VT*>(dx + row * H)[c] = ob;
      if constexpr (DROP) {  // from the bf16-rounded dx, as the standalone kernel would see it
        float od[VEC];
        unpackv(ob, od);
#pragma unroll
        for (int q = 0; q < VEC; ++q)
          od[q] = drop_keep(dbase, row * H + c * VEC + q, dr.thr) ? od[q] * dr.scale : 0.f;
        const VT odb = packv<VT>(od);
        reinterpret_cast<VT*>(dxd + row * H)[c] = odb;
        if constexpr (BSUM) {
          unpackv(odb, od);
#pragma unroll
          for (int q = 0; q < VEC; ++q) accd[k][q] += od[q];
        }
      } else if constexpr (BSUM) {
        unpackv(ob, o);
#pragma unroll
        for (int q = 0; q < VEC; ++q) accd[k][q] += o[q];
      }
    }
  }
  __shared__ float red[W][H];
  for (int arr = 0; arr < (BSUM ? 3 : 2); ++arr) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NC; ++k)
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        red[w][(lane + k * 64) * VEC + q] = arr == 0 ? accg[k][q] : arr == 1 ? accb[k][q] : accd[k][q];
    __syncthreads();
    float* dst = (arr == 0 ? pg : arr == 1 ? pb : pd) + (long)blockIdx.x * H;
    for (int c = threadIdx.x; c < H; c += W * 64) {
      float t[W];
#pragma unroll
      for (int i = 0; i < W; ++i) t[i] = red[i][c];
#pragma unroll
      for (int s = 1; s < W; s *= 2)
#pragma unroll
        for (int i = 0; i + s < W; i += 2 * s) t[i] += t[i + s];
      dst[c] = t[0];
    }
  }
}

static void layernorm_bwd_grid(long rows, int& G, int& rpb) {
  // >= 16 rows (4 per wave, each next one prefetched) per block and <= 256 blocks: the partial
  // rows then take ONE fixed-order summing pass (det_sum_rows goes two-level above 256 rows;
  // BERT 32x128: 512 blocks of 8 rows cost a second launch per call)
  G = (int)std::max<long>(1, std::min<long>(256, (rows + 15) / 16));
  rpb = (int)((rows + G - 1) / G);
  G = (int)((rows + rpb - 1) / rpb);
}

int layernorm_bwd_blocks(long rows) {
  int G, rpb;
  layernorm_bwd_grid(rows, G, rpb);
  return G;
}

void layernorm_bwd(const void* dy, const void* x, const float* mean, const float* rstd,
                   const float* gamma, void* dx, float* dgamma, float* dbeta, float* work,
                   long rows, int H, hipStream_t st, void* dxd, const DropSpec* drop,
                   float* dbias) {
  // dgamma / dbeta (and dbias) are ACCUMULATED into (zeroed buffers or the flat gradient views)
  // from the per-block partial rows in work ([2 or 3][layernorm_bwd_blocks(rows)][H])
  int G, rpb;
  layernorm_bwd_grid(rows, G, rpb);
  float* wg = work;
  float* wb = work + (long)G * H;
  float* wd = dbias != nullptr ? work + 2l * G * H : nullptr;
  // register arrays sized for H: 2 chunks of 8 per lane up to H = 1024 (BERT-base), else 4
  const DropArgs dr = drop_args(drop);
  const bool dp = dr.thr != 0u && dxd != nullptr;
  int vec, nc;
  ln_exact_shape(H, vec, nc);
  if (vec != 0) {
    auto go = [&](auto vec_c, auto nc_c, auto w_c, auto drop_c, auto bsum_c) {
      constexpr int VEC = decltype(vec_c)::value, NC = decltype(nc_c)::value;
      constexpr int W = decltype(w_c)::value;
      constexpr bool DROP = decltype(drop_c)::value, BSUM = decltype(bsum_c)::value;
      hipLaunchKernelGGL((layernorm_bwd_exact_kernel<VEC, NC, W, DROP, BSUM>), dim3(G),
                         dim3(W * 64), 0, st, (const __bf16*)dy, (const __bf16*)x, mean, rstd,
                         gamma, (__bf16*)dx, wg, wb, rows, rpb, (__bf16*)dxd, dr, wd);
    };
    auto go_w = [&](auto vec_c, auto nc_c, auto drop_c, auto bsum_c) {
      if (g_ln_mode == 4) go(vec_c, nc_c, std::integral_constant<int, 4>(), drop_c, bsum_c);
      else if (g_ln_mode == 8) go(vec_c, nc_c, std::integral_constant<int, 8>(), drop_c, bsum_c);
      else go(vec_c, nc_c, std::integral_constant<int, 16>(), drop_c, bsum_c);
    };
    auto go_s = [&](auto drop_c, auto bsum_c) {
      using I8 = std::integral_constant<int, 8>;
      using I4 = std::integral_constant<int, 4>;
      if (vec == 8 && nc == 1) go_w(I8(), std::integral_constant<int, 1>(), drop_c, bsum_c);
      else if (vec == 8) go_w(I8(), std::integral_constant<int, 2>(), drop_c, bsum_c);
      else if (nc == 1) go_w(I4(), std::integral_constant<int, 1>(), drop_c, bsum_c);
      else go_w(I4(), std::integral_constant<int, 3>(), drop_c, bsum_c);
    };
    auto go_d = [&](auto drop_c) {
      if (wd != nullptr) go_s(drop_c, std::true_type());
      else go_s(drop_c, std::false_type());
    };
    if (dp) go_d(std::true_type());
    else go_d(std::false_type());
    det_sum_rows(wg, wb, G, H, dgamma, dbeta, true, st, wd, dbias);
    return;
  }
  auto go = [&](auto nch, auto drop_c, auto bsum_c) {
    constexpr int NCH = decltype(nch)::value;
    constexpr bool DROP = decltype(drop_c)::value, BSUM = decltype(bsum_c)::value;
    hipLaunchKernelGGL((layernorm_bwd_kernel<NCH, DROP, BSUM>), dim3(G), dim3(256), 0, st,
                       (const __bf16*)dy, (const __bf16*)x, mean, rstd, gamma, (__bf16*)dx, wg,
                       wb, rows, H, rpb, (__bf16*)dxd, dr, wd);
  };
  auto go_b = [&](auto nch, auto drop_c) {
    if (wd != nullptr) go(nch, drop_c, std::true_type());
    else go(nch, drop_c, std::false_type());
  };
  if (H <= 1024) {
    if (dp) go_b(std::integral_constant<int, 2>(), std::true_type());
    else go_b(std::integral_constant<int, 2>(), std::false_type());
  } else {
    if (dp) go_b(std::integral_constant<int, LN_MAXC>(), std::true_type());
    else go_b(std::integral_constant<int, LN_MAXC>(), std::false_type());
  }
  det_sum_rows(wg, wb, G, H, dgamma, dbeta, true, st, wd, dbias);
}

// ------------------------------------------------------------------------------ dropout

__global__ __launch_bounds__(256) void dropout_kernel(const __bf16* __restrict__ x,
                                                      __bf16* __restrict__ y, long n8, float scale,
                                                      uint32_t thr, uint32_t seed,
                                                      const uint32_t* __restrict__ seed_dev) {
  const uint32_t base = drop_base(seed, seed_dev);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (long)gridDim.x * blockDim.x) {
    float f[8];
    unpack8(reinterpret_cast<const uint4*>(x)[i], f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = drop_keep(base, i * 8 + e, thr) ? f[e] * scale : 0.f;
    reinterpret_cast<uint4*>(y)[i] = pack8(f);
  }
}

void dropout_fwd(const void* x, void* y, long n, float p, uint32_t seed, hipStream_t st,
                 const uint32_t* seed_dev) {
  const long n8 = n / 8;
  double t = (double)p * 4294967296.0;
  uint32_t thr = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
  hipLaunchKernelGGL(dropout_kernel, dim3(grid1d(n8)), dim3(256), 0, st, (const __bf16*)x,
                     (__bf16*)y, n8, 1.f / (1.f - p), thr, seed, seed_dev);
}

// ------------------------------------------------------------------------------ stem packing
// One thread per output super-pixel: 2 horizontally adjacent padded pixels x 4 channels.
// The same launch also packs the stem FILTER (w != nullptr): wp[co][kh][j][p*4 + c] =
// w[co][c][kh][2j + p] (zero for kw = 7 and c >= C), from the fp32 parameter with any strides
// (channels_last), in the activation dtype — the work of a zero-fill, a strided copy and a cast
// in separate launches.
struct StemWPack {
  const float* w = nullptr;
  void* wp = nullptr;
  int Co = 0, K = 0;
  long s0 = 0, s1 = 0, s2 = 0, s3 = 0;
};
template <class T>
__device__ void stem_wpack(const StemWPack& k, int C) {
  const int K2 = (k.K + 1) / 2;
  const long total = (long)k.Co * k.K * K2 * 8;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int q = (int)(t % 8), j = (int)((t / 8) % K2), kh = (int)((t / 8 / K2) % k.K);
    const int co = (int)(t / 8 / K2 / k.K);
    const int p = q / 4, c = q % 4, kw = 2 * j + p;
    const float v = (kw < k.K && c < C) ? k.w[co * k.s0 + c * k.s1 + kh * k.s2 + kw * k.s3] : 0.f;
    reinterpret_cast<T*>(k.wp)[t] = from_f32<T>(v);
  }
}

template <bool IN_BF16, class T>
__global__ __launch_bounds__(256) void stem_pack_kernel(const void* __restrict__ xin,
                                                        T* __restrict__ y, int N, int C,
                                                        int H, int W, int pad, int Hp, int Wsp,
                                                        StemWPack wk) {
  if (wk.w != nullptr) stem_wpack<T>(wk, C);
  const long total = (long)N * Hp * Wsp;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int j = (int)(t % Wsp);
    const long r = t / Wsp;
    const int hp = (int)(r % Hp);
    const int n = (int)(r / Hp);
    const int h = hp - pad;
    // all 8 loads issued unconditionally at clamped (in-image) addresses, then the padding
    // zeroed by selects: a load behind its bounds branch was closed by a vmcnt(0) each
    float v[8];
    bool inb[8];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int w = 2 * j + p - pad;
      const bool in = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      const int hc = min(max(h, 0), H - 1), wc = min(max(w, 0), W - 1);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int cc = c < C ? c : C - 1;
        const long idx = (((long)n * C + cc) * H + hc) * W + wc;
        v[p * 4 + c] = IN_BF16 ? (float)reinterpret_cast<const __bf16*>(xin)[idx]
                               : reinterpret_cast<const float*>(xin)[idx];
        inb[p * 4 + c] = in && c < C;
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = inb[q] ? v[q] : 0.f;
    store8(y + t * 8, v);
  }
}

void stem_pack(const void* x, bool x_is_bf16, void* y, int N, int C, int H, int W, int pad,
               int Hp, int Wsp, hipStream_t st, bool y_f32, const float* w, void* wp, int Co,
               int K, const long* ws) {
  const long total = (long)N * Hp * Wsp;
  dim3 g(grid1d(total));
  StemWPack wk;
  if (w != nullptr) {
    wk.w = w; wk.wp = wp; wk.Co = Co; wk.K = K;
    wk.s0 = ws[0]; wk.s1 = ws[1]; wk.s2 = ws[2]; wk.s3 = ws[3];
  }
  if (y_f32) {
    if (x_is_bf16) hipLaunchKernelGGL((stem_pack_kernel<true, float>), g, dim3(256), 0, st, x, (float*)y, N, C, H, W, pad, Hp, Wsp, wk);
    else hipLaunchKernelGGL((stem_pack_kernel<false, float>), g, dim3(256), 0, st, x, (float*)y, N, C, H, W, pad, Hp, Wsp, wk);
  } else {
    if (x_is_bf16) hipLaunchKernelGGL((stem_pack_kernel<true, __bf16>), g, dim3(256), 0, st, x, (__bf16*)y, N, C, H, W, pad, Hp, Wsp, wk);
    else hipLaunchKernelGGL((stem_pack_kernel<false, __bf16>), g, dim3(256), 0, st, x, (__bf16*)y, N, C, H, W, pad, Hp, Wsp, wk);
  }
}

// Stem filter gradient, kernel layout [Co][K][K2][8] -> ACCUMULATED into the parameter's
// gradient [Co][C][K][K] (any strides: the flat DDP bucket view), one launch instead of a
// strided copy + autograd's accumulate.
__global__ __launch_bounds__(256) void stem_wgrad_unpack_kernel(const float* __restrict__ dwp,
                                                                float* __restrict__ g, int Co,
                                                                int C, int K, long s0, long s1,
                                                                long s2, long s3) {
  const int K2 = (K + 1) / 2;
  const long total = (long)Co * C * K * K;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int kw = (int)(t % K), kh = (int)((t / K) % K), c = (int)((t / K / K) % C);
    const int co = (int)(t / K / K / C);
    const float v = dwp[(((long)co * K + kh) * K2 + kw / 2) * 8 + (kw % 2) * 4 + c];
    g[co * s0 + c * s1 + kh * s2 + kw * s3] += v;
  }
}

void stem_wgrad_unpack(const float* dwp, float* g, int Co, int C, int K, const long* gs,
                       hipStream_t st) {
  const long total = (long)Co * C * K * K;
  hipLaunchKernelGGL(stem_wgrad_unpack_kernel, dim3(grid1d(total)), dim3(256), 0, st, dwp, g, Co,
                     C, K, gs[0], gs[1], gs[2], gs[3]);
}

}  // namespace mipipe
