// AdamW flat-buffer kernel variants at BERT-base size (110M fp32 params + bf16 shadow):
// v0 = shipped (one float4 per iteration), v1 = two float4 per iteration with all loads first,
// v2 = v1 + nontemporal stores.  Prints us per step and effective TB/s (30 B / param).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef float f4v __attribute__((ext_vector_type(4)));
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  bf16x2 v = {(__bf16)a, (__bf16)b};
  return *reinterpret_cast<uint32_t*>(&v);
}

struct Hp { float lr, b1, b2, eps, wd, bc1, rbc2; };

__device__ __forceinline__ void upd(float4& pv, float4 gv, float4& mv, float4& vv, const Hp& h) {
  float* pa = &pv.x; const float* ga = &gv.x; float* ma = &mv.x; float* va = &vv.x;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float gq = ga[q];
    pa[q] *= 1.f - h.lr * h.wd;
    ma[q] = h.b1 * ma[q] + (1.f - h.b1) * gq;
    va[q] = h.b2 * va[q] + (1.f - h.b2) * gq * gq;
    float denom = sqrtf(va[q]) * h.rbc2 + h.eps;
    pa[q] -= (h.lr / h.bc1) * ma[q] / denom;
  }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void k(float4* __restrict__ p, const float4* __restrict__ g,
                                         float4* __restrict__ m, float4* __restrict__ v,
                                         uint2* __restrict__ sh, long n4, Hp h) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x; i0 < n4; i0 += stride * U) {
    float4 pv[U], gv[U], mv[U], vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long i = i0 + u * stride;
      if (i < n4) { pv[u] = p[i]; gv[u] = g[i]; mv[u] = m[i]; vv[u] = v[i]; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long i = i0 + u * stride;
      if (i < n4) {
        upd(pv[u], gv[u], mv[u], vv[u], h);
        uint2 s = make_uint2(pack2(pv[u].x, pv[u].y), pack2(pv[u].z, pv[u].w));
        if (NT) {
          __builtin_nontemporal_store(*reinterpret_cast<f4v*>(&pv[u]), reinterpret_cast<f4v*>(p + i));
          __builtin_nontemporal_store(*reinterpret_cast<f4v*>(&mv[u]), reinterpret_cast<f4v*>(m + i));
          __builtin_nontemporal_store(*reinterpret_cast<f4v*>(&vv[u]), reinterpret_cast<f4v*>(v + i));
          __builtin_nontemporal_store(*reinterpret_cast<u2v*>(&s), reinterpret_cast<u2v*>(sh + i));
        } else {
          p[i] = pv[u]; m[i] = mv[u]; v[i] = vv[u]; sh[i] = s;
        }
      }
    }
  }
}

int main() {
  const long n = 110000000 / 64 * 64, n4 = n / 4;
  float4 *p, *g, *m, *v; uint2* sh;
  hipMalloc(&p, n * 4); hipMalloc(&g, n * 4); hipMalloc(&m, n * 4); hipMalloc(&v, n * 4);
  hipMalloc(&sh, n * 2);
  hipMemset(p, 0, n * 4); hipMemset(g, 0, n * 4); hipMemset(m, 0, n * 4); hipMemset(v, 0, n * 4);
  Hp h{1e-4f, 0.9f, 0.999f, 1e-8f, 0.01f, 0.1f, 1.f};
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto run = [&](const char* name, auto kern, int grid) {
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, p, g, m, v, sh, n4, h);
    hipEventRecord(a);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, p, g, m, v, sh, n4, h);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    double us = ms / 20 * 1e3;
    printf("%-24s grid %6d  %7.1f us  %.2f TB/s\n", name, grid, us, 30.0 * n / (us * 1e-6) / 1e12);
  };
  for (int grid : {8192, 16384, 32768}) {
    run("v0 u1", k<1, false>, grid);
    run("v1 u2", k<2, false>, grid);
    run("v2 u2 nt", k<2, true>, grid);
    run("v3 u1 nt", k<1, true>, grid);
  }
  return 0;
}
