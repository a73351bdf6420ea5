// BN apply lab: standalone variants of the bf16 BN forward apply (z = relu(y*s+b)) and the BN
// backward apply (dy = A*g' + B*y + C, g' = relu-mask(g)) at ResNet-50 b256 shapes, timed with
// hipEvents over buffer sets rotated past the 256 MB last-level cache.
//   v0   = the production kernels' structure (grid-stride rows, grid capped at 2048 blocks)
//   tU   = contiguous row tile per block, U rows per thread with all loads issued first
//   mU   = tU, ReLU mask read as bits (1 bit/element) instead of z (backward only)
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/kernels tools/r2/bnlab.hip -o tools/r2/bnlab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "common.hpp"

using namespace mipipe;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1); } } while (0)

constexpr int kT = 256;

struct RowMap { int tpr, rpb; };
__host__ __device__ inline RowMap row_map(int C) {
  int chunks = C / 8;  // lab: C/8 <= 256
  return {chunks, kT / chunks};
}

// ------------------------------------------------------------------ forward
__global__ __launch_bounds__(256) void fwd_v0(const __bf16* __restrict__ y, const float* __restrict__ sc_,
                                              const float* __restrict__ bi_, __bf16* __restrict__ z,
                                              long M, int C) {
  const RowMap mp = row_map(C);
  const int t = threadIdx.x, rg = t / mp.tpr;
  if (rg >= mp.rpb) return;
  const int c0 = (t % mp.tpr) * 8;
  float sc[8], bi[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) { sc[q] = sc_[c0 + q]; bi[q] = bi_[c0 + q]; }
  for (long row = (long)blockIdx.x * mp.rpb + rg; row < M; row += (long)gridDim.x * mp.rpb) {
    const long off = row * C + c0;
    float v[8];
    load8(y + off, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q] * sc[q] + bi[q], 0.f);
    store8(z + off, v);
  }
}

template <int U>
__global__ __launch_bounds__(256) void fwd_tile(const __bf16* __restrict__ y, const float* __restrict__ sc_,
                                                const float* __restrict__ bi_, __bf16* __restrict__ z,
                                                long M, int C) {
  const RowMap mp = row_map(C);
  const int t = threadIdx.x, rg = t / mp.tpr;
  if (rg >= mp.rpb) return;
  const int c0 = (t % mp.tpr) * 8;
  const long row0 = (long)blockIdx.x * mp.rpb * U + rg;
  uint4 raw[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long row = row0 + (long)u * mp.rpb;
    if (row < M) raw[u] = *reinterpret_cast<const uint4*>(y + row * C + c0);
  }
  float sc[8], bi[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) { sc[q] = sc_[c0 + q]; bi[q] = bi_[c0 + q]; }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long row = row0 + (long)u * mp.rpb;
    if (row >= M) break;
    float v[8];
    unpack8(raw[u], v);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q] * sc[q] + bi[q], 0.f);
    store8(z + row * C + c0, v);
  }
}

// ------------------------------------------------------------------ backward
__global__ __launch_bounds__(256) void bwd_v0(const __bf16* __restrict__ dz, const __bf16* __restrict__ z,
                                              const __bf16* __restrict__ y, const float* __restrict__ Aa,
                                              const float* __restrict__ Ba, const float* __restrict__ Ca,
                                              __bf16* __restrict__ dy, long M, int C) {
  const RowMap mp = row_map(C);
  const int t = threadIdx.x, rg = t / mp.tpr;
  if (rg >= mp.rpb) return;
  const int c0 = (t % mp.tpr) * 8;
  float A[8], B[8], Cc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) { A[q] = Aa[c0 + q]; B[q] = Ba[c0 + q]; Cc[q] = Ca[c0 + q]; }
  for (long row = (long)blockIdx.x * mp.rpb + rg; row < M; row += (long)gridDim.x * mp.rpb) {
    const long off = row * C + c0;
    float g[8], zv[8], yv[8], o[8];
    load8(dz + off, g);
    load8(z + off, zv);
    load8(y + off, yv);
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = A[q] * (zv[q] > 0.f ? g[q] : 0.f) + B[q] * yv[q] + Cc[q];
    store8(dy + off, o);
  }
}

template <int U, bool BITS>
__global__ __launch_bounds__(256) void bwd_tile(const __bf16* __restrict__ dz, const __bf16* __restrict__ z,
                                                const uint8_t* __restrict__ mask,
                                                const __bf16* __restrict__ y, const float* __restrict__ Aa,
                                                const float* __restrict__ Ba, const float* __restrict__ Ca,
                                                __bf16* __restrict__ dy, long M, int C) {
  const RowMap mp = row_map(C);
  const int t = threadIdx.x, rg = t / mp.tpr;
  if (rg >= mp.rpb) return;
  const int cg = t % mp.tpr, c0 = cg * 8;
  const long row0 = (long)blockIdx.x * mp.rpb * U + rg;
  uint4 rgv[U], rz[U], ry[U];
  uint32_t mb[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long row = row0 + (long)u * mp.rpb;
    if (row < M) {
      const long off = row * C + c0;
      rgv[u] = *reinterpret_cast<const uint4*>(dz + off);
      if (BITS) mb[u] = mask[row * (C / 8) + cg];
      else rz[u] = *reinterpret_cast<const uint4*>(z + off);
      ry[u] = *reinterpret_cast<const uint4*>(y + off);
    }
  }
  float A[8], B[8], Cc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) { A[q] = Aa[c0 + q]; B[q] = Ba[c0 + q]; Cc[q] = Ca[c0 + q]; }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long row = row0 + (long)u * mp.rpb;
    if (row >= M) break;
    float g[8], yv[8], o[8];
    unpack8(rgv[u], g);
    unpack8(ry[u], yv);
    if (BITS) {
#pragma unroll
      for (int q = 0; q < 8; ++q) g[q] = (mb[u] >> q) & 1u ? g[q] : 0.f;
    } else {
      float zv[8];
      unpack8(rz[u], zv);
#pragma unroll
      for (int q = 0; q < 8; ++q) g[q] = zv[q] > 0.f ? g[q] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = A[q] * g[q] + B[q] * yv[q] + Cc[q];
    store8(dy + row * C + c0, o);
  }
}

// ------------------------------------------------------------------ harness
struct Set { __bf16 *a, *b, *c, *d; uint8_t* m; };

template <class F>
static float time_it(F launch, int sets, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < sets; ++i) launch(i);  // warm
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch(r % sets);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipGetLastError());
  return ms * 1000.f / reps;
}

int main() {
  const long shapes[][2] = {{802816, 64}, {802816, 256}, {200704, 128}, {200704, 512},
                            {50176, 256}, {50176, 1024}, {12544, 512}, {12544, 2048}};
  const int NS = 4, reps = 40;
  float *s, *b, *A, *B, *Cc;
  CK(hipMalloc(&s, 2048 * 4)); CK(hipMalloc(&b, 2048 * 4)); CK(hipMalloc(&A, 2048 * 4));
  CK(hipMalloc(&B, 2048 * 4)); CK(hipMalloc(&Cc, 2048 * 4));
  std::vector<float> h(2048, 0.5f);
  for (float* p : {s, b, A, B, Cc}) CK(hipMemcpy(p, h.data(), 2048 * 4, hipMemcpyHostToDevice));
  const long maxe = 802816L * 256;
  std::vector<Set> S(NS);
  for (auto& st : S) {
    CK(hipMalloc(&st.a, maxe * 2)); CK(hipMalloc(&st.b, maxe * 2));
    CK(hipMalloc(&st.c, maxe * 2)); CK(hipMalloc(&st.d, maxe * 2));
    CK(hipMalloc(&st.m, maxe / 8));
    CK(hipMemset(st.a, 0x3f, maxe * 2)); CK(hipMemset(st.b, 0x3f, maxe * 2));
    CK(hipMemset(st.c, 0x3f, maxe * 2)); CK(hipMemset(st.m, 0x55, maxe / 8));
  }
  printf("%-14s %8s %5s | %-10s %8s %7s\n", "op", "M", "C", "variant", "us", "TB/s");
  for (auto& sh : shapes) {
    const long M = sh[0];
    const int C = (int)sh[1];
    const RowMap mp = row_map(C);
    const double el = (double)M * C;
    auto rep = [&](const char* op, const char* v, float us, double bytes) {
      printf("%-14s %8ld %5d | %-10s %8.1f %7.2f\n", op, M, C, v, us, bytes / (us * 1e-6) / 1e12);
    };
    const int g0 = (int)std::min<long>((M + mp.rpb - 1) / mp.rpb, 2048);
    const double fb = el * 4;
    rep("fwd", "v0", time_it([&](int i) { hipLaunchKernelGGL(fwd_v0, dim3(g0), dim3(256), 0, 0, S[i].a, s, b, S[i].d, M, C); }, NS, reps), fb);
#define FT(U) { int g = (int)((M + mp.rpb * U - 1) / (mp.rpb * U)); \
    rep("fwd", "t" #U, time_it([&](int i) { hipLaunchKernelGGL((fwd_tile<U>), dim3(g), dim3(256), 0, 0, S[i].a, s, b, S[i].d, M, C); }, NS, reps), fb); }
    FT(1) FT(2) FT(4) FT(8)
    const double bb = el * 8, bm = el * (6 + 0.125);
    rep("bwd_relu", "v0", time_it([&](int i) { hipLaunchKernelGGL(bwd_v0, dim3(g0), dim3(256), 0, 0, S[i].a, S[i].b, S[i].c, A, B, Cc, S[i].d, M, C); }, NS, reps), bb);
#define BT(U) { int g = (int)((M + mp.rpb * U - 1) / (mp.rpb * U)); \
    rep("bwd_relu", "t" #U, time_it([&](int i) { hipLaunchKernelGGL((bwd_tile<U, false>), dim3(g), dim3(256), 0, 0, S[i].a, S[i].b, S[i].m, S[i].c, A, B, Cc, S[i].d, M, C); }, NS, reps), bb); \
    rep("bwd_relu", "m" #U, time_it([&](int i) { hipLaunchKernelGGL((bwd_tile<U, true>), dim3(g), dim3(256), 0, 0, S[i].a, S[i].b, S[i].m, S[i].c, A, B, Cc, S[i].d, M, C); }, NS, reps), bm); }
    BT(1) BT(2) BT(4)
  }
  return 0;
}
