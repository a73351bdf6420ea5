// GEMM main-loop lab: times the dense MFMA GEMM (the Linear / 1x1-conv kernel) for every
// (tile config x main-loop schedule variant) on BERT-base and square shapes, checks each result
// against a naive fp32-accumulation kernel, prints one JSON line per (shape, config, variant).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I csrc tools/gemm_lab/lab.hip -o lab && ./lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kernels/conv_common.hpp"

using namespace mipipe;
using namespace mipipe::gk;

static __device__ __attribute__((aligned(64))) uint4 lab_zero[8];

template <class C, bool A_KC, bool B_KC, int OUT, int V>
__global__ __launch_bounds__(C::THREADS, (conv_occ<__bf16, C>())) void lab_kernel(
    const __bf16* __restrict__ A, long lda, const __bf16* __restrict__ B, long ldb, uint32_t K,
    uint32_t tilesN, int kt_per_split, EpiParams e) {
  constexpr int BM = C::BM, BN = C::BN, NW = C::NW;
  typedef typename std::conditional<A_KC, KCDense<BM, __bf16, NW>, MCDense<BM, __bf16, NW>>::type OpA;
  typedef typename std::conditional<B_KC, KCDense<BN, __bf16, NW>, MCDense<BN, __bf16, NW>>::type OpB;
  typedef MainLoop<BM, BN, OpA, OpB, C::NS, C::WM, C::WN, V> ML;
  constexpr int main_lds = ML::LDS_BYTES;
  constexpr int epi_lds = OUT == 0 ? kEpiLdsBytes<BM, BN, __bf16, C::WM>() : BM * (BN * 4 + 16);
  __shared__ __attribute__((aligned(16))) char smem[main_lds > epi_lds ? main_lds : epi_lds];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t id = xcd_remap(blockIdx.x, gridDim.x);
  const uint32_t tm = id / tilesN, tn = id % tilesN;
  const uint32_t m0 = tm * BM, n0 = tn * BN;
  const int nk = (int)((K + BK - 1) / BK);
  const int kt0 = blockIdx.y * kt_per_split;
  const int kt1 = min(nk, kt0 + kt_per_split);
  OpA a;
  a.init(A, lda, e.M, K, m0, wave, lane, lab_zero);
  OpB b;
  b.init(B, ldb, e.N, K, n0, wave, lane, lab_zero);
  f32x4 acc[BM / C::WM / 16][BN / C::WN / 16];
  ML::run(smem, a, b, kt0, kt1, acc, wave, lane);
  if constexpr (OUT == 0) epilogue_out<BM, BN, false, __bf16, C::WM, C::WN>(smem, acc, e, m0, n0, 0, wave, lane);
  else epilogue_f32<BM, BN, true, C::WM, C::WN>(smem, acc, e, m0, n0, wave, lane);
}

// naive reference: Cref[m][n] = sum_k A(m,k) B(k,n) in fp32
__global__ void ref_kernel(const __bf16* A, bool akc, const __bf16* B, bool bkc, int M, int N,
                           int K, float* C) {
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)M * N) return;
  int m = (int)(t / N), n = (int)(t % N);
  float s = 0.f;
  for (int k = 0; k < K; ++k) {
    float a = (float)(akc ? A[(long)m * K + k] : A[(long)k * M + m]);
    float b = (float)(bkc ? B[(long)n * K + k] : B[(long)k * N + n]);
    s += a * b;
  }
  C[t] = s;
}

__global__ void fill_kernel(__bf16* p, long n, uint32_t seed) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t h = (uint32_t)i * 2654435761u ^ seed;
  h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
  p[i] = (__bf16)(((h & 0xffff) / 65535.f) * 2.f - 1.f);
}

__global__ void to_f32(const __bf16* p, float* q, long n) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) q[i] = (float)p[i];
}

struct Shape { const char* name; int M, N, K; bool akc, bkc; int out; };

static float g_err;
static void check(hipError_t e, const char* w) {
  if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", w, hipGetErrorString(e)); exit(1); }
}

template <class C, bool AK, bool BK_, int OUT, int V>
static void run_one(const Shape& s, const __bf16* A, const __bf16* B, void* Cout, float* Cf,
                    const float* Cref, int cfg) {
  uint32_t tN = (s.N + C::BN - 1) / C::BN, tiles = ((s.M + C::BM - 1) / C::BM) * tN;
  int nk = (s.K + 63) / 64, splits = 1, per = nk;
  if (OUT == 2) {
    splits = std::max<int>(1, std::min<int>(512 / std::max<uint32_t>(1, tiles), nk / 4));
    per = (nk + splits - 1) / splits;
    splits = (nk + per - 1) / per;
  }
  EpiParams e{};
  e.C = Cout; e.ldc = s.N; e.M = s.M; e.N = s.N;
  long lda = AK ? s.K : s.M, ldb = BK_ ? s.K : s.N;
  dim3 grid(tiles, splits);
  auto launch = [&]() {
    if (OUT == 2) hipMemsetAsync(Cout, 0, (size_t)s.M * s.N * 4, 0);
    hipLaunchKernelGGL((lab_kernel<C, AK, BK_, OUT, V>), grid, dim3(C::THREADS), 0, 0, A, lda, B,
                       ldb, (uint32_t)s.K, tN, per, e);
  };
  launch();
  check(hipDeviceSynchronize(), "launch");
  // error vs reference
  long n = (long)s.M * s.N;
  const float* cmp = Cf;
  if (OUT == 0) {
    hipLaunchKernelGGL(to_f32, dim3((n + 255) / 256), dim3(256), 0, 0, (const __bf16*)Cout, Cf, n);
  } else {
    cmp = (const float*)Cout;
  }
  std::vector<float> h(n), r(n);
  check(hipMemcpy(h.data(), cmp, n * 4, hipMemcpyDeviceToHost), "copy");
  check(hipMemcpy(r.data(), Cref, n * 4, hipMemcpyDeviceToHost), "copy");
  double mx = 0, ref = 0;
  for (long i = 0; i < n; ++i) {
    mx = std::max(mx, (double)fabsf(h[i] - r[i]));
    ref = std::max(ref, (double)fabsf(r[i]));
  }
  const int reps = 20;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) launch();
  float best = 1e30f;
  for (int round = 0; round < 3; ++round) {
    hipEventRecord(e0, 0);
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = std::min(best, ms / reps);
  }
  double tf = 2.0 * s.M * s.N * s.K / (best * 1e-3) / 1e12;
  printf("{\"shape\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"cfg\": %d, \"var\": %d, "
         "\"us\": %.2f, \"tflops\": %.1f, \"rel_err\": %.2e, \"blocks\": %u, \"splits\": %d}\n",
         s.name, s.M, s.N, s.K, cfg, V, best * 1e3, tf, mx / (ref + 1e-9), tiles, splits);
  fflush(stdout);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

template <bool AK, bool BK_, int OUT, int V>
static void sweep_cfgs(const Shape& s, const __bf16* A, const __bf16* B, void* Cout, float* Cf,
                       const float* Cref) {
  run_one<T0, AK, BK_, OUT, V>(s, A, B, Cout, Cf, Cref, 0);
  run_one<T1, AK, BK_, OUT, V>(s, A, B, Cout, Cf, Cref, 1);
  run_one<T3, AK, BK_, OUT, V>(s, A, B, Cout, Cf, Cref, 3);
  run_one<T4, AK, BK_, OUT, V>(s, A, B, Cout, Cf, Cref, 4);
  run_one<T5, AK, BK_, OUT, V>(s, A, B, Cout, Cf, Cref, 5);
  if constexpr (OUT == 0) run_one<T6, AK, BK_, OUT, V>(s, A, B, Cout, Cf, Cref, 6);
}

template <bool AK, bool BK_, int OUT>
static void sweep(const Shape& s, const __bf16* A, const __bf16* B, void* Cout, float* Cf,
                  const float* Cref, int vmask) {
  if (vmask & 1) sweep_cfgs<AK, BK_, OUT, 0>(s, A, B, Cout, Cf, Cref);
  if (vmask & 2) sweep_cfgs<AK, BK_, OUT, 1>(s, A, B, Cout, Cf, Cref);
  if (vmask & 4) sweep_cfgs<AK, BK_, OUT, 3>(s, A, B, Cout, Cf, Cref);
  if (vmask & 8) sweep_cfgs<AK, BK_, OUT, 7>(s, A, B, Cout, Cf, Cref);
  if (vmask & 16) sweep_cfgs<AK, BK_, OUT, 5>(s, A, B, Cout, Cf, Cref);
}

int main(int argc, char** argv) {
  int vmask = argc > 1 ? atoi(argv[1]) : 31;
  int only = argc > 2 ? atoi(argv[2]) : -1;
  std::vector<Shape> shapes = {
      {"bert_qkv_fwd", 4096, 2304, 768, true, true, 0},
      {"bert_ao_fwd", 4096, 768, 768, true, true, 0},
      {"bert_ffn1_fwd", 4096, 3072, 768, true, true, 0},
      {"bert_ffn2_fwd", 4096, 768, 3072, true, true, 0},
      {"bert_qkv_dx", 4096, 768, 2304, true, false, 0},
      {"bert_ffn2_dx", 4096, 3072, 768, true, false, 0},
      {"bert_ffn1_dx", 4096, 768, 3072, true, false, 0},
      {"bert_qkv_dw", 2304, 768, 4096, false, false, 2},
      {"bert_ao_dw", 768, 768, 4096, false, false, 2},
      {"bert_ffn1_dw", 3072, 768, 4096, false, false, 2},
      {"bert_ffn2_dw", 768, 3072, 4096, false, false, 2},
      {"sq4096", 4096, 4096, 4096, true, true, 0},
      {"r50_l1_c3_fwd", 200704, 256, 64, true, true, 0},
      {"r50_l3_c1_fwd", 50176, 256, 1024, true, true, 0},
  };
  size_t maxA = 0, maxB = 0, maxC = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K);
    maxB = std::max(maxB, (size_t)s.N * s.K);
    maxC = std::max(maxC, (size_t)s.M * s.N);
  }
  __bf16 *A, *B;
  void* C;
  float *Cf, *Cref;
  check(hipMalloc(&A, maxA * 2), "malloc");
  check(hipMalloc(&B, maxB * 2), "malloc");
  check(hipMalloc(&C, maxC * 4), "malloc");
  check(hipMalloc(&Cf, maxC * 4), "malloc");
  check(hipMalloc(&Cref, maxC * 4), "malloc");
  for (size_t si = 0; si < shapes.size(); ++si) {
    if (only >= 0 && (int)si != only) continue;
    const Shape& s = shapes[si];
    long na = (long)s.M * s.K, nb = (long)s.N * s.K;
    hipLaunchKernelGGL(fill_kernel, dim3((na + 255) / 256), dim3(256), 0, 0, A, na, 17u + si);
    hipLaunchKernelGGL(fill_kernel, dim3((nb + 255) / 256), dim3(256), 0, 0, B, nb, 91u + si);
    long nc = (long)s.M * s.N;
    hipLaunchKernelGGL(ref_kernel, dim3((nc + 255) / 256), dim3(256), 0, 0, A, s.akc, B, s.bkc,
                       s.M, s.N, s.K, Cref);
    check(hipDeviceSynchronize(), "ref");
    if (s.akc && s.bkc) sweep<true, true, 0>(s, A, B, C, Cf, Cref, vmask);
    else if (s.akc) sweep<true, false, 0>(s, A, B, C, Cf, Cref, vmask);
    else sweep<false, false, 2>(s, A, B, C, Cf, Cref, vmask);
  }
  return 0;
}
