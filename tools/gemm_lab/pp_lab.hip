// Ping-pong main-loop lab (csrc/kernels/gemm_pp.hpp) against the 2-phase main loop's best
// 256x256 config (gemm_core.hpp, tile config 6), same process, same random operands
// (uniform [-1, 1)), variants timed in interleaved rounds (cdna_hip_programming.md §5.4 rule 24).
// Every result is checked against a naive fp32-accumulation kernel.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I csrc tools/gemm_lab/pp_lab.hip -o pp_lab
//   ./pp_lab [shape_index]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kernels/conv_common.hpp"
#include "kernels/gemm_pp.hpp"

using namespace mipipe;
using namespace mipipe::gk;

static __device__ __attribute__((aligned(64))) uint4 lab_zero[8];

// ---- new loop: 256 x 256 tile, 8 waves 2 x 4, half-tile policies -----------------------------
template <bool A_KC, bool B_KC, int V>
__global__ __launch_bounds__(512, 1) void pp_kernel(const __bf16* __restrict__ A, long lda,
                                                    const __bf16* __restrict__ B, long ldb,
                                                    __bf16* __restrict__ C, uint32_t M,
                                                    uint32_t N, uint32_t K, uint32_t tilesN) {
  constexpr int BM = 256, BN = 256, HM = 128, HN = 128;
  typedef typename std::conditional<A_KC, KCDense<HM, __bf16, 8>, MCDense<HM, __bf16, 8>>::type OpA;
  typedef typename std::conditional<B_KC, KCDense<HN, __bf16, 8>, MCDense<HN, __bf16, 8>>::type OpB;
  typedef MainLoopPP<BM, BN, OpA, OpB, 2, 4, V> ML;
  __shared__ __attribute__((aligned(16))) char smem[ML::LDS_BYTES];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t id = xcd_remap(blockIdx.x, gridDim.x);
  const uint32_t tm = id / tilesN, tn = id % tilesN;
  const uint32_t m0 = tm * BM, n0 = tn * BN;
  const int nk = (int)((K + BK - 1) / BK);
  OpA a[2];
  OpB b[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    a[h].init(A, lda, M, K, m0 + h * HM, wave, lane, lab_zero);
    b[h].init(B, ldb, N, K, n0 + h * HN, wave, lane, lab_zero);
  }
  f32x4 acc[ML::MT][ML::NT];
  ML::run(smem, a, b, 0, nk, acc, wave, lane);
  const int wr = wave / 4, wc = wave % 4;
#pragma unroll
  for (int i = 0; i < ML::MT; ++i)
#pragma unroll
    for (int j = 0; j < ML::NT; ++j) {
      const uint32_t m = m0 + ML::row(wr, i) + (lane & 15);
      const uint32_t n = n0 + ML::col(wc, j) + (lane >> 4) * 4;
      if (m < M && n < N) {
        uint2 v = make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
        *reinterpret_cast<uint2*>(C + (long)m * N + n) = v;
      }
    }
}

// ---- old loop, tile config 6 (256 x 256, 2 stages, 4 x 2 waves, raw barrier + prio) -----------
template <bool A_KC, bool B_KC>
__global__ __launch_bounds__(512, 1) void old_kernel(const __bf16* __restrict__ A, long lda,
                                                     const __bf16* __restrict__ B, long ldb,
                                                     __bf16* __restrict__ C, uint32_t M,
                                                     uint32_t N, uint32_t K, uint32_t tilesN) {
  typedef T6 Cf;
  constexpr int BM = Cf::BM, BN = Cf::BN, NW = Cf::NW;
  typedef typename std::conditional<A_KC, KCDense<BM, __bf16, NW>, MCDense<BM, __bf16, NW>>::type OpA;
  typedef typename std::conditional<B_KC, KCDense<BN, __bf16, NW>, MCDense<BN, __bf16, NW>>::type OpB;
  typedef MainLoop<BM, BN, OpA, OpB, Cf::NS, Cf::WM, Cf::WN, 3> ML;
  __shared__ __attribute__((aligned(16))) char smem[ML::LDS_BYTES];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t id = xcd_remap(blockIdx.x, gridDim.x);
  const uint32_t tm = id / tilesN, tn = id % tilesN;
  const uint32_t m0 = tm * BM, n0 = tn * BN;
  const int nk = (int)((K + BK - 1) / BK);
  OpA a;
  a.init(A, lda, M, K, m0, wave, lane, lab_zero);
  OpB b;
  b.init(B, ldb, N, K, n0, wave, lane, lab_zero);
  f32x4 acc[BM / Cf::WM / 16][BN / Cf::WN / 16];
  ML::run(smem, a, b, 0, nk, acc, wave, lane);
  const int wr = wave / Cf::WN, wc = wave % Cf::WN;
#pragma unroll
  for (int i = 0; i < BM / Cf::WM / 16; ++i)
#pragma unroll
    for (int j = 0; j < BN / Cf::WN / 16; ++j) {
      const uint32_t m = m0 + wr * (BM / Cf::WM) + i * 16 + (lane & 15);
      const uint32_t n = n0 + wc * (BN / Cf::WN) + j * 16 + (lane >> 4) * 4;
      if (m < M && n < N) {
        uint2 v = make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
        *reinterpret_cast<uint2*>(C + (long)m * N + n) = v;
      }
    }
}

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

static void check(hipError_t e, const char* w) {
  if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", w, hipGetErrorString(e)); exit(1); }
}

struct Shape { const char* name; int M, N, K; bool akc, bkc; };
typedef void (*Kern)(const __bf16*, long, const __bf16*, long, __bf16*, uint32_t, uint32_t,
                     uint32_t, uint32_t);
struct Variant { const char* name; Kern k; int threads; };

template <bool AK, bool BK_>
static std::vector<Variant> variants() {
  return {
      {"old_cfg6", old_kernel<AK, BK_>, 512},
      {"pp_stag_prio", pp_kernel<AK, BK_, kPPPrio | kPPStagger>, 512},
      {"pp_stag", pp_kernel<AK, BK_, kPPStagger>, 512},
      {"pp_lockstep_prio", pp_kernel<AK, BK_, kPPPrio>, 512},
  };
}

int main(int argc, char** argv) {
  int only = argc > 1 ? atoi(argv[1]) : -1;
  int rounds = argc > 2 ? atoi(argv[2]) : 5;
  std::vector<Shape> shapes = {
      {"sq4096", 4096, 4096, 4096, true, true},
      {"sq8192", 8192, 8192, 8192, true, true},
      {"bert_qkv_fwd", 4096, 2304, 768, true, true},
      {"bert_ffn1_fwd", 4096, 3072, 768, true, true},
      {"bert_ffn2_fwd", 4096, 768, 3072, true, true},
      {"bert_ao_fwd", 4096, 768, 768, true, true},
      {"bert_ffn1_dx", 4096, 768, 3072, true, false},
      {"bert_qkv_dx", 4096, 768, 2304, true, false},
      {"bert_ffn1_dw", 3072, 768, 4096, false, false},
      {"sq4096_nn", 4096, 4096, 4096, true, false},
      {"sq4096_tn", 4096, 4096, 4096, false, false},
      {"ragged", 1000, 1500, 700, true, true},
  };
  size_t maxA = 0, maxB = 0, maxC = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K);
    maxB = std::max(maxB, (size_t)s.N * s.K);
    maxC = std::max(maxC, (size_t)s.M * s.N);
  }
  __bf16 *A, *B, *C;
  float* Cref;
  check(hipMalloc(&A, maxA * 2), "malloc");
  check(hipMalloc(&B, maxB * 2), "malloc");
  check(hipMalloc(&C, maxC * 2), "malloc");
  check(hipMalloc(&Cref, maxC * 4), "malloc");
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (size_t si = 0; si < shapes.size(); ++si) {
    if (only >= 0 && (int)si != only) continue;
    const Shape& s = shapes[si];
    long na = (long)s.M * s.K, nb = (long)s.N * s.K, nc = (long)s.M * s.N;
    hipLaunchKernelGGL(fill_kernel, dim3((na + 255) / 256), dim3(256), 0, 0, A, na, 17u + si);
    hipLaunchKernelGGL(fill_kernel, dim3((nb + 255) / 256), dim3(256), 0, 0, B, nb, 91u + si);
    hipLaunchKernelGGL(ref_kernel, dim3((nc + 255) / 256), dim3(256), 0, 0, A, s.akc, B, s.bkc,
                       s.M, s.N, s.K, Cref);
    check(hipDeviceSynchronize(), "ref");
    std::vector<float> ref(nc);
    check(hipMemcpy(ref.data(), Cref, nc * 4, hipMemcpyDeviceToHost), "copy");
    std::vector<Variant> vs = s.akc ? (s.bkc ? variants<true, true>() : variants<true, false>())
                                    : (s.bkc ? variants<false, true>() : variants<false, false>());
    const uint32_t tN = (s.N + 255) / 256, tiles = ((s.M + 255) / 256) * tN;
    const long lda = s.akc ? s.K : s.M, ldb = s.bkc ? s.K : s.N;
    std::vector<double> err(vs.size());
    std::vector<std::vector<float>> times(vs.size());
    for (size_t v = 0; v < vs.size(); ++v) {
      hipMemset(C, 0xFF, nc * 2);
      hipLaunchKernelGGL(vs[v].k, dim3(tiles), dim3(vs[v].threads), 0, 0, A, lda, B, ldb, C,
                         (uint32_t)s.M, (uint32_t)s.N, (uint32_t)s.K, tN);
      check(hipDeviceSynchronize(), vs[v].name);
      std::vector<__bf16> h(nc);
      check(hipMemcpy(h.data(), C, nc * 2, hipMemcpyDeviceToHost), "copy");
      double mx = 0, rm = 0;
      for (long i = 0; i < nc; ++i) {
        double d = fabs((double)(float)h[i] - ref[i]);
        if (!(d == d)) d = 1e30;
        mx = std::max(mx, d);
        rm = std::max(rm, (double)fabsf(ref[i]));
      }
      err[v] = mx / (rm + 1e-9);
    }
    const int reps = s.M * (double)s.N * s.K > 1e11 ? 5 : 20;
    for (int r = 0; r < rounds; ++r)
      for (size_t v = 0; v < vs.size(); ++v) {
        for (int i = 0; i < 2; ++i)
          hipLaunchKernelGGL(vs[v].k, dim3(tiles), dim3(vs[v].threads), 0, 0, A, lda, B, ldb, C,
                             (uint32_t)s.M, (uint32_t)s.N, (uint32_t)s.K, tN);
        hipEventRecord(e0, 0);
        for (int i = 0; i < reps; ++i)
          hipLaunchKernelGGL(vs[v].k, dim3(tiles), dim3(vs[v].threads), 0, 0, A, lda, B, ldb, C,
                             (uint32_t)s.M, (uint32_t)s.N, (uint32_t)s.K, tN);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        times[v].push_back(ms / reps);
      }
    for (size_t v = 0; v < vs.size(); ++v) {
      std::vector<float> t = times[v];
      std::sort(t.begin(), t.end());
      const double flop = 2.0 * s.M * s.N * s.K;
      printf("{\"shape\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"var\": \"%s\", "
             "\"us_min\": %.2f, \"us_med\": %.2f, \"tflops_min\": %.1f, \"tflops_med\": %.1f, "
             "\"rel_err\": %.2e}\n",
             s.name, s.M, s.N, s.K, vs[v].name, t[0] * 1e3, t[t.size() / 2] * 1e3,
             flop / (t[0] * 1e-3) / 1e12, flop / (t[t.size() / 2] * 1e-3) / 1e12, err[v]);
      fflush(stdout);
    }
  }
  return 0;
}
