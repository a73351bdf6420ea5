// Dense bf16 / fp32 (split-bf16) GEMM on the shared MFMA core (Linear forward / data-grad / weight-grad).
//   C[M][N] = op(A) op(B);  A stored [M][K] (KC) or [K][M] (MC);  B stored [N][K] (KC) or [K][N] (MC)
// Output: bf16 (+bias +ReLU epilogue), fp32 store (+bias) or fp32 split-K atomic accumulate.
#include "epilogue.hpp"
#include "launchers.hpp"

namespace mipipe {
int g_splitk_target = 512;
int g_ns1_max_k_gather = 1152;  // measured: tools/sweep_ns1_gather.py (profiles/r1_ns1_gather_sweep.jsonl)
int g_stat_rows = kStatReplicas;
int g_ns1_max_k = 512;  // measured: tools/sweep_ns1.py (profiles/r1_ns1_sweep.jsonl)
namespace gk {

__device__ __attribute__((aligned(64))) uint4 g_gemm_zero[8];

template <int BM, int BN, bool A_KC, bool B_KC, int OUT, class T = __bf16>
__global__ __launch_bounds__(256, 2) void gemm_dense_kernel(const T* __restrict__ A, long lda,
                                                             const T* __restrict__ B, long ldb,
                                                             uint32_t K, uint32_t tilesN,
                                                             int kt_per_split, EpiParams e) {
  typedef typename std::conditional<A_KC, KCDense<BM, T>, MCDense<BM, T>>::type OpA;
  typedef typename std::conditional<B_KC, KCDense<BN, T>, MCDense<BN, T>>::type OpB;
  typedef MainLoopFor<T, BM, BN, OpA, OpB> ML;
  constexpr int main_lds = ML::LDS_BYTES;
  constexpr int epi_lds = OUT == 0 ? kEpiLdsBytes<BM, BN, T>() : BM * (BN * 4 + 16);
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
  a.init(A, lda, e.M, K, m0, wave, lane, g_gemm_zero);
  OpB b;
  b.init(B, ldb, e.N, K, n0, wave, lane, g_gemm_zero);
  f32x4 acc[BM / 32][BN / 32];
  ML::type::run(smem, a, b, kt0, kt1, acc, wave, lane);
  if constexpr (OUT == 0) epilogue_out<BM, BN, false, T>(smem, acc, e, m0, n0, 0, wave, lane);
  else if constexpr (OUT == 1) epilogue_f32<BM, BN, false>(smem, acc, e, m0, n0, wave, lane);
  else epilogue_f32<BM, BN, true>(smem, acc, e, m0, n0, wave, lane);
}

}  // namespace gk

using namespace gk;

static inline uint32_t cdiv_u(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

template <int BM, int BN, bool AK, bool BK_, class T>
static void launch_out(const void* A, long lda, const void* B, long ldb, int K, uint32_t tN,
                       uint32_t tiles, int splits, int per, int out, const EpiParams& e,
                       hipStream_t st) {
  dim3 grid(tiles, splits);
  const T* a = (const T*)A;
  const T* b = (const T*)B;
  if (out == 0)
    hipLaunchKernelGGL((gemm_dense_kernel<BM, BN, AK, BK_, 0, T>), grid, dim3(256), 0, st, a, lda, b, ldb, (uint32_t)K, tN, per, e);
  else if (out == 1)
    hipLaunchKernelGGL((gemm_dense_kernel<BM, BN, AK, BK_, 1, T>), grid, dim3(256), 0, st, a, lda, b, ldb, (uint32_t)K, tN, per, e);
  else
    hipLaunchKernelGGL((gemm_dense_kernel<BM, BN, AK, BK_, 2, T>), grid, dim3(256), 0, st, a, lda, b, ldb, (uint32_t)K, tN, per, e);
}

template <int BM, int BN, class T>
static void launch_tile(const void* A, long lda, bool a_kc, const void* B, long ldb, bool b_kc,
                        int M, int N, int K, int out, const EpiParams& e, hipStream_t st) {
  uint32_t tN = cdiv_u(N, BN), tiles = cdiv_u(M, BM) * tN;
  int nk = (int)cdiv_u(K, 64);
  int splits = 1, per = nk;
  if (out == 2 && !g_deterministic) {  // split-K until ~g_splitk_target blocks, >= 4 k-steps per split
    // (deterministic mode: one split, so every output element is written by one block)
    splits = std::max<int>(1, std::min<int>(g_splitk_target / std::max<uint32_t>(1, tiles), nk / 4));
    per = (int)cdiv_u(nk, splits);
    splits = (int)cdiv_u(nk, per);
  }
  if (a_kc && b_kc) launch_out<BM, BN, true, true, T>(A, lda, B, ldb, K, tN, tiles, splits, per, out, e, st);
  else if (a_kc && !b_kc) launch_out<BM, BN, true, false, T>(A, lda, B, ldb, K, tN, tiles, splits, per, out, e, st);
  else if (!a_kc && b_kc) launch_out<BM, BN, false, true, T>(A, lda, B, ldb, K, tN, tiles, splits, per, out, e, st);
  else launch_out<BM, BN, false, false, T>(A, lda, B, ldb, K, tN, tiles, splits, per, out, e, st);
}

template <class T>
static void gemm_t(const void* A, long lda, bool a_kc, const void* B, long ldb, bool b_kc,
                   int M, int N, int K, int out, const EpiParams& e, hipStream_t st) {
  // tile choice: 64-wide tiles for narrow dimensions (MC images support W = 64 and 128)
  if (N <= 64) launch_tile<128, 64, T>(A, lda, a_kc, B, ldb, b_kc, M, N, K, out, e, st);
  else if (M <= 64) launch_tile<64, 128, T>(A, lda, a_kc, B, ldb, b_kc, M, N, K, out, e, st);
  else launch_tile<128, 128, T>(A, lda, a_kc, B, ldb, b_kc, M, N, K, out, e, st);
}

void gemm(const void* A, long lda, bool a_kc, const void* B, long ldb, bool b_kc, void* C,
          long ldc, int M, int N, int K, const float* bias, int act, int out, hipStream_t st,
          bool f32) {
  EpiParams e{};
  e.C = C; e.ldc = ldc; e.M = (uint32_t)M; e.N = (uint32_t)N; e.bias = bias; e.act = act;
  if (f32) gemm_t<float>(A, lda, a_kc, B, ldb, b_kc, M, N, K, out, e, st);
  else gemm_t<__bf16>(A, lda, a_kc, B, ldb, b_kc, M, N, K, out, e, st);
}

}  // namespace mipipe
