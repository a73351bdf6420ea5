// Dense bf16 / fp32 (split-bf16) GEMM on the shared MFMA core (Linear forward / data-grad /
// weight-grad).
//   C[M][N] = op(A) op(B);  A stored [M][K] (KC) or [K][M] (MC);  B stored [N][K] (KC) or [K][N] (MC)
// Output modes: 0 activation dtype (+bias +ReLU epilogue), 1 fp32 store (+bias),
// 2 fp32 accumulate into C (beta = 1): split-K with fp32 atomics (splits > 1) or one block per
// output element with a plain read-modify-write (splits == 1, no atomics; also the
// deterministic path).
// Every kernel is a template over the conv tile table (conv_common.hpp); the host picks a
// (tile, splits) plan per shape: the benchmark-mode tuning table (bindings.cpp, tune::) or the
// heuristic below.  Dense GEMMs run the main loop with the raw-barrier / MFMA-priority schedule
// (tools/gemm_lab: +1..12 % over plain __syncthreads on BERT / square shapes).
#include "conv_common.hpp"

namespace mipipe {
int g_splitk_target = 512;
int g_ns1_max_k_gather = 1152;  // measured: tools/sweep_ns1_gather.py (profiles/r1_ns1_gather_sweep.jsonl)
int g_stat_rows = kStatReplicas;
// Non-temporal (streaming) stores of large activation outputs, a bit mask: 1 conv forward,
// 2 conv data-grad, 4 BN forward apply, 8 BN backward apply, 16 the stem's stored conv output,
// 32 / 64 streaming LOADS in the BN forward / backward apply, 128 Linear (GEMM) outputs,
// 256 streaming loads of the fused data-grad epilogue operands, 512 the stem backward's y,
// 1024 streaming fp32 state in AdamW
// (MIPIPE_NT_STORE overrides; A/B in profiles/r4_nt_store_ab.txt)
int g_nt_store = [] {
  const char* v = getenv("MIPIPE_NT_STORE");
  return v != nullptr ? atoi(v) : 1379;  // conv stores, BN-pass + dgrad-epi loads, AdamW state
}();
// Outputs up to this many bytes keep the default (cached) store policy even when their g_nt_store
// bit is set: a tensor that fits the 256 MB MALL is re-read from it by the pass right after
// (the BN apply reading a layer-3/4 conv output); only larger ones stream past it
// (MIPIPE_NT_MIN_MB overrides; 0 = the bit alone decides)
long g_nt_min_bytes = [] {
  const char* v = getenv("MIPIPE_NT_MIN_MB");
  return (long)(v != nullptr ? atof(v) : 0.0) * (1l << 20);
}();
int g_ns1_max_k = 512;  // measured: tools/sweep_ns1.py (profiles/r1_ns1_sweep.jsonl)
// (e.pf_lines[1] == 0xFFFFFFFF would enable pf_sink's store: lines are capped below it)
void set_prefetch(gk::EpiParams& e, const TouchRanges* pf) {
  if (pf == nullptr) return;
  for (int r = 0; r < 2 && r < pf->count; ++r) {
    e.pf_ptr[r] = pf->ptr[r];
    e.pf_lines[r] = (uint32_t)std::min<long>(pf->bytes[r] >> 6, 0x7FFFFFFF);
  }
  if (e.pf_lines[0] == 0) {  // keep "range 0 empty" meaning "no prefetch"
    e.pf_ptr[0] = e.pf_ptr[1];
    e.pf_lines[0] = e.pf_lines[1];
    e.pf_lines[1] = 0;
  }
}
namespace gk {

__device__ __attribute__((aligned(64))) uint4 g_gemm_zero[8];
constexpr int kGemmLoop = kLoopRawBarrier | kLoopPrio;

// OUT: 0 activation dtype, 1 fp32 store / read-modify-write (e.rmw), 2 fp32 atomic (split-K),
// 3 activation dtype + e.addend (a same-shape tensor added in the epilogue: the second gradient
// of a tensor consumed twice, e.g. a residual stream, without a separate add)
template <class C, bool A_KC, bool B_KC, int OUT, class T>
__global__ __launch_bounds__(C::THREADS, (conv_occ<T, C>())) void gemm_dense_kernel(
    const T* __restrict__ A, long lda, const T* __restrict__ B, long ldb, uint32_t K,
    uint32_t tilesN, int kt_per_split, EpiParams e) {
  constexpr int BM = C::BM, BN = C::BN;
  typedef typename std::conditional<A_KC, PolKCDense<T>, PolMCDense<T>>::type PA;
  typedef typename std::conditional<B_KC, PolKCDense<T>, PolMCDense<T>>::type PB;
  constexpr int main_lds = main_lds_bytes<T, C>();
  constexpr int epi_lds = (OUT == 0 || OUT == 3) ? kEpiLdsBytes<BM, BN, T, C::WM>()
                                                 : kEpiF32Rows<BM, BN, C::PP>() * (BN * 4 + 16);
  __shared__ __attribute__((aligned(16))) char smem[main_lds > epi_lds ? main_lds : epi_lds];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t id = xcd_remap(blockIdx.x, gridDim.x);
  const uint32_t tm = id / tilesN, tn = id % tilesN;
  const uint32_t m0 = tm * BM, n0 = tn * BN;
  const int nk = (int)((K + BK - 1) / BK);
  const int kt0 = blockIdx.y * kt_per_split;
  const int kt1 = min(nk, kt0 + kt_per_split);
  auto ia = [&](auto& a, uint32_t origin) { a.init(A, lda, e.M, K, origin, wave, lane, g_gemm_zero); };
  auto ib = [&](auto& b, uint32_t origin) { b.init(B, ldb, e.N, K, origin, wave, lane, g_gemm_zero); };
  // cache warming for the next GEMM (e.pf_*): issued first, so the loads overlap the main loop
  const uint32_t pf_acc =
      pf_issue<C::THREADS>(e, blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  f32x4 acc[BM / C::WM / 16][BN / C::WN / 16];
  run_main_loop<T, C, PA, PB, kGemmLoop>(smem, ia, ib, m0, n0, kt0, kt1, acc, wave, lane);
  if constexpr (OUT == 0)
    epilogue_out<BM, BN, false, T, C::WM, C::WN, false, C::PP>(smem, acc, e, m0, n0, 0, wave, lane);
  else if constexpr (OUT == 3)
    epilogue_out<BM, BN, true, T, C::WM, C::WN, false, C::PP>(smem, acc, e, m0, n0, 0, wave, lane);
  else
    epilogue_f32<BM, BN, OUT == 2, C::WM, C::WN, C::PP>(smem, acc, e, m0, n0, wave, lane);
  pf_sink(e, pf_acc, smem);
}

}  // namespace gk

using namespace gk;

static inline uint32_t cdiv_u(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

template <class C, bool AK, bool BK_, class T>
static void launch_out(const void* A, long lda, const void* B, long ldb, int K, uint32_t tN,
                       uint32_t tiles, int splits, int per, int out, const EpiParams& e,
                       hipStream_t st) {
  dim3 grid(tiles, splits);
  const T* a = (const T*)A;
  const T* b = (const T*)B;
  // a 256 x 256 fp32 tile does not fit the LDS: the 2-phase loop's 256 x 256 tile only serves
  // out 0 (with_tile maps the fp32-output modes to 256 x 128); the ping-pong one stages halves
  constexpr bool kWide = C::BM * C::BN > 256 * 128 && !C::PP;
  if (out == 3) {  // addend epilogue: instantiated for the data-grad layout (A [M][K], B [K][N])
    if constexpr (AK && !BK_)
      hipLaunchKernelGGL((gemm_dense_kernel<C, AK, BK_, 3, T>), grid, dim3(C::THREADS), 0, st, a, lda, b, ldb, (uint32_t)K, tN, per, e);
  } else if (out == 0) {
    hipLaunchKernelGGL((gemm_dense_kernel<C, AK, BK_, 0, T>), grid, dim3(C::THREADS), 0, st, a, lda, b, ldb, (uint32_t)K, tN, per, e);
  } else if constexpr (!kWide) {
    if (out == 1)
      hipLaunchKernelGGL((gemm_dense_kernel<C, AK, BK_, 1, T>), grid, dim3(C::THREADS), 0, st, a, lda, b, ldb, (uint32_t)K, tN, per, e);
    else
      hipLaunchKernelGGL((gemm_dense_kernel<C, AK, BK_, 2, T>), grid, dim3(C::THREADS), 0, st, a, lda, b, ldb, (uint32_t)K, tN, per, e);
  }
}

// split count for an accumulating (out == 2) GEMM: `splits` > 0 is the tuned value; else split
// K until ~g_splitk_target blocks with >= 4 k-steps per split, at most 4 ways (every split
// adds M*N*4 bytes of atomics, and those run at ~1.3 TB/s chip-wide).
static int plan_splits(uint32_t tiles, int nk, int splits) {
  if (g_deterministic) return 1;  // one block per output element: read-modify-write, no atomics
  if (splits > 0) return std::min(splits, std::max(1, nk));
  int s = std::min<int>(g_splitk_target / std::max<uint32_t>(1, tiles), nk / 4);
  return std::max(1, std::min(s, 4));
}

int gemm_ws_splits(int K, int splits) {
  const int nk = (int)cdiv_u(K, 64);
  const int per = (int)cdiv_u(nk, std::max(1, std::min(splits, nk)));
  return (int)cdiv_u(nk, per);
}

template <class C, class T>
static void launch_tile(const void* A, long lda, bool a_kc, const void* B, long ldb, bool b_kc,
                        int M, int N, int K, int out, EpiParams e, int splits_req,
                        hipStream_t st, bool ws_split, const WsFinish* fin) {
  uint32_t tN = cdiv_u(N, C::BN), tiles = cdiv_u(M, C::BM) * tN;
  int nk = (int)cdiv_u(K, 64);
  int splits = 1, per = nk;
  if (out == 2 && ws_split) {  // per-split workspace slices (epilogue_f32's det_rows path)
    splits = gemm_ws_splits(K, splits_req);
    per = (int)cdiv_u(nk, splits);
    e.det_rows = 1;
    if (fin != nullptr) e.fin = *fin;  // the last split of each tile finishes the sum
  } else if (out == 2) {
    splits = plan_splits(tiles, nk, splits_req);
    per = (int)cdiv_u(nk, splits);
    splits = (int)cdiv_u(nk, per);
    if (splits == 1) {  // sole writer of its tile: plain read-modify-write epilogue
      out = 1;
      e.rmw = 1;
    }
  }
  if (a_kc && b_kc) launch_out<C, true, true, T>(A, lda, B, ldb, K, tN, tiles, splits, per, out, e, st);
  else if (a_kc && !b_kc) launch_out<C, true, false, T>(A, lda, B, ldb, K, tN, tiles, splits, per, out, e, st);
  else if (!a_kc && b_kc) launch_out<C, false, true, T>(A, lda, B, ldb, K, tN, tiles, splits, per, out, e, st);
  else launch_out<C, false, false, T>(A, lda, B, ldb, K, tN, tiles, splits, per, out, e, st);
}

// heuristic tile (no tuning-table entry): 64-wide tiles for narrow dimensions, else 128x128
int default_gemm_cfg(int M, int N, bool f32) {
  (void)f32;
  if (N <= 64) return 2;
  if (M <= 64) return 8;
  return 0;
}

template <class T>
static void gemm_t(const void* A, long lda, bool a_kc, const void* B, long ldb, bool b_kc, int M,
                   int N, int K, int out, const EpiParams& e, int cfg, int splits,
                   hipStream_t st, bool ws_split, const WsFinish* fin) {
  if (cfg < 0 || !tile_ok_for<T>(cfg)) cfg = default_gemm_cfg(M, N, std::is_same<T, float>::value);
  auto go = [&](auto tile) {
    typedef decltype(tile) C;
    launch_tile<C, T>(A, lda, a_kc, B, ldb, b_kc, M, N, K, out, e, splits, st, ws_split, fin);
  };
  // fp32-output modes stage BM x BN fp32 in LDS: no 256 x 256 tile there
  if (out == 0 || out == 3) with_tile<T, false>(cfg, go);
  else with_tile<T, true>(cfg, go);
}

void gemm(const void* A, long lda, bool a_kc, const void* B, long ldb, bool b_kc, void* C,
          long ldc, int M, int N, int K, const float* bias, int act, int out, hipStream_t st,
          bool f32, int cfg, int splits, const void* addend, bool ws_split, const WsFinish* fin,
          void* aux, const TouchRanges* pf) {
  EpiParams e{};
  set_prefetch(e, pf);
  e.C = C; e.ldc = ldc; e.M = (uint32_t)M; e.N = (uint32_t)N; e.bias = bias; e.act = act;
  if (act == 2) {  // GELU: bf16 activation output with the pre-activation in aux
    e.act = 0;
    e.aux = aux;
  }
  e.nt = (g_nt_store >> 7) & 1;
  if (addend != nullptr && out == 0 && a_kc && !b_kc) {
    e.addend = addend;
    out = 3;
  }
  ws_split = ws_split && out == 2 && splits > 1 && bias == nullptr;
  if (fin != nullptr && (!ws_split || N % 4 != 0 || ldc != N || fin->ticket == nullptr)) fin = nullptr;
  if (f32) gemm_t<float>(A, lda, a_kc, B, ldb, b_kc, M, N, K, out, e, cfg, splits, st, ws_split, fin);
  else gemm_t<__bf16>(A, lda, a_kc, B, ldb, b_kc, M, N, K, out, e, cfg, splits, st, ws_split, fin);
}

}  // namespace mipipe
