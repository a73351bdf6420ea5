// GEMM epilogues: bf16 store (+bias, +ReLU, +BatchNorm partial statistics) and fp32
// store / split-K atomic accumulate.  All stage the tile through LDS so global traffic is
// whole 16-B (bf16) or 256-B-contiguous (fp32 atomics) row segments.
#pragma once
#include "gemm_core.hpp"
#include "launchers.hpp"

namespace mipipe {
namespace gk {

struct EpiParams {
  void* C;           // bf16 or fp32 output
  long ldc;
  uint32_t M, N;
  const float* bias;  // per column, may be null
  int act;            // 0 none, 1 relu
  // BatchNorm partials (per column, shifted): slab[prow][N] sum / sumsq; null if unused
  float* st_sum;
  float* st_sq;
  const float* st_shift;
  int st_R;  // number of replica rows in the stats slabs
  // optional output-row remap (strided dgrad classes): m -> (img, i, j) over an Hc x Wc grid,
  // stored at dx row (img*H + ph + s*i)*W + pw + s*j.  rm_s == 0 disables.
  int rm_s, rm_ph, rm_pw, rm_H, rm_W, rm_Hc, rm_Wc;
  FastDiv rm_fHcWc, rm_fWc;
  // optional [rows][ldc] tensor (output dtype) added to the output (residual-gradient fusion)
  const void* addend;
  // optional BatchNorm-backward fusion (conv dgrad whose input was relu(bn(y))): the output
  // becomes g = dx * [y*scale + bias > 0] and Σg, Σg·(y-mean)*invstd are accumulated into
  // replica rows (blockIdx % R) of rep[0] / rep[1] ([3][R][N] slab)
  const void* bnr_y;  // output dtype
  const float *bnr_mean, *bnr_invstd, *bnr_scale, *bnr_bias;
  float* bnr_rep;
  // when set, the ReLU mask is read from this stored post-activation tensor (z > 0) instead of
  // recomputed from y (needed when a residual was added before the ReLU)
  const void* bnr_z;  // output dtype
  // two-branch BN (ResNet downsample block output relu(bn(y) + bn2(y2))): Σg·x̂₂ goes to the
  // third slab array (TWO epilogues only)
  const void* bnr_y2;
  const float *bnr_mean2, *bnr_invstd2;
  const uint8_t* bnr_mask;  // or the mask as bits: [rows][ldc / 8] bytes, bit q = column 8c+q
  // deterministic mode (det_rows > 0): no float atomics.  Statistics partials (st_sum / st_sq,
  // bnr_rep) are WRITTEN at row det_row0 + (m0 / BM) of [det_rows][N] slabs (bnr_rep: two
  // arrays det_rows apart) and summed in a fixed order afterwards (det.hip); split-K fp32
  // outputs (epilogue_f32) are written to slice blockIdx.y of a [splits][M][ldc] workspace.
  int det_rows;
  int det_row0;
  // epilogue_f32 without ATOMIC: add the tile to the existing C (read-modify-write; each
  // element owned by one block) instead of overwriting it
  int rmw;
  // optional BN-backward collect done by block (0,0) of this launch (launchers.hpp BnCollect)
  BnCollect col;
  // workspace split-K finished by the last-arriving split (det_rows path; launchers.hpp)
  WsFinish fin;
  // non-temporal (streaming) stores of the output tile; streaming loads of the fused
  // data-grad epilogue's operand ring (addend / y / z)
  int nt, ntl;
  // act == 2 (GELU, plain bf16 store loop): the pre-activation goes to aux, GELU of it to C
  void* aux;
  // conv forward only: blocks >= fl_tiles write the tap-flipped sub-kernels its data-grad will
  // use (launchers.hpp FlipPlan: conv_dgrad's workspace layout) instead of an output tile
  const void* fl_w;
  void* fl_wt;
  int fl_Co, fl_KH, fl_KW, fl_Ci;
  uint32_t fl_tiles;
  FlipPlan fl;
  // split-K conv forward / forward-style data-grad (conv_common.hpp): split blockIdx.y runs
  // k-steps [y*split_kt, (y+1)*split_kt) and stores its fp32 partial tile in slice y of
  // split_ws [splits][M][N]; conv_splitk_finish_kernel sums the slices in order and runs the
  // regular epilogue (statistics / BN-backward fusions) on the sum
  int split_kt;
  float* split_ws;
  // folded BatchNorm on the conv INPUT (dense 1x1 bf16 forward / weight-grad, BNIN kernels): the
  // operand is y and the conv consumes relu(y*in_scale + in_bias) (gemm_core.hpp KCDenseBufBN /
  // MCDenseBufBN)
  const float* in_scale;
  const float* in_bias;
  // GEMM only: cache warming of the NEXT GEMM's cold operands (mipipe/ops/prefetch.py) — every
  // block issues one load per 64-B line of its share of these ranges before its main loop
  const uint8_t* pf_ptr[2];
  uint32_t pf_lines[2];
};

// Cache warming (EpiParams::pf_*): block b of nb issues one 4-B load per 64-B line of its share of
// each range, before its main loop; the returned sum goes to pf_sink after the epilogue, which
// stores it (to LDS) only under a condition the host never sets — keeping the loads alive.
template <int THREADS>
__device__ __forceinline__ uint32_t pf_issue(const EpiParams& e, uint32_t b, uint32_t nb) {
  uint32_t acc = 0;
  if (e.pf_lines[0] != 0) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const uint32_t per = (e.pf_lines[r] + nb - 1) / nb;
      const uint32_t l1 = min(e.pf_lines[r], (b + 1) * per);
      for (uint32_t l = b * per + threadIdx.x; l < l1; l += THREADS)
        acc += *reinterpret_cast<const uint32_t*>(e.pf_ptr[r] + ((size_t)l << 6));
    }
  }
  return acc;
}
__device__ __forceinline__ void pf_sink(const EpiParams& e, uint32_t acc, char* smem) {
  if (acc == 0x2545F491u && e.pf_lines[1] == 0xFFFFFFFFu)  // (lines are capped at 2^31 - 1)
    reinterpret_cast<uint32_t*>(smem)[threadIdx.x] = acc;
}

// One 64 x 64 (co x ci) transpose of one tap of one parity class's flipped sub-kernel, riding in
// a conv forward launch (the work of conv_dgrad.hip's conv_weight_flip_kernel).
template <class T, int THREADS>
__device__ void flip_block(const EpiParams& e, uint32_t b, char* smem) {
  T(*tile)[65] = reinterpret_cast<T(*)[65]>(smem);
  int c = 0;  // this block's parity class (block-uniform)
  while (c + 1 < e.fl.ncls && b >= e.fl.cls[c + 1].b0) ++c;
  const FlipClass& fc = e.fl.cls[c];
  b -= fc.b0;
  const int nci = (e.fl_Ci + 63) / 64, nco = (e.fl_Co + 63) / 64;
  const int bx = (int)(b % (uint32_t)nci), by = (int)((b / (uint32_t)nci) % (uint32_t)nco);
  const int tap = (int)(b / (uint32_t)(nci * nco));
  const int a = tap / fc.nkw, bb = tap - a * fc.nkw;
  const int kh = fc.kh0 + e.fl.S * (fc.nkh - 1 - a), kw = fc.kw0 + e.fl.S * (fc.nkw - 1 - bb);
  const T* w = reinterpret_cast<const T*>(e.fl_w);
  T* wt = reinterpret_cast<T*>(e.fl_wt) + fc.off;
  constexpr int NY = THREADS / 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int ci0 = bx * 64, co0 = by * 64;
#pragma unroll
  for (int r = ty; r < 64; r += NY) {
    const int co = co0 + r, ci = ci0 + tx;
    tile[r][tx] = (co < e.fl_Co && ci < e.fl_Ci)
                      ? w[(((long)co * e.fl_KH + kh) * e.fl_KW + kw) * e.fl_Ci + ci]
                      : T(0.f);
  }
  __syncthreads();
  const long taps = (long)fc.nkh * fc.nkw;
#pragma unroll
  for (int r = ty; r < 64; r += NY) {
    const int ci = ci0 + r, co = co0 + tx;
    if (co < e.fl_Co && ci < e.fl_Ci) wt[((long)ci * taps + tap) * e.fl_Co + co] = tile[tx][r];
  }
}

// The last split of a workspace split-K tile sums the tile's slices (slice order) into the final
// output.  Release: each split fences its slice stores (agent scope) before taking its ticket;
// acquire: the last one fences again before reading the other splits' slices.
template <int BM, int BN, int kThreads>
__device__ void ws_finish(char* smem, const EpiParams& e, uint32_t m0, uint32_t n0) {
  // release only (L2 write-back, no invalidate): a full __threadfence() also invalidates the
  // XCD's L2 in every block
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem);
  if (threadIdx.x == 0) {
    const int old = atomicAdd(e.fin.ticket + blockIdx.x, 1);
    *flag = old == (int)gridDim.y - 1 ? 1 : 0;
  }
  __syncthreads();
  if (*flag == 0) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the last split only
  const int S = (int)gridDim.y;
  const float* ws = reinterpret_cast<const float*>(e.C);
  const long slice = (long)e.M * e.ldc;
  constexpr int CPR = BN / 4;  // float4 chunks per tile row
  for (int c = threadIdx.x; c < BM * CPR; c += kThreads) {
    const uint32_t m = m0 + c / CPR, n = n0 + (c % CPR) * 4;
    if (m >= e.M || n >= e.N) continue;
    const float* p = ws + (long)m * e.ldc + n;
    float4 a = *reinterpret_cast<const float4*>(p);
    for (int s = 1; s < S; ++s) {
      const float4 b = *reinterpret_cast<const float4*>(p + s * slice);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    if (e.fin.bf16 == 0) {
      float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(e.fin.out) + (long)m * e.fin.ldo + n);
      float4 v = *o;
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
      *o = v;
    } else {
      float f[4] = {a.x, a.y, a.z, a.w};
      if (e.fin.bias != nullptr) {
        const float4 b = *reinterpret_cast<const float4*>(e.fin.bias + n);
        f[0] += b.x; f[1] += b.y; f[2] += b.z; f[3] += b.w;
      }
      if (e.fin.addend != nullptr) {
        const uint2 ad = *reinterpret_cast<const uint2*>(
            reinterpret_cast<const __bf16*>(e.fin.addend) + (long)m * e.N + n);
        f[0] += __uint_as_float(ad.x << 16); f[1] += __uint_as_float(ad.x & 0xffff0000u);
        f[2] += __uint_as_float(ad.y << 16); f[3] += __uint_as_float(ad.y & 0xffff0000u);
      }
      *reinterpret_cast<uint2*>(reinterpret_cast<__bf16*>(e.fin.out) + (long)m * e.fin.ldo + n) =
          make_uint2(pack2(f[0], f[1]), pack2(f[2], f[3]));
    }
  }
  if (threadIdx.x == 0) atomicExch(e.fin.ticket + blockIdx.x, 0);  // ready for the next launch
}

// BnCollect riding in a kernel: the block sums the replica rows of a bwd slab that the previous
// kernel filled, re-zeroes them and writes Σg / Σg·x̂ (+ dβ, dγ).  Each thread issues all of a
// channel's replica loads before any add (one memory latency per channel group).
template <int THREADS>
__device__ void bn_collect_block(const BnCollect c) {
  constexpr int R = kStatReplicas;
  const long rs = (long)R * c.C;
  for (int ch = threadIdx.x; ch < c.C; ch += THREADS) {
    float va[R], vb[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      va[r] = c.rep[(long)r * c.C + ch];
      vb[r] = c.rep[rs + (long)r * c.C + ch];
    }
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) {  // fixed order: deterministic
      a += va[r];
      b += vb[r];
      c.rep[(long)r * c.C + ch] = 0.f;
      c.rep[rs + (long)r * c.C + ch] = 0.f;
    }
    c.out[ch] = a;
    c.out[c.C + ch] = b;
    if (c.dgamma != nullptr) {
      c.dgamma[ch] += b;
      c.dbeta[ch] += a;
    }
    if (c.two) {  // Σg·x̂₂ of the second branch (dβ₂ = Σg as well)
      float d = 0.f;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        d += c.rep[2 * rs + (long)r * c.C + ch];
        c.rep[2 * rs + (long)r * c.C + ch] = 0.f;
      }
      c.out[2 * c.C + ch] = d;
      if (c.dgamma2 != nullptr) {
        c.dgamma2[ch] += d;
        c.dbeta2[ch] += a;
      }
    }
  }
}

// Workgroup barrier that orders LDS only.  __syncthreads() also drains every outstanding global
// load / store / atomic (s_waitcnt vmcnt(0)), which here would expose the latency of the
// epilogue's prefetched operands and of the statistics atomics at every barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Tile-local row / column of accumulator tile (i, j) of wave (wr, wc) (before the lane offset
// (lane & 15) / (lane >> 4) * 4): contiguous wave tiles, or the ping-pong loop's half-tile map
// (gemm_pp.hpp MainLoopPP::row / col).
template <int BM, int BN, int WM, int WN, bool HALVES>
struct AccMap {
  static constexpr int MT = BM / WM / 16, NT = BN / WN / 16;
  __device__ static uint32_t row(int wr, int i) {
    if constexpr (HALVES)
      return (uint32_t)((i / (MT / 2)) * (BM / 2) + wr * (MT / 2) * 16 + (i % (MT / 2)) * 16);
    else
      return (uint32_t)(wr * (BM / WM) + i * 16);
  }
  __device__ static uint32_t col(int wc, int j) {
    if constexpr (HALVES)
      return (uint32_t)((j / (NT / 2)) * (BN / 2) + wc * (NT / 2) * 16 + (j % (NT / 2)) * 16);
    else
      return (uint32_t)(wc * (BN / WN) + j * 16);
  }
};

// Rows of the fp32 output tile staged in LDS at once: all of them, or one m-half at a time for
// the ping-pong 256-row tiles (a 256 x 256 fp32 tile would need 260 KB).
template <int BM, int BN, bool HALVES>
constexpr int kEpiF32Rows() {
  return (HALVES && BM * (BN * 4 + 16) > 160 * 1024) ? BM / 2 : BM;
}

__device__ __forceinline__ long out_row(const EpiParams& e, uint32_t m) {
  if (e.rm_s == 0) return (long)m;
  uint32_t img = fdiv(e.rm_fHcWc, m);
  uint32_t rem = m - img * (uint32_t)(e.rm_Hc * e.rm_Wc);
  uint32_t i = fdiv(e.rm_fWc, rem);
  uint32_t j = rem - i * (uint32_t)e.rm_Wc;
  return ((long)img * e.rm_H + e.rm_ph + e.rm_s * (long)i) * e.rm_W + e.rm_pw + e.rm_s * (long)j;
}

// LDS pitch of the staged output tile (T elements + 16 B pad) and where the statistics
// partials live behind it.
template <int BN, class T = __bf16>
constexpr int kEpiPitch() { return BN * (int)sizeof(T) + 16; }
template <int BM, int BN, class T = __bf16>
constexpr int kStatsLdsOffset() { return ((BM * kEpiPitch<BN, T>()) + 255) / 256 * 256; }
template <int BM, int BN, class T = __bf16, int WM = 2>
constexpr int kEpiLdsBytes() { return kStatsLdsOffset<BM, BN, T>() + 2 * WM * BN * 4; }

// The fused epilogue's operand ring: each thread's addend / y / z chunks (PF iterations ahead).
// (Priming it before a short main loop was measured slower in round 2: the seven ResNet-50
// layer-1 1x1 data-grads went from ~1.9 ms to 3.4 ms per step — the early loads stretch the main
// loop's vmcnt waits and the registers' lifetime.)
// The loads are UNCONDITIONAL: an absent stream reads a 16-B zero line (g_epi_zero, L1/L2
// resident) instead of sitting behind `if (ptr != nullptr)`.  A load behind a runtime branch
// made hipcc close every ring slot with `s_waitcnt vmcnt(0)` right after issuing it (round 3,
// .s of the two-branch data-grad: 126 full drains), serialising the prefetch ring into one
// memory latency per 16-B chunk.
__device__ __attribute__((aligned(64))) uint4 g_epi_zero[4];

template <int BM, int BN, bool FUSE, class T, int WM, int WN, bool TWO = false>
struct EpiOps {
  static constexpr int kThreads = 64 * WM * WN;
  static constexpr int CPR = BN / 8;  // 8-element chunks per row
  static constexpr int ITER = BM * CPR / kThreads;
  static constexpr int PF = FUSE ? (ITER < 4 ? ITER : 4) : 1;
  Raw8<T> ad[PF], y[PF], z[PF], y2[TWO ? PF : 1];
  uint32_t mk[PF];
  // stream bases (the zero line when absent) and presence flags: wave-uniform
  const T *p_ad, *p_y, *p_z, *p_y2;
  const uint8_t* p_mk;
  bool h_ad, h_y, h_z, h_y2, h_mk;
  __device__ __forceinline__ void setup(const EpiParams& e) {
    const T* zt = reinterpret_cast<const T*>(g_epi_zero);
    const bool bnr = e.bnr_rep != nullptr;
    h_ad = e.addend != nullptr;
    h_y = bnr;
    h_z = bnr && e.bnr_mask == nullptr && e.bnr_z != nullptr;
    h_y2 = TWO && bnr && e.bnr_y2 != nullptr;
    h_mk = bnr && e.bnr_mask != nullptr;
    p_ad = h_ad ? reinterpret_cast<const T*>(e.addend) : zt;
    p_y = h_y ? reinterpret_cast<const T*>(e.bnr_y) : zt;
    p_z = h_z ? reinterpret_cast<const T*>(e.bnr_z) : zt;
    p_y2 = h_y2 ? reinterpret_cast<const T*>(e.bnr_y2) : zt;
    p_mk = h_mk ? e.bnr_mask : reinterpret_cast<const uint8_t*>(g_epi_zero);
  }
  __device__ __forceinline__ void issue(const EpiParams& e, uint32_t m0, uint32_t n0, int it,
                                        int slot) {
    const uint32_t my_n = n0 + (threadIdx.x % CPR) * 8;
    const uint32_t ld_n = my_n < e.N ? my_n : 0;
    const uint32_t r = (threadIdx.x + it * kThreads) / CPR;
    const uint32_t m = min(m0 + r, e.M - 1);
    const long orow = out_row(e, m);
    const long off = orow * e.ldc + ld_n;  // one element offset shared by every present stream
    const bool ntl = e.ntl != 0;  // streaming operand loads (g_nt_store & 256)
    ad[slot] = ld_raw8(p_ad + (h_ad ? off : 0), ntl);
    y[slot] = ld_raw8(p_y + (h_y ? off : 0), ntl);
    z[slot] = ld_raw8(p_z + (h_z ? off : 0), ntl);
    if constexpr (TWO) y2[slot] = ld_raw8(p_y2 + (h_y2 ? off : 0), ntl);
    mk[slot] = p_mk[h_mk ? off / 8 : 0];  // ldc % 8 == 0: the mask byte of columns ld_n..+7
  }
  __device__ __forceinline__ void prime(const EpiParams& e, uint32_t m0, uint32_t n0) {
    setup(e);
    if (FUSE && (e.addend != nullptr || e.bnr_rep != nullptr)) {
#pragma unroll
      for (int it = 0; it < PF; ++it) issue(e, m0, n0, it, it);
    }
  }
};

// BatchNorm partial statistics by MFMA from the STAGED bf16 output tile (the stored values, as
// the VALU path's as_stored): per 16-column group, Σy = 1ᵀY and Σy² = diag(YᵀY) over the tile's
// rows (bf16 x bf16 products are exact in the fp32 accumulator), from transposed LDS reads (the MC fragment map of FragLoader<false>); then the shifted
// moments Σ(y-s) = Σy - n·s and Σ(y-s)² = Σy² - 2s·Σy + n·s² per column, in double (n = rows
// of the tile inside M; rows past M are masked out of the fragments).  Replaces
// ~4 VALU per output element plus 16 DPP row sums per lane (the VALU path cost the wide
// ResNet-50 1x1 forwards up to 50 %: profiles/r5_epilogue_cost.jsonl).
#ifndef MIPIPE_VALU_STATS
constexpr bool kMfmaStats = true;
#else
constexpr bool kMfmaStats = false;
#endif
template <int BM, int BN, int NWV>
__device__ __forceinline__ void stats_mfma(const char* smem, const EpiParams& e, uint32_t m0,
                                           uint32_t n0, int wave, int lane) {
  constexpr int P = kEpiPitch<BN, __bf16>();
  constexpr int NCG = BN / 16, NKC = BM / 32;
  static_assert(BN % 16 == 0 && BM % 32 == 0, "MFMA statistics tile");
  const uint32_t g = (uint32_t)lane >> 4, q4 = ((uint32_t)lane & 15) >> 2, p = (uint32_t)lane & 3;
  bf16x8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (__bf16)1.0f;
  const uint32_t nv = e.M - m0 < (uint32_t)BM ? e.M - m0 : (uint32_t)BM;
  for (int cg = wave; cg < NCG; cg += NWV) {  // wave-uniform
    f32x4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};
    const uint32_t ch = (uint32_t)cg * 2 + (p >> 1);  // 8-column chunk of this lane's reads
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) {
      const char* a0 = smem + (kc * 32 + 8 * g + q4) * P + ch * 16 + 8 * (p & 1);
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a0);
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0 + 4 * P));
      typedef __attribute__((ext_vector_type(8))) short s16x8;
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      bf16x8 y = __builtin_bit_cast(bf16x8, v);
      if (nv < (uint32_t)BM) {  // partial tile (wave-uniform): rows past M add nothing, whatever
        // was staged there (a bias, say); this lane's 8 values are rows kc*32 + 8g + 0..7
#pragma unroll
        for (int r = 0; r < 8; ++r)
          if ((uint32_t)(kc * 32) + 8 * g + (uint32_t)r >= nv) y[r] = (__bf16)0.0f;
      }
      s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, y, s1, 0, 0, 0);  // rows: Σ_k Y[k][j]
      s2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(y, y, s2, 0, 0, 0);     // Σ_k Y[k][i] Y[k][j]
    }
    // lane holds D[i = 4(lane>>4) + q][j = lane & 15]: column j's diagonal sits at q = j & 3 of
    // the lane with lane >> 4 == j >> 2 (which also holds its column sum)
    const uint32_t j = (uint32_t)lane & 15;
    if (g == (j >> 2)) {
      const uint32_t n = n0 + (uint32_t)cg * 16 + j;
      if (n < e.N) {
        const int q = (int)(j & 3);
        const double sy = (double)s1[q], syy = (double)s2[q], sh = (double)e.st_shift[n];
        const double nd = (double)nv;
        const float a = (float)(sy - nd * sh);
        const float b = (float)(syy - 2.0 * sh * sy + nd * sh * sh);
        if (e.det_rows > 0) {
          const long row = (long)(e.det_row0 + m0 / BM) * e.N + n;
          e.st_sum[row] = a;
          e.st_sq[row] = b;
        } else {
          const long row = (long)(blockIdx.x % e.st_R) * e.N + n;
          atomicAdd(e.st_sum + row, a);
          atomicAdd(e.st_sq + row, b);
        }
      }
    }
  }
}

// Output in the activation dtype T (bf16, or fp32 on the reference-precision path).
// acc layout: lane holds C[m][n..n+3] for tile (i, j).
// FUSE: compile the dgrad fusions (addend / BN-backward reduction); kernels that never use
// them keep their register budget.  early: an operand ring the kernel already primed.
// TWO: the BN-backward fusion of a two-branch block output (e.bnr_y2 set, FUSE only).
template <int BM, int BN, bool FUSE = false, class T = __bf16, int WM = 2, int WN = 2,
          bool TWO = false, bool HALVES = false>
__device__ void epilogue_out(char* smem, f32x4 (&acc)[BM / WM / 16][BN / WN / 16],
                             const EpiParams& e, uint32_t m0, uint32_t n0, uint32_t prow_base,
                             int wave, int lane,
                             EpiOps<BM, BN, FUSE, T, WM, WN, TWO>* early = nullptr) {
  constexpr int MT = BM / WM / 16, NT = BN / WN / 16;
  constexpr int kThreads = 64 * WM * WN;
  // BN-backward Σg·x̂ as invstd·(Σg·y - mean·Σg): exact products for bf16 g, y only; the fp32
  // path (and -DMIPIPE_BNR_CENTERED) accumulates the centred g·(y - mean)·invstd instead
#ifdef MIPIPE_BNR_CENTERED
  constexpr bool kBnrUncentered = false;
#else
  constexpr bool kBnrUncentered = !std::is_same<T, float>::value;
#endif
  const int wr = wave / WN, wc = wave % WN;
  typedef AccMap<BM, BN, WM, WN, HALVES> Map;
  const uint32_t lr = lane & 15, lc = (lane >> 4) * 4;
  // dgrad fusions: issue this thread's addend / y loads now so their latency overlaps the
  // accumulator staging below (a thread always owns the same 8-column chunk)
  constexpr int CPR = BN / 8;  // 8-element chunks per row
  constexpr int ITER = BM * CPR / kThreads;
  static_assert(kThreads % CPR == 0 && (BM * CPR) % kThreads == 0, "epilogue thread map");
  const bool bnr = FUSE && e.bnr_rep != nullptr;
  const bool has_add = FUSE && e.addend != nullptr;
  const bool zmask = bnr && e.bnr_z != nullptr && e.bnr_mask == nullptr;
  const bool bmask = bnr && e.bnr_mask != nullptr;
  const uint32_t my_cc = threadIdx.x % CPR, my_n = n0 + my_cc * 8;
  const uint32_t ld_n = my_n < e.N ? my_n : 0;
  // software-pipelined operand ring: PF iterations in flight; the first PF are issued now (unless
  // the kernel primed them before its main loop) so their latency overlaps the staging below
  typedef EpiOps<BM, BN, FUSE, T, WM, WN, TWO> Ops;
  constexpr int PF = Ops::PF;
  Ops local;
  Ops& ops = early != nullptr ? *early : local;
  // the ring is primed after the accumulators went to LDS (below): priming it here kept the
  // 64 accumulator registers and the ring live together — 168 VGPRs and ~100 spilled to scratch
  // in the fused 128x128 data-grads (round 3 .s) — for an overlap of one short LDS staging
  (void)ld_n;
  // BN-backward coefficients of this thread's 8 columns, requested now (16-B vector loads; the
  // host checks N % 8 == 0 and 16-B alignment) so their latency hides under the staging below:
  // issued as 32 scalar loads at the store loop they cost the layer-1 fused data-grads ~35 %
  // (tools/r2/knob_probe.py).  scale / bias only when the ReLU mask is recomputed from y.
  float b_sc[8], b_bi[8], b_mu[8], b_is[8];
  if (bnr) {
    const bool okc = my_n < e.N;
    const uint32_t cn = okc ? my_n : 0;
    if (!bmask && !zmask) {
      ld_f32x8(e.bnr_scale + cn, b_sc);
      ld_f32x8(e.bnr_bias + cn, b_bi);
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) b_sc[q] = b_bi[q] = 0.f;
    }
    ld_f32x8(e.bnr_mean + cn, b_mu);
    ld_f32x8(e.bnr_invstd + cn, b_is);
  }
  float b_mu2[TWO ? 8 : 1], b_is2[TWO ? 8 : 1], sgx2[TWO ? 8 : 1];
  if constexpr (TWO) {
    const uint32_t cn = my_n < e.N ? my_n : 0;
    ld_f32x8(e.bnr_mean2 + cn, b_mu2);
    ld_f32x8(e.bnr_invstd2 + cn, b_is2);
#pragma unroll
    for (int q = 0; q < 8; ++q) sgx2[q] = 0.f;
  }
  // bias / activation
  if (e.bias != nullptr || e.act) {
    // every bias quad loaded before use, at a clamped column (N % 4 == 0: a quad is all in or
    // all out; the zero line when there is no bias): loads behind per-element branches cost a
    // vmcnt(0) drain each (see EpiOps)
    float bv[NT][4];
    const float* bp = e.bias != nullptr ? e.bias : reinterpret_cast<const float*>(g_epi_zero);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const uint32_t n = n0 + Map::col(wc, j) + lc;
      const uint32_t nc = (e.bias != nullptr && n < e.N) ? n : 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[j][q] = bp[nc + q];
    }
    // the activation is a wave-uniform branch (not a per-element select of both results)
    auto add_bias = [&](auto relu_tag) {
      constexpr bool RELU = decltype(relu_tag)::value;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        uint32_t n = n0 + Map::col(wc, j) + lc;
        float b[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) b[q] = n < e.N ? bv[j][q] : 0.f;
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float v = acc[i][j][q] + b[q];
            acc[i][j][q] = RELU ? fmaxf(v, 0.f) : v;
          }
      }
    };
    if (e.act == 1) add_bias(std::true_type());
    else add_bias(std::false_type());
  }
  // BatchNorm partial statistics from the fp32 accumulators, reduced over the block's BM rows
  // and added with fp32 atomics into replica slab (blockIdx % st_R) — 256-B-contiguous
  // wave-instructions, no per-block partial rows to reduce later.  (bf16 outputs: stats_mfma
  // after the staging below instead.)
  constexpr bool MSTATS = kMfmaStats && std::is_same<T, __bf16>::value;
  if (!MSTATS && e.st_sum != nullptr) {
    float* lst = reinterpret_cast<float*>(smem + kStatsLdsOffset<BM, BN, T>());  // [2][WM][BN]
    // every column's shift requested before any is used (clamped column: unconditional loads),
    // so the block waits one memory latency here, not one per 16-column group
    float shv[NT][4];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const uint32_t n = n0 + Map::col(wc, j) + lc;
      const uint32_t nc = n < e.N ? n : 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) shv[j][q] = e.st_shift[nc + q];
    }
    // column pairs in packed fp32 (v_pk_add_f32 / v_pk_fma_f32: two columns per instruction)
    typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const float* sh = shv[j];
      const f2 sh01 = {sh[0], sh[1]}, sh23 = {sh[2], sh[3]};
      f2 s01 = {0.f, 0.f}, s23 = {0.f, 0.f}, ss01 = {0.f, 0.f}, ss23 = {0.f, 0.f};
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        uint32_t m = m0 + Map::row(wr, i) + lr;
        const f2 w = m < e.M ? f2{1.f, 1.f} : f2{0.f, 0.f};  // rows past M add nothing
        const f2 d01 = (f2{as_stored<T>(acc[i][j][0]), as_stored<T>(acc[i][j][1])} - sh01) * w;
        const f2 d23 = (f2{as_stored<T>(acc[i][j][2]), as_stored<T>(acc[i][j][3])} - sh23) * w;
        s01 += d01;
        s23 += d23;
        ss01 += d01 * d01;
        ss23 += d23 * d23;
      }
      float s[4] = {s01.x, s01.y, s23.x, s23.y}, ss[4] = {ss01.x, ss01.y, ss23.x, ss23.y};
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // over the 16 lanes (rows) of each DPP row: VALU only
        s[q] = row16_sum(s[q]);
        ss[q] = row16_sum(ss[q]);
      }
      if ((lane & 15) == 0) {
        uint32_t nl = Map::col(wc, j) + lc;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          lst[(0 * WM + wr) * BN + nl + q] = s[q];
          lst[(1 * WM + wr) * BN + nl + q] = ss[q];
        }
      }
    }
  }
  // every wave is past the main loop (whose LDS the staging tile overwrites) and the
  // statistics partials are in LDS
  lds_barrier();
  // stage the output tile in LDS: pitch BN*sizeof(T) + 16 bytes
  constexpr int P = kEpiPitch<BN, T>();
  constexpr bool F32 = std::is_same<T, float>::value;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      uint32_t ml = Map::row(wr, i) + lr, nl = Map::col(wc, j) + lc;
      if constexpr (F32) {
        *reinterpret_cast<float4*>(smem + ml * P + nl * 4) =
            make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      } else {
        uint2 v = make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
        *reinterpret_cast<uint2*>(smem + ml * P + nl * 2) = v;
      }
    }
  if (early == nullptr) ops.prime(e, m0, n0);  // accumulators are dead now
  lds_barrier();
  if (MSTATS && e.st_sum != nullptr) {
    stats_mfma<BM, BN, kThreads / 64>(smem, e, m0, n0, wave, lane);
  } else if (e.st_sum != nullptr) {
    // one fp32 atomic per column per block into replica row blockIdx % st_R (fire and forget:
    // no barrier below waits for them)
    const float* lst = reinterpret_cast<const float*>(smem + kStatsLdsOffset<BM, BN, T>());
    for (int t = threadIdx.x; t < 2 * BN; t += kThreads) {
      int arr = t / BN, c = t % BN;
      uint32_t n = n0 + c;
      if (n < e.N) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) v += lst[(arr * WM + w) * BN + c];
        float* base = arr == 0 ? e.st_sum : e.st_sq;
        if (e.det_rows > 0) {
          base[(long)(e.det_row0 + m0 / BM) * e.N + n] = v;
        } else {
          atomicAdd(base + (long)(blockIdx.x % e.st_R) * e.N + n, v);
        }
      }
    }
  }
  T* C = reinterpret_cast<T*>(e.C);
  float sg[8], sgx[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) sg[q] = sgx[q] = 0.f;
  if (FUSE && (has_add || bnr)) {
    // fused loop: the ring's next loads are issued unconditionally (absent streams read the
    // zero line), so hipcc keeps PF iterations of loads in flight with counted waits
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int c = threadIdx.x + it * kThreads;
      const uint32_t r = c / CPR, cc = c % CPR;
      const uint32_t m = m0 + r, n = n0 + cc * 8;
      Raw8<T> v;
#pragma unroll
      for (int h = 0; h < (int)(sizeof(T) / 2); ++h)
        v.v[h] = *reinterpret_cast<const uint4*>(smem + r * P + cc * 8 * sizeof(T) + 16 * h);
      float f[8], a[8];
      unpack_raw(v, f);
      unpack_raw(ops.ad[it % PF], a);  // zeros when there is no addend
#pragma unroll
      for (int q = 0; q < 8; ++q) f[q] += a[q];
      const bool ok = m < e.M && n < e.N;
      if (bnr) {
        float yv[8], zv[8];
        unpack_raw(ops.y[it % PF], yv);
        unpack_raw(ops.z[it % PF], zv);
        const uint32_t bits = ops.mk[it % PF];
        const float w = ok ? 1.f : 0.f;  // rows past M add nothing to the sums
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float zq = bmask ? (float)((bits >> q) & 1u)
                                 : (zmask ? zv[q] : yv[q] * b_sc[q] + b_bi[q]);
          const float gq = zq > 0.f ? as_stored<T>(f[q]) : 0.f;  // stats of the stored g
          f[q] = gq;
          if constexpr (kBnrUncentered) {
            // Σg and Σg·y here (2 VALU); Σg·x̂ = invstd·(Σg·y - mean·Σg) once per thread below.
            // bf16 g and y: each product is exact in fp32
            const float gw = w * gq;
            sg[q] += gw;
            sgx[q] = fmaf(gw, yv[q], sgx[q]);
          } else {  // fp32 (the reference's precision): centred, no cancellation at |mean| >> std
            sg[q] += w * gq;
            sgx[q] += w * gq * (yv[q] - b_mu[q]) * b_is[q];
          }
        }
        if constexpr (TWO) {
          float y2v[8];
          unpack_raw(ops.y2[it % PF], y2v);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            if constexpr (kBnrUncentered)
              sgx2[q] = fmaf(w * f[q], y2v[q], sgx2[q]);
            else
              sgx2[q] += w * f[q] * (y2v[q] - b_mu2[q]) * b_is2[q];
          }
        }
      }
      if (ok) store8(C + out_row(e, m) * e.ldc + n, f, e.nt != 0);
      if (it + PF < ITER) ops.issue(e, m0, n0, it + PF, it % PF);
    }
  } else {
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int c = threadIdx.x + it * kThreads;
      const uint32_t r = c / CPR, cc = c % CPR;
      const uint32_t m = m0 + r, n = n0 + cc * 8;
      if (m < e.M && n < e.N) {
        const long orow = out_row(e, m);
#pragma unroll
        for (int h = 0; h < (int)(sizeof(T) / 2); ++h) {
          uint4 v = *reinterpret_cast<const uint4*>(smem + r * P + cc * 8 * sizeof(T) + 16 * h);
          uint4* dst = reinterpret_cast<uint4*>(C + orow * e.ldc + n) + h;
          if constexpr (!std::is_same<T, float>::value) {
            if (e.aux != nullptr) {  // GELU Linear: h to aux, gelu(h) (bf16-rounded h, as the
              // gelu_fwd kernel computes it) to C
              reinterpret_cast<uint4*>(reinterpret_cast<T*>(e.aux) + orow * e.ldc + n)[h] = v;
              float f[8];
              unpack8(v, f);
#pragma unroll
              for (int q = 0; q < 8; ++q) f[q] = gelu_erf(f[q]);
              v = pack8(f);
            }
          }
          if (e.nt) {  // streaming output (g_nt_store)
            __builtin_nontemporal_store(u32v4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32v4*>(dst));
          } else {
            *dst = v;
          }
        }
      }
    }
  }
  if (FUSE && bnr) {
    if constexpr (kBnrUncentered) {
      // this thread's columns: Σg·x̂ = invstd·(Σg·y - mean·Σg) (linear: the sums below add these)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        sgx[q] = b_is[q] * (sgx[q] - b_mu[q] * sg[q]);
        if constexpr (TWO) sgx2[q] = b_is2[q] * (sgx2[q] - b_mu2[q] * sg[q]);
      }
    }
    // threads t, t+CPR, ... share a column chunk: reduce them through LDS, then one atomic
    // per column per block into replica row blockIdx % R
    lds_barrier();  // all staging-tile reads done (red overlaps it)
    // [16][RP] floats, value-major: the stores (consecutive threads) and the column sums
    // (8 columns x 8 chunks per wave: bank 8q + cc) are both bank-conflict-free
    constexpr int RP = kThreads + 8;
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      red[q * RP + threadIdx.x] = sg[q];
      red[(8 + q) * RP + threadIdx.x] = sgx[q];
    }
    lds_barrier();
    const uint32_t R = kStatReplicas, Rw = (uint32_t)e.st_R;  // layout rows / rows written
    for (int j = threadIdx.x; j < 2 * BN; j += kThreads) {
      const int arr = j / BN, col = j % BN, cc = col >> 3, q = col & 7;
      float a = 0.f;
      for (int t = cc; t < kThreads; t += CPR) a += red[(arr * 8 + q) * RP + t];
      if (n0 + col < e.N) {
        if (e.det_rows > 0)
          e.bnr_rep[((long)arr * e.det_rows + e.det_row0 + m0 / BM) * e.N + n0 + col] = a;
        else
          atomicAdd(e.bnr_rep + ((long)arr * R + blockIdx.x % Rw) * e.N + n0 + col, a);
      }
    }
    if constexpr (TWO) {  // Σg·x̂₂: third array, through the same LDS rows
      lds_barrier();
#pragma unroll
      for (int q = 0; q < 8; ++q) red[q * RP + threadIdx.x] = sgx2[q];
      lds_barrier();
      for (int col = threadIdx.x; col < BN; col += kThreads) {
        const int cc = col >> 3, q = col & 7;
        float a = 0.f;
        for (int t = cc; t < kThreads; t += CPR) a += red[q * RP + t];
        if (n0 + col < e.N) {
          if (e.det_rows > 0)
            e.bnr_rep[((long)2 * e.det_rows + e.det_row0 + m0 / BM) * e.N + n0 + col] = a;
          else
            atomicAdd(e.bnr_rep + ((long)2 * R + blockIdx.x % Rw) * e.N + n0 + col, a);
        }
      }
    }
  }
}

template <int BM, int BN, bool FUSE = false>
__device__ void epilogue_bf16(char* smem, f32x4 (&acc)[BM / 32][BN / 32], const EpiParams& e,
                              uint32_t m0, uint32_t n0, uint32_t prow_base, int wave, int lane) {
  epilogue_out<BM, BN, FUSE, __bf16, 2, 2>(smem, acc, e, m0, n0, prow_base, wave, lane);
}

// fp32 output; ATOMIC accumulates into C (split-K), otherwise plain store (beta = 0) or, with
// e.rmw, a non-atomic accumulate (beta = 1, one block per element).  The tile is staged through
// LDS in passes of kEpiF32Rows rows (two m-halves for the ping-pong 256 x 256 tile).
template <int BM, int BN, bool ATOMIC, int WM = 2, int WN = 2, bool HALVES = false>
__device__ void epilogue_f32(char* smem, f32x4 (&acc)[BM / WM / 16][BN / WN / 16],
                             const EpiParams& e, uint32_t m0, uint32_t n0, int wave, int lane) {
  constexpr int MT = BM / WM / 16, NT = BN / WN / 16;
  constexpr int kThreads = 64 * WM * WN;
  constexpr int RP = kEpiF32Rows<BM, BN, HALVES>();  // rows per pass
  constexpr int PASSES = BM / RP;
  static_assert(PASSES == 1 || HALVES, "multi-pass fp32 staging needs the half-tile map");
  const int wr = wave / WN, wc = wave % WN;
  typedef AccMap<BM, BN, WM, WN, HALVES> Map;
  const uint32_t lr = lane & 15, lc = (lane >> 4) * 4;
  // stage fp32 tile: pitch BN*4 + 16 bytes (RP*(BN*4+16) <= LDS of the kernel)
  constexpr int P = BN * 4 + 16;
  float* C = reinterpret_cast<float*>(e.C);
  if (ATOMIC && e.det_rows > 0) C += (long)blockIdx.y * e.M * e.ldc;
#pragma unroll
  for (int pass = 0; pass < PASSES; ++pass) {
    if (pass > 0) __syncthreads();  // the previous pass's staging reads are done
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if (PASSES > 1 && i / (MT / 2) != pass) continue;  // compile-time after unrolling
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        uint32_t ml = Map::row(wr, i) + lr - pass * RP, nl = Map::col(wc, j) + lc;
        *reinterpret_cast<float4*>(smem + ml * P + nl * 4) =
            make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    __syncthreads();
    const uint32_t pm0 = m0 + pass * RP;  // first output row of this pass
    if (ATOMIC && e.det_rows > 0) {
      // deterministic split-K: this split's partial tile goes to its own workspace slice
      for (int c = threadIdx.x; c < RP * BN; c += kThreads) {
        uint32_t r = c / BN, cc = c % BN;
        uint32_t m = pm0 + r, n = n0 + cc;
        if (m < e.M && n < e.N) C[(long)m * e.ldc + n] = *reinterpret_cast<const float*>(smem + r * P + cc * 4);
      }
    } else if constexpr (ATOMIC) {
      // each wave-instruction: 64 lanes x 4 B = 256 contiguous bytes of one row
      for (int c = threadIdx.x; c < RP * BN; c += kThreads) {
        uint32_t r = c / BN, cc = c % BN;
        uint32_t m = pm0 + r, n = n0 + cc;
        if (m < e.M && n < e.N) {
          float v = *reinterpret_cast<const float*>(smem + r * P + cc * 4);
          atomicAdd(C + (long)m * e.ldc + n, v);
        }
      }
    } else {
      // the C quads of a group of iterations (read-modify-write) are requested before any is
      // used, unconditionally at clamped addresses: a load behind `if (e.rmw)` / a bounds branch
      // was closed by a vmcnt(0) each — one memory latency per 16-B chunk, ITER per block
      constexpr int CPR = BN / 4;
      constexpr int ITER = (RP * CPR + kThreads - 1) / kThreads;
      constexpr int G = ITER < 8 ? ITER : 8;  // 8 quads in flight: 32 VGPRs
      static_assert(ITER % G == 0, "epilogue_f32 groups");
      const bool rmw = e.rmw != 0, has_b = e.bias != nullptr;
      const float* bp = has_b ? e.bias : reinterpret_cast<const float*>(g_epi_zero);
#pragma unroll
      for (int g0 = 0; g0 < ITER; g0 += G) {
        float4 old[G];
#pragma unroll
        for (int k = 0; k < G; ++k) {
          const int c = threadIdx.x + (g0 + k) * kThreads;
          const uint32_t r = c / CPR, cc = c % CPR;
          const uint32_t m = min(pm0 + r, e.M - 1), n = n0 + cc * 4;
          const float* src = rmw ? C + (long)m * e.ldc + (n < e.N ? n : 0)
                                 : reinterpret_cast<const float*>(g_epi_zero);
          old[k] = *reinterpret_cast<const float4*>(src);
        }
#pragma unroll
        for (int k = 0; k < G; ++k) {
          const int c = threadIdx.x + (g0 + k) * kThreads;
          const uint32_t r = c / CPR, cc = c % CPR;
          const uint32_t m = pm0 + r, n = n0 + cc * 4;
          if (c < RP * CPR && m < e.M && n < e.N) {
            float4 v = *reinterpret_cast<const float4*>(smem + r * P + cc * 16);
            v.x += old[k].x; v.y += old[k].y; v.z += old[k].z; v.w += old[k].w;  // 0 unless rmw
            if (has_b) {
              const float4 b = *reinterpret_cast<const float4*>(bp + n);
              v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
            }
            *reinterpret_cast<float4*>(C + (long)m * e.ldc + n) = v;
          }
        }
      }
    }
  }
  if constexpr (ATOMIC) {
    if (e.det_rows > 0 && e.fin.ticket != nullptr) {
      __syncthreads();  // the staging reads of the last pass are done (ws_finish reuses smem)
      ws_finish<BM, BN, kThreads>(smem, e, m0, n0);
    }
  }
}

}  // namespace gk
// host: copy cache-warming ranges into a GEMM launch's params (gemm.hip)
void set_prefetch(gk::EpiParams& e, const TouchRanges* pf);
}  // namespace mipipe
