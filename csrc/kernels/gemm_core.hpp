// Implicit-GEMM core on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16), shared by convolution
// forward / data-grad / weight-grad and the Linear (GEMM) kernels.
//
//   C[m][n] = sum_k A(m,k) * B(k,n),  bf16 operands, fp32 accumulation.
//
// Structure (cdna_hip_programming.md §5 "minimum 2-phase" + T1/T2/T10):
//  * 256 threads = 4 waves (2x2), block tile BM x BN x 64, wave tile (BM/2) x (BN/2) made of
//    16x16 MFMA tiles; LDS double buffer, one barrier per K-step.
//  * Operands reach LDS with global_load_lds_dwordx4 (16 B per lane, 1 KiB per wave-instruction,
//    lane-linear LDS destination).  Each operand policy computes a per-lane *source* address, so
//    im2col / data-grad gathers are free, and padding taps point at a zero page.
//  * Two LDS image formats:
//      KC ("K-contiguous"): [rows][64 k] 128-B rows, 16-B chunk c stored at c ^ (row & 7);
//          fragments by ds_read_b128 (conflict-free for the 16x16x32 lane map).
//      MC ("M/N-contiguous"): [64 k][W cols] (W = 64 or 128) with an XOR chunk swizzle chosen so
//          ds_read_b64_tr_b16 (hardware transpose, guide T10) is conflict-free; used when the
//          operand is stored k-major in memory (weight-grad, Linear backward, dgrad weights).
//    The swizzle is applied on the SOURCE address (glds writes linearly; guide rule 21).
//  * MFMA runs in the swapped orientation D = B^T A^T so each lane ends with 4 consecutive
//    output columns of one row -> 8-byte LDS writes in the epilogue, then fully coalesced 16-B
//    global stores (or 256-B-contiguous fp32 atomics for split-K).
//  * Workgroup ids are remapped XCD-aware (guide T1) so blocks sharing A-rows share an L2.
#pragma once
#include "common.hpp"

namespace mipipe {
namespace gk {

constexpr int BK = 64;
constexpr int kThreads = 256;

// ---------------------------------------------------------------------------------------------
// LDS image addressing
__device__ __forceinline__ uint32_t kc_off(uint32_t row, uint32_t chunk) {
  return row * 128u + ((chunk ^ (row & 7u)) << 4);
}

template <int W>
__device__ __forceinline__ uint32_t mc_swz(uint32_t row) {
  if constexpr (W == 256) return ((row & 3u) << 1) | (((row >> 3) & 1u) << 3);
  else if constexpr (W == 128) return ((row & 3u) << 2) | ((row >> 2) & 3u);
  else return (((row >> 1) & 1u) << 1) | (((row >> 3) & 1u) << 2);
}

template <int W>
__device__ __forceinline__ uint32_t mc_off(uint32_t row, uint32_t chunk) {
  return row * (uint32_t)(W * 2) + ((chunk ^ mc_swz<W>(row)) << 4);
}

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

// Buffer LDS-DMA (bf16 operand policies with BUF = true): a 128-bit descriptor over the operand
// (wave-uniform: built from kernel arguments only), a per-lane 32-bit voffset that is FIXED for
// the whole k-loop, and a wave-uniform soffset (SGPR) that carries the k-step.  A lane that must
// read zeros (padding tap, row past M / column past N, k past K) gets voffset kOOB, which lies
// past every descriptor's range (the hardware range check returns zeros): no per-lane 64-bit
// pointer math and no zero-page selects in the main loop.  Host contract: descriptor bytes
// < 2^31 (bindings.cpp checks bf16 operand sizes).
constexpr uint32_t kOOB = 0x80000000u;
// The operands are uniform by construction; the readfirstlanes pin them to SGPRs, because a
// descriptor (or soffset) the backend finds in VGPRs turns every LDS-DMA piece into a waterfall
// loop (measured in the 256x256 dense data-grad before this).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gk_rsrc(const void* base, uint64_t bytes) {
  const uint32_t b = bytes < (uint64_t)kOOB ? (uint32_t)bytes : kOOB - 16u;
  const uint64_t p = (uint64_t)(uintptr_t)base;
  const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)p);
  const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(lo | (hi << 32)), 0,
                                           __builtin_amdgcn_readfirstlane((int)b), 0x00020000);
}

__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, char* lds_wave_base,
                                       uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds_wave_base, 16, voff, soff, 0, 0);
}

template <class Op, class = void>
struct IsBufOp : std::false_type {};
template <class Op>
struct IsBufOp<Op, std::void_t<decltype(Op::BUF)>> : std::integral_constant<bool, Op::BUF> {};

// Buffer policies whose voffsets need a k < K test on ONE k-step (kt_tail: the last step of a K
// that is not a multiple of 64) expose tail(kt); every other step takes the fixed voffsets vo[i].
template <class Op, class = void>
struct HasTail : std::false_type {};
template <class Op>
struct HasTail<Op, std::void_t<decltype(&Op::tail)>> : std::true_type {};
template <class Op>
__device__ __forceinline__ bool is_tail(const Op& op, int kt) {
  if constexpr (HasTail<Op>::value) return op.tail(kt);
  else return false;
}

// one 1-KiB LDS-DMA wave-instruction of piece i of operand `op` at k-step kt (prep(kt) done).
// CHECK = false: the caller knows kt is not op's tail step (no per-piece compare / select).
template <bool CHECK = true, class Op>
__device__ __forceinline__ void dma16(const Op& op, int kt, int i, char* lds_wave_base) {
  if constexpr (IsBufOp<Op>::value) {
    if constexpr (CHECK || !HasTail<Op>::value) blds16(op.rsrc, lds_wave_base, op.voff(kt, i), op.soff);
    else blds16(op.rsrc, lds_wave_base, op.vo[i], op.soff);
  } else {
    glds16(op.src(kt, i), lds_wave_base);
  }
}

// Marks the end of a tail-step DMA block.  The checked and unchecked blocks otherwise end in the
// same buffer loads, and the optimizer would sink them into one block with a select per voffset
// (the per-piece compare + cndmask this split exists to remove).
__device__ __forceinline__ void tail_block_end() { asm volatile("; k-tail stage" ::: "memory"); }

// ---------------------------------------------------------------------------------------------
// Operand policies.  Each describes one operand (A: rows = M, or B: rows = N) and exposes
//   static constexpr bool KC;               // image format
//   __device__ void init(const P&, uint32_t tile_origin, int wave, int lane);
//   __device__ const void* src(int kt, int i) const;   // i-th glds of this wave at k-step kt
// KC: NI = R/32 instructions per wave, row = (wave*NI+i)*8 + lane/8, chunk = (lane&7)^(lane>>3)
// MC: NI = W/32, RPI = 512/W rows per instruction, row = (wave*NI+i)*RPI + lane/(W/8)

template <int R, int NW = 4>
struct KCGeom {
  static constexpr int NI = R / (8 * NW);
  __device__ static uint32_t row(int wave, int i, int lane) { return (wave * NI + i) * 8 + (lane >> 3); }
  __device__ static uint32_t chunk(int lane) { return (lane & 7) ^ (lane >> 3); }
};

template <int W, int NW = 4>
struct MCGeom {
  static constexpr int NI = W / (8 * NW);
  static constexpr int RPI = 512 / W;
  static constexpr int LPR = W / 8;
  __device__ static uint32_t row(int wave, int i, int lane) { return (wave * NI + i) * RPI + lane / LPR; }
  __device__ static uint32_t chunk(int wave, int i, int lane) {
    return (uint32_t)(lane % LPR) ^ mc_swz<W>(row(wave, i, lane));
  }
};

// Dense K-contiguous rows: element (r, k) at base[r*ld + k].
template <int R, class T = __bf16, int NW = 4>
struct KCDense {
  static constexpr bool KC = true;
  static constexpr int NI = R / (8 * NW);
  const T* ptr[NI];
  uint32_t kcol;
  uint32_t K;
  const void* zero;
  __device__ void prep(int) {}
  __device__ void init(const T* base, long ld, uint32_t rows_total, uint32_t K_,
                       uint32_t origin, int wave, int lane, const void* zero_page) {
    K = K_;
    zero = zero_page;
    kcol = KCGeom<R, NW>::chunk(lane) * 8;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      uint32_t r = origin + KCGeom<R, NW>::row(wave, i, lane);
      ptr[i] = r < rows_total ? base + (long)r * ld + kcol : nullptr;
    }
  }
  __device__ const void* src(int kt, int i) const {
    uint32_t k = (uint32_t)kt * BK + kcol;
    return (ptr[i] != nullptr && k < K) ? (const void*)(ptr[i] + (long)kt * BK) : zero;
  }
};

// Dense K-contiguous rows through a buffer descriptor (bf16): element (r, k) at base[r*ld + k].
// voffset = the lane's row start + its 16-B chunk (fixed), soffset = k-step * 128 B.  Only the
// last k-step of a K that is not a multiple of 64 tests k < K.
template <int R, class T = __bf16, int NW = 4>
struct KCDenseBuf {
  static constexpr bool KC = true;
  static constexpr bool BUF = true;
  static constexpr int NI = R / (8 * NW);
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t vo[NI];
  uint32_t soff;
  uint32_t kcol, K;
  int kt_tail;  // the k-step whose chunks may pass K (-1: K % 64 == 0)
  __device__ void prep(int kt) { soff = (uint32_t)kt * (BK * sizeof(T)); }
  __device__ void init(const T* base, long ld, uint32_t rows_total, uint32_t K_,
                       uint32_t origin, int wave, int lane, const void*) {
    K = K_;
    kcol = KCGeom<R, NW>::chunk(lane) * 8;
    kt_tail = __builtin_amdgcn_readfirstlane((K % BK) ? (int)(K / BK) : -1);  // SGPR: a scalar branch
    rsrc = gk_rsrc(base, (uint64_t)rows_total * (uint64_t)ld * sizeof(T));
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const uint32_t r = origin + KCGeom<R, NW>::row(wave, i, lane);
      vo[i] = r < rows_total ? (uint32_t)(((long)r * ld + kcol) * sizeof(T)) : kOOB;
    }
  }
  __device__ bool tail(int kt) const { return kt == kt_tail; }
  __device__ uint32_t voff(int kt, int i) const {
    if (kt == kt_tail) return (uint32_t)kt * BK + kcol < K ? vo[i] : kOOB;  // wave-uniform test
    return vo[i];
  }
};

// Dense MN-contiguous operand through a buffer descriptor (bf16): element (k, col) at
// base[k*ld + col].  voffset = the lane's (k row within the step, 8-column chunk), soffset =
// k-step * 64 * ld * 2 B.
template <int W, class T = __bf16, int NW = 4>
struct MCDenseBuf {
  static constexpr bool KC = false;
  static constexpr bool BUF = true;
  static constexpr int NI = W / (8 * NW);
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t vo[NI];
  uint32_t krow[NI];
  uint32_t soff, K;
  long ld;
  int kt_tail;
  __device__ void prep(int kt) { soff = (uint32_t)((long)kt * BK * ld * (long)sizeof(T)); }
  __device__ void init(const T* base, long ld_, uint32_t cols_total, uint32_t K_,
                       uint32_t origin, int wave, int lane, const void*) {
    ld = ld_;
    K = K_;
    kt_tail = __builtin_amdgcn_readfirstlane((K % BK) ? (int)(K / BK) : -1);  // SGPR: a scalar branch
    rsrc = gk_rsrc(base, (uint64_t)K * (uint64_t)ld * sizeof(T));
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      krow[i] = MCGeom<W, NW>::row(wave, i, lane);
      const uint32_t col = origin + MCGeom<W, NW>::chunk(wave, i, lane) * 8;
      vo[i] = col < cols_total ? (uint32_t)(((long)krow[i] * ld + col) * sizeof(T)) : kOOB;
    }
  }
  __device__ bool tail(int kt) const { return kt == kt_tail; }
  __device__ uint32_t voff(int kt, int i) const {
    if (kt == kt_tail) return (uint32_t)kt * BK + krow[i] < K ? vo[i] : kOOB;
    return vo[i];
  }
};

// ---------------------------------------------------------------------------------------------
// Folded BatchNorm on an operand (the producing BN's apply + ReLU moved into its consumer's
// operand path, so the normalised activation is never written): policies with XFORM = true
// transform each bf16 fragment after its LDS read, v -> bf16(max(v*scale[c] + bias[c], 0)) —
// the bits bn_act_fwd would have stored (same fused multiply-add, ReLU, round-to-nearest).
template <class Op, class = void>
struct HasXform : std::false_type {};
template <class Op>
struct HasXform<Op, std::void_t<decltype(Op::XFORM)>> : std::integral_constant<bool, Op::XFORM> {};

__device__ __forceinline__ bf16x8 bn_relu_frag(bf16x8 v, const float (&sc)[8], const float (&bi)[8]) {
  const uint4 u = __builtin_bit_cast(uint4, v);
  float f[8];
  unpack8(u, f);
#pragma unroll
  for (int q = 0; q < 8; ++q) f[q] = fmaxf(f[q] * sc[q] + bi[q], 0.f);
  return __builtin_bit_cast(bf16x8, pack8(f));
}

// A operand of a dense 1x1 conv whose input is relu(bn(y)) (x = y in memory): k = input
// channel.  The per-channel (scale, bias) pairs sit in an LDS table the kernel fills before the
// main loop (tab: float2 per channel, zeros past K so padded channels stay 0).  Each k-step's
// landed A image is transformed IN PLACE once per block (xform_lds), before any wave reads a
// fragment: a thread owns one 8-channel chunk slot (t & 7) for every row it visits, so its 16
// coefficients are four ds_read_b128 per k-step, and each element is transformed once per block
// (a per-fragment transform redid it in every wave that reads the fragment, in front of the
// MFMAs: profiles/r6_bn_fold_negative.txt).
template <int R, class T = __bf16, int NW = 4>
struct KCDenseBufBN : KCDenseBuf<R, T, NW> {
  static constexpr bool XFORM = true;
  const char* tab;
  __device__ void xform_lds(char* img, int kt, int tid, int nthreads) const {
    const uint32_t c = (uint32_t)tid & 7u;
    const float4* t = reinterpret_cast<const float4*>(tab + ((uint32_t)kt * BK + c * 8) * 8);
    const float4 t0 = t[0], t1 = t[1], t2 = t[2], t3 = t[3];
    const float sc[8] = {t0.x, t0.z, t1.x, t1.z, t2.x, t2.z, t3.x, t3.z};
    const float bi[8] = {t0.y, t0.w, t1.y, t1.w, t2.y, t2.w, t3.y, t3.w};
    for (uint32_t r = (uint32_t)tid >> 3; r < (uint32_t)R; r += (uint32_t)nthreads >> 3) {
      bf16x8* p = reinterpret_cast<bf16x8*>(img + kc_off(r, c));
      *p = bn_relu_frag(*p, sc, bi);
    }
  }
};

// B operand of a dense 1x1 conv's weight-grad whose input was relu(bn(y)): B(k = pixel, n =
// input channel) = y (MN-contiguous image [64 k][W cols]).  Transformed in place once per block
// and k-step like KCDenseBufBN: a thread owns one 8-column chunk (t % (W/8)) — its 16
// coefficients are loaded once per tile (xform_setup) — and visits rows t / (W/8), +nthreads/(W/8)...
// Rows past K (the tail k-step) stay the range check's zeros (relu(bias) otherwise).
template <int W, class T = __bf16, int NW = 4>
struct MCDenseBufBN : MCDenseBuf<W, T, NW> {
  static constexpr bool XFORM = true;
  static constexpr int CPR = W / 8;  // 8-column chunks per image row
  const float* g_sc;
  const float* g_bi;
  uint32_t origin, ncols;
  float sc[8], bi[8];
  __device__ void xform_setup(int tid) {
    const uint32_t n0 = origin + ((uint32_t)tid % CPR) * 8;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const bool ok = n0 + q < ncols;
      sc[q] = ok ? g_sc[n0 + q] : 0.f;
      bi[q] = ok ? g_bi[n0 + q] : 0.f;
    }
  }
  __device__ void xform_lds(char* img, int kt, int tid, int nthreads) const {
    const uint32_t cc = (uint32_t)tid % CPR;
    uint32_t rows = (uint32_t)BK;
    if (kt == this->kt_tail) rows = this->K - (uint32_t)kt * BK;  // wave-uniform
    for (uint32_t r = (uint32_t)tid / CPR; r < rows; r += (uint32_t)nthreads / CPR) {
      bf16x8* p = reinterpret_cast<bf16x8*>(img + mc_off<W>(r, cc));
      *p = bn_relu_frag(*p, sc, bi);
    }
  }
};

// Conv forward A operand: im2col of NHWC x.  row m -> (img, ho, wo); k -> (kh, kw, ci).
struct ConvGeom {
  int N, H, W, C;        // input
  int Ho, Wo;            // output
  int KH, KW, stride, pad;
  FastDiv fHoWo, fWo, fC, fKW;
  int stride_w;          // horizontal stride (== stride for square strides)
  int pad_w;             // horizontal padding (== pad for square padding)
};

template <int R, bool ALIGNED = false, class T = __bf16, int NW = 4>
struct KCIm2col {
  static constexpr bool KC = true;
  static constexpr int NI = R / (8 * NW);
  const T* x;
  int hi0[NI], wi0[NI];
  int rowoff[NI];   // ((img*H + hi0)*W + wi0)*C  (32-bit: host checks numel < 2^31)
  uint32_t kcol, K;
  ConvGeom g;
  const void* zero;
  int p_kh, p_kw, p_toff;  // ALIGNED: this k-step's tap (kh, kw) and (kh*W + kw)*C + ci0 + kcol
  bool p_kok;
  __device__ void init(const T* x_, const ConvGeom& g_, uint32_t M, uint32_t origin, int wave,
                       int lane, const void* zero_page) {
    x = x_;
    g = g_;
    zero = zero_page;
    K = (uint32_t)(g.KH * g.KW * g.C);
    kcol = KCGeom<R, NW>::chunk(lane) * 8;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      uint32_t m = origin + KCGeom<R, NW>::row(wave, i, lane);
      if (m < M) {
        uint32_t img = fdiv(g.fHoWo, m);
        uint32_t rem = m - img * (uint32_t)(g.Ho * g.Wo);
        uint32_t ho = fdiv(g.fWo, rem);
        uint32_t wo = rem - ho * (uint32_t)g.Wo;
        hi0[i] = (int)ho * g.stride - g.pad;
        wi0[i] = (int)wo * g.stride_w - g.pad_w;
        rowoff[i] = (((int)img * g.H + hi0[i]) * g.W + wi0[i]) * g.C;
      } else {
        hi0[i] = wi0[i] = -100000;  // fails every bounds check
        rowoff[i] = 0;
      }
    }
  }
  // Branch-free, 32-bit address math.  ALIGNED (C % 64 == 0): a 64-wide k-step never
  // straddles a filter tap, so (kh, kw, ci0) are computed once per k-step in prep() as
  // wave-uniform scalars and a lane adds only its row offset; out-of-image taps select the
  // zero page.
  __device__ void prep(int kt) {
    if constexpr (ALIGNED) {
      const uint32_t k0 = (uint32_t)kt * BK;
      const uint32_t tap = fdiv(g.fC, k0);
      const uint32_t kh = fdiv(g.fKW, tap);
      const uint32_t kw = tap - kh * (uint32_t)g.KW;
      p_kh = (int)kh;
      p_kw = (int)kw;
      p_toff = ((int)kh * g.W + (int)kw) * g.C + (int)(k0 - tap * (uint32_t)g.C) + (int)kcol;
      p_kok = k0 < K;
    }
  }
  __device__ const void* src(int kt, int i) const {
    int kh, kw, off;
    bool kok;
    if constexpr (ALIGNED) {
      kh = p_kh; kw = p_kw; kok = p_kok;
      off = rowoff[i] + p_toff;
    } else {
      const uint32_t k = (uint32_t)kt * BK + kcol;
      const uint32_t tap = fdiv(g.fC, k);
      const uint32_t ukh = fdiv(g.fKW, tap);
      kh = (int)ukh;
      kw = (int)(tap - ukh * (uint32_t)g.KW);
      kok = k < K;
      off = rowoff[i] + (kh * g.W + kw) * g.C + (int)(k - tap * (uint32_t)g.C);
    }
    const int hi = hi0[i] + kh, wi = wi0[i] + kw;
    const bool ok = kok & ((unsigned)hi < (unsigned)g.H) & ((unsigned)wi < (unsigned)g.W);
    return ok ? (const void*)(x + off) : zero;
  }
};

// Conv forward A operand (bf16, C % 64 == 0, KH*KW <= 32) through a buffer descriptor: the
// descriptor starts SHIFT = (pad*W + pad_w)*C elements before x, so a lane's row offset
// rowoff + SHIFT is never negative; per k-step the tap (kh, kw) and channel block are
// wave-uniform (soffset = ((kh*W + kw)*C + ci0) * 2 B), and a per-row bit mask over the taps,
// built once per tile, decides whether the tap lies inside the image (else kOOB: zeros).
// Per piece: one bit test + select, instead of 64-bit address math + bounds compares.
template <int R, class T = __bf16, int NW = 4>
struct KCIm2colBuf {
  static constexpr bool KC = true;
  static constexpr bool BUF = true;
  static constexpr int NI = R / (8 * NW);
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t vo[NI];
  uint32_t mask[NI];
  uint32_t soff, tap;
  ConvGeom g;
  __device__ void init(const T* x_, const ConvGeom& g_, uint32_t M, uint32_t origin, int wave,
                       int lane, const void*) {
    g = g_;
    const long shift = ((long)g.pad * g.W + g.pad_w) * g.C;
    rsrc = gk_rsrc(x_ - shift, ((uint64_t)g.N * g.H * g.W * g.C + shift) * sizeof(T));
    const uint32_t kcol = KCGeom<R, NW>::chunk(lane) * 8;
    // tap bit t = kh*KW + kw.  A row's valid taps are a kh range x a kw range: one KW-bit group
    // pattern P (the kw range) replicated into every group by a carry-free multiply with
    // REP = sum_kh 2^(kh*KW), then cut to the kh range.
    uint64_t rep = 0;
    for (int kh = 0; kh < g.KH; ++kh) rep |= 1ull << (kh * g.KW);  // wave-uniform
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const uint32_t m = origin + KCGeom<R, NW>::row(wave, i, lane);
      uint32_t mk = 0u, v = kOOB;
      if (m < M) {
        const uint32_t img = fdiv(g.fHoWo, m);
        const uint32_t rem = m - img * (uint32_t)(g.Ho * g.Wo);
        const uint32_t ho = fdiv(g.fWo, rem);
        const uint32_t wo = rem - ho * (uint32_t)g.Wo;
        const int hi0 = (int)ho * g.stride - g.pad, wi0 = (int)wo * g.stride_w - g.pad_w;
        v = (uint32_t)(((((long)img * g.H + hi0) * g.W + wi0) * g.C + shift + kcol) * sizeof(T));
        const int kh_lo = max(0, -hi0), kh_hi = min(g.KH, g.H - hi0);
        const int kw_lo = max(0, -wi0), kw_hi = min(g.KW, g.W - wi0);
        if (kh_hi > kh_lo && kw_hi > kw_lo) {
          const uint64_t pat = ((1ull << (kw_hi - kw_lo)) - 1ull) << kw_lo;
          const uint64_t rng = ((1ull << (kh_hi * g.KW)) - 1ull) & ~((1ull << (kh_lo * g.KW)) - 1ull);
          mk = (uint32_t)((pat * rep) & rng);
        }
      }
      vo[i] = v;
      mask[i] = mk;
    }
  }
  __device__ void prep(int kt) {
    const uint32_t k0 = (uint32_t)kt * BK;
    const uint32_t t = fdiv(g.fC, k0);
    const uint32_t kh = fdiv(g.fKW, t);
    const uint32_t kw = t - kh * (uint32_t)g.KW;
    // wave-uniform; the readfirstlane keeps it provably so: a soffset the backend finds in a VGPR
    // turns every LDS-DMA piece into a waterfall loop (readfirstlane / cmp / saveexec / branch)
    tap = __builtin_amdgcn_readfirstlane(t);
    soff = __builtin_amdgcn_readfirstlane(
        (uint32_t)((((long)kh * g.W + kw) * g.C + (k0 - t * (uint32_t)g.C)) * sizeof(T)));
  }
  __device__ uint32_t voff(int, int i) const { return (mask[i] >> tap) & 1u ? vo[i] : kOOB; }
};

// Conv data-grad, sub-pixel ("parity class") form.  For stride s the dx pixels split into s*s
// classes (ph, pw); class pixels (h, w) = (ph + s*i, pw + s*j) receive contributions only from the
// taps with kh = (ph + pad) mod s (and kw likewise), each through dy[i + dh, j + dw] with a fixed
// offset (dh, dw) = ((ph + pad - kh)/s, (pw + pad - kw)/s).  So every class is a dense GEMM over
// its own tap list — no MFMA work is spent on the (s*s - 1)/(s*s) structurally-zero products a
// masked implicit GEMM would do.  Stride 1 is the single class with every tap.
struct DgradClass {
  int Hc, Wc;          // class grid
  int ph, pw;          // phase
  int ntaps;           // nkh * nkw
  int kh0, kw0;        // first tap of the class; taps kh = kh0 + s*a, kw = kw0 + s*b
  int nkw;             // taps along kw
  int dh0, dw0;        // dy offset of the first tap: dh = dh0 - a, dw = dw0 - b
  int S, KW;
  FastDiv fHcWc, fWc, fnkw;
};

template <int R, bool ALIGNED = false, class T = __bf16, int NW = 4>
struct KCDgrad {
  static constexpr bool KC = true;
  static constexpr int NI = R / (8 * NW);
  const T* dy;
  int ib[NI], jb[NI];   // i + dh0, j + dw0 (dy row/col of the class's first tap)
  int rowoff[NI];       // ((img*Ho + ib)*Wo + jb)*Co  (32-bit: host checks numel < 2^31)
  uint32_t kcol, K;
  int Ho, Wo, Co;
  FastDiv fCo, fnkw;
  const void* zero;
  int p_a, p_b, p_toff;  // ALIGNED: this k-step's tap offsets and -(a*Wo + b)*Co + co0 + kcol
  bool p_kok;
  __device__ void init(const T* dy_, int Ho_, int Wo_, int Co_, FastDiv fCo_,
                       const DgradClass& cls, uint32_t M, uint32_t origin, int wave, int lane,
                       const void* zero_page) {
    dy = dy_; Ho = Ho_; Wo = Wo_; Co = Co_; fCo = fCo_; fnkw = cls.fnkw;
    zero = zero_page;
    K = (uint32_t)(cls.ntaps * Co);
    kcol = KCGeom<R, NW>::chunk(lane) * 8;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      uint32_t m = origin + KCGeom<R, NW>::row(wave, i, lane);
      if (m < M) {
        uint32_t img = fdiv(cls.fHcWc, m);
        uint32_t rem = m - img * (uint32_t)(cls.Hc * cls.Wc);
        uint32_t ii = fdiv(cls.fWc, rem);
        ib[i] = (int)ii + cls.dh0;
        jb[i] = (int)(rem - ii * (uint32_t)cls.Wc) + cls.dw0;
        rowoff[i] = (((int)img * Ho + ib[i]) * Wo + jb[i]) * Co;
      } else {
        ib[i] = jb[i] = -100000;
        rowoff[i] = 0;
      }
    }
  }
  __device__ void prep(int kt) {
    if constexpr (ALIGNED) {  // Co % 64 == 0: the tap index is wave-uniform per k-step
      const uint32_t k0 = (uint32_t)kt * BK;
      const uint32_t t = fdiv(fCo, k0);
      const uint32_t a = fdiv(fnkw, t);
      const uint32_t b = t - a * fnkw.d;
      p_a = (int)a;
      p_b = (int)b;
      p_toff = -((int)a * Wo + (int)b) * Co + (int)(k0 - t * (uint32_t)Co) + (int)kcol;
      p_kok = k0 < K;
    }
  }
  __device__ const void* src(int kt, int i) const {
    int a, b, off;
    bool kok;
    if constexpr (ALIGNED) {
      a = p_a; b = p_b; kok = p_kok;
      off = rowoff[i] + p_toff;
    } else {
      const uint32_t k = (uint32_t)kt * BK + kcol;
      const uint32_t t = fdiv(fCo, k);
      const uint32_t ua = fdiv(fnkw, t);
      a = (int)ua;
      b = (int)(t - ua * fnkw.d);
      kok = k < K;
      off = rowoff[i] - (a * Wo + b) * Co + (int)(k - t * (uint32_t)Co);
    }
    const int ho = ib[i] - a, wo = jb[i] - b;
    const bool ok = kok & ((unsigned)ho < (unsigned)Ho) & ((unsigned)wo < (unsigned)Wo);
    return ok ? (const void*)(dy + off) : zero;
  }
};

// Conv data-grad A operand (bf16, Co % 64 == 0: the class tap is wave-uniform per k-step)
// through a buffer descriptor.  dy element offset = rowoff - (a*Wo + b)*Co + co0 + kcol; the
// descriptor starts SH = ((nkh-1)*Wo + nkw-1)*Co elements before dy, so soffset =
// (SH - (a*Wo + b)*Co + co0) * 2 B is never negative.  Valid taps (ho = ib - a in [0, Ho),
// wo = jb - b in [0, Wo)) are an a range x b range: a per-row bit mask as in KCIm2colBuf.
template <int R, class T = __bf16, int NW = 4>
struct KCDgradBuf {
  static constexpr bool KC = true;
  static constexpr bool BUF = true;
  static constexpr int NI = R / (8 * NW);
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t vo[NI];
  uint32_t mask[NI];
  uint32_t soff, tap;
  int Wo, Co, sh;
  FastDiv fCo, fnkw;
  __device__ void init(const T* dy_, int Ho_, int Wo_, int Co_, FastDiv fCo_,
                       const DgradClass& cls, uint32_t M, uint32_t origin, int wave, int lane,
                       const void*) {
    Wo = Wo_; Co = Co_; fCo = fCo_; fnkw = cls.fnkw;
    const int nkw = (int)cls.fnkw.d;
    const int nkh = nkw > 0 ? cls.ntaps / nkw : 0;
    sh = ((nkh > 0 ? nkh - 1 : 0) * Wo + (nkw > 0 ? nkw - 1 : 0)) * Co;
    const int N = (int)(M / (uint32_t)(cls.Hc * cls.Wc));
    rsrc = gk_rsrc(dy_ - sh, ((uint64_t)(N > 0 ? N : 1) * Ho_ * Wo_ * Co_ + sh) * sizeof(T));
    const uint32_t kcol = KCGeom<R, NW>::chunk(lane) * 8;
    uint64_t rep = 0;
    for (int a = 0; a < nkh; ++a) rep |= 1ull << (a * nkw);  // wave-uniform
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const uint32_t m = origin + KCGeom<R, NW>::row(wave, i, lane);
      uint32_t mk = 0u, v = kOOB;
      if (m < M) {
        const uint32_t img = fdiv(cls.fHcWc, m);
        const uint32_t rem = m - img * (uint32_t)(cls.Hc * cls.Wc);
        const uint32_t ii = fdiv(cls.fWc, rem);
        const int ib = (int)ii + cls.dh0;
        const int jb = (int)(rem - ii * (uint32_t)cls.Wc) + cls.dw0;
        v = (uint32_t)(((((long)img * Ho_ + ib) * Wo + jb) * Co + kcol) * sizeof(T));
        const int a_lo = max(0, ib - Ho_ + 1), a_hi = min(nkh, ib + 1);
        const int b_lo = max(0, jb - Wo + 1), b_hi = min(nkw, jb + 1);
        if (a_hi > a_lo && b_hi > b_lo) {
          const uint64_t pat = ((1ull << (b_hi - b_lo)) - 1ull) << b_lo;
          const uint64_t rng = ((1ull << (a_hi * nkw)) - 1ull) & ~((1ull << (a_lo * nkw)) - 1ull);
          mk = (uint32_t)((pat * rep) & rng);
        }
      }
      vo[i] = v;
      mask[i] = mk;
    }
  }
  __device__ void prep(int kt) {
    const uint32_t k0 = (uint32_t)kt * BK;
    const uint32_t t = fdiv(fCo, k0);
    const uint32_t a = fdiv(fnkw, t);
    const uint32_t b = t - a * fnkw.d;
    tap = __builtin_amdgcn_readfirstlane(t);  // uniform: keep soffset an SGPR (KCIm2colBuf)
    soff = __builtin_amdgcn_readfirstlane(
        (uint32_t)(((long)sh - ((long)a * Wo + b) * Co + (k0 - t * (uint32_t)Co)) * sizeof(T)));
  }
  __device__ uint32_t voff(int, int i) const { return (mask[i] >> tap) & 1u ? vo[i] : kOOB; }
};

// Conv data-grad B operand (bf16, Co % 64 == 0) through a buffer descriptor: B(k = (t, co),
// n = ci) = W[co][tap(t)][ci]; per k-step t and co0 are wave-uniform, so the lane's part
// (krow*taps*Ci + col) is fixed and (co0*taps + tap)*Ci goes to soffset.
template <int W, class T = __bf16, int NW = 4>
struct MCDgradWBuf {
  static constexpr bool KC = false;
  static constexpr bool BUF = true;
  static constexpr int NI = W / (8 * NW);
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t vo[NI];
  uint32_t soff;
  uint32_t Co, taps, Ci;
  FastDiv fCo, fnkw;
  int kh0, kw0, S, KW;
  __device__ void init(const T* w, uint32_t Co_, uint32_t taps_, uint32_t Ci_, FastDiv fCo_,
                       const DgradClass& cls, uint32_t origin, int wave, int lane, const void*) {
    Co = Co_; taps = taps_; Ci = Ci_; fCo = fCo_; fnkw = cls.fnkw;
    kh0 = cls.kh0; kw0 = cls.kw0; S = cls.S; KW = cls.KW;
    rsrc = gk_rsrc(w, (uint64_t)Co * taps * Ci * sizeof(T));
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const uint32_t krow = MCGeom<W, NW>::row(wave, i, lane);
      const uint32_t col = origin + MCGeom<W, NW>::chunk(wave, i, lane) * 8;
      vo[i] = col < Ci ? (uint32_t)(((long)krow * taps * Ci + col) * sizeof(T)) : kOOB;
    }
  }
  __device__ void prep(int kt) {
    const uint32_t k0 = (uint32_t)kt * BK;
    const uint32_t t = fdiv(fCo, k0);
    const uint32_t co0 = k0 - t * Co;
    const uint32_t a = fdiv(fnkw, t);
    const uint32_t b = t - a * fnkw.d;
    const uint32_t tp = (uint32_t)(kh0 + S * (int)a) * (uint32_t)KW + (uint32_t)(kw0 + S * (int)b);
    soff = __builtin_amdgcn_readfirstlane((uint32_t)(((long)co0 * taps + tp) * Ci * sizeof(T)));
  }
  __device__ uint32_t voff(int, int i) const { return vo[i]; }
};

// Dense MN-contiguous operand: element (k, col) at base[k*ld + col]; W columns per tile.
template <int W, class T = __bf16, int NW = 4>
struct MCDense {
  static constexpr bool KC = false;
  static constexpr int NI = W / (8 * NW);
  const T* colptr[NI];
  uint32_t krow[NI];
  long ld;
  uint32_t K;
  const void* zero;
  __device__ void prep(int) {}
  __device__ void init(const T* base, long ld_, uint32_t cols_total, uint32_t K_,
                       uint32_t origin, int wave, int lane, const void* zero_page) {
    ld = ld_;
    K = K_;
    zero = zero_page;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      krow[i] = MCGeom<W, NW>::row(wave, i, lane);
      uint32_t col = origin + MCGeom<W, NW>::chunk(wave, i, lane) * 8;
      colptr[i] = col < cols_total ? base + col : nullptr;
    }
  }
  __device__ const void* src(int kt, int i) const {
    uint32_t k = (uint32_t)kt * BK + krow[i];
    return (colptr[i] != nullptr && k < K) ? (const void*)(colptr[i] + (long)k * ld) : zero;
  }
};

// Conv data-grad B operand: B(k = (t, co), n = ci) = W[co][tap(t)][ci] (weights [Co,KH,KW,Ci]).
template <int W, class T = __bf16, int NW = 4>
struct MCDgradW {
  static constexpr bool KC = false;
  static constexpr int NI = W / (8 * NW);
  const T* colptr[NI];
  uint32_t krow[NI];
  uint32_t K, Co, taps, Ci;
  FastDiv fCo, fnkw;
  int kh0, kw0, S, KW;
  const void* zero;
  __device__ void prep(int) {}
  __device__ void init(const T* w, uint32_t Co_, uint32_t taps_, uint32_t Ci_, FastDiv fCo_,
                       const DgradClass& cls, uint32_t origin, int wave, int lane,
                       const void* zero_page) {
    Co = Co_; taps = taps_; Ci = Ci_; fCo = fCo_; fnkw = cls.fnkw;
    kh0 = cls.kh0; kw0 = cls.kw0; S = cls.S; KW = cls.KW;
    K = Co * (uint32_t)cls.ntaps;
    zero = zero_page;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      krow[i] = MCGeom<W, NW>::row(wave, i, lane);
      uint32_t col = origin + MCGeom<W, NW>::chunk(wave, i, lane) * 8;
      colptr[i] = col < Ci ? w + col : nullptr;
    }
  }
  __device__ const void* src(int kt, int i) const {
    uint32_t k = (uint32_t)kt * BK + krow[i];
    if (colptr[i] == nullptr || k >= K) return zero;
    uint32_t t = fdiv(fCo, k);
    uint32_t co = k - t * Co;
    uint32_t a = fdiv(fnkw, t);
    uint32_t b = t - a * fnkw.d;
    uint32_t tap = (uint32_t)(kh0 + S * (int)a) * (uint32_t)KW + (uint32_t)(kw0 + S * (int)b);
    return colptr[i] + ((long)co * taps + tap) * Ci;
  }
};

// Conv weight-grad B operand: B(k = output pixel, n = (kh,kw,ci)) = x[img, ho*s-p+kh, wo*s-p+kw, ci].
template <int W, class T = __bf16, int NW = 4>
struct MCIm2colT {
  static constexpr bool KC = false;
  static constexpr int NI = W / (8 * NW);
  const T* x;
  uint32_t krow[NI];
  int kh[NI], kw[NI], ci[NI];
  bool colok[NI];
  uint32_t K;
  ConvGeom g;
  const void* zero;
  __device__ void prep(int) {}
  __device__ void init(const T* x_, const ConvGeom& g_, uint32_t origin, int wave, int lane,
                       const void* zero_page, int /*kt0*/ = 0) {
    x = x_;
    g = g_;
    zero = zero_page;
    K = (uint32_t)(g.N * g.Ho * g.Wo);
    uint32_t Ntot = (uint32_t)(g.KH * g.KW * g.C);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      krow[i] = MCGeom<W, NW>::row(wave, i, lane);
      uint32_t n = origin + MCGeom<W, NW>::chunk(wave, i, lane) * 8;
      colok[i] = n < Ntot;
      uint32_t tap = fdiv(g.fC, n);
      ci[i] = (int)(n - tap * (uint32_t)g.C);
      uint32_t a = fdiv(g.fKW, tap);
      kh[i] = (int)a;
      kw[i] = (int)(tap - a * (uint32_t)g.KW);
    }
  }
  // branch-free, 32-bit offsets (host checks numel < 2^31); the zero page via select
  __device__ const void* src(int kt, int i) const {
    const uint32_t k = (uint32_t)kt * BK + krow[i];
    const uint32_t img = fdiv(g.fHoWo, k);
    const uint32_t rem = k - img * (uint32_t)(g.Ho * g.Wo);
    const uint32_t ho = fdiv(g.fWo, rem);
    const uint32_t wo = rem - ho * (uint32_t)g.Wo;
    const int hi = (int)ho * g.stride - g.pad + kh[i];
    const int wi = (int)wo * g.stride_w - g.pad_w + kw[i];
    const bool ok = colok[i] & (k < K) & ((unsigned)hi < (unsigned)g.H) &
                    ((unsigned)wi < (unsigned)g.W);
    const int off = (((int)img * g.H + hi) * g.W + wi) * g.C + ci[i];
    return ok ? (const void*)(x + off) : zero;
  }
};

// Conv weight-grad B operand (bf16) through a buffer descriptor, pixel state carried per lane.
// The k index (output pixel) of a lane's row advances by 64 each k-step; instead of two fast
// divisions + address math per piece and step (MCIm2colT), each piece keeps its pixel as scaled
// coordinates (hs = ho*s, ws = wo*s_w) and its descriptor-relative element offset, and prep()
// adds the mixed-radix digits of 64 (d_img, d_ho, d_wo) with two carries.  prep(kt) must be
// called for kt0, kt0+1, ... in order (every main loop does; init takes kt0).  The descriptor
// starts SHIFT = (pad*W + pad_w)*C elements before x, so offsets are never negative; padding
// taps, pixels past N*Ho*Wo and columns past KH*KW*C get kOOB (zeros).
template <int W, class T = __bf16, int NW = 4>
struct MCIm2colTBuf {
  static constexpr bool KC = false;
  static constexpr bool BUF = true;
  static constexpr int NI = W / (8 * NW);
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t soff;            // always 0: the k-step lives in the per-lane state
  uint32_t vcur[NI];        // this k-step's voffsets (bytes), set by prep()
  uint32_t off[NI], kk[NI];
  int hs[NI], ws[NI], th[NI], tw[NI];
  bool colok[NI];
  int H, Wd, Hos, Wos, dhs, dws, s;
  uint32_t K, doff, cw, ch;
  __device__ void init(const T* x_, const ConvGeom& g, uint32_t origin, int wave, int lane,
                       const void*, int kt0) {
    H = g.H;
    Wd = g.W;
    s = g.stride;
    K = (uint32_t)(g.N * g.Ho * g.Wo);
    soff = 0;
    const long shift = ((long)g.pad * g.W + g.pad_w) * g.C;
    rsrc = gk_rsrc(x_ - shift, ((uint64_t)g.N * g.H * g.W * g.C + shift) * sizeof(T));
    const uint32_t HoWo = (uint32_t)(g.Ho * g.Wo);
    const uint32_t d_img = (uint32_t)BK / HoWo, rem = (uint32_t)BK - d_img * HoWo;
    const uint32_t d_ho = rem / (uint32_t)g.Wo, d_wo = rem - d_ho * (uint32_t)g.Wo;
    dws = (int)d_wo * g.stride_w;
    dhs = (int)d_ho * g.stride;
    Wos = g.Wo * g.stride_w;
    Hos = g.Ho * g.stride;
    doff = ((d_img * (uint32_t)g.H + (uint32_t)dhs) * (uint32_t)g.W + (uint32_t)dws) * (uint32_t)g.C;
    cw = (uint32_t)((g.stride * g.W - Wos) * g.C);         // wo wraps: ws -= Wo*s_w, hs += s
    ch = (uint32_t)((g.H - Hos) * g.W * g.C);              // ho wraps: hs -= Ho*s, img += 1
    const uint32_t Ntot = (uint32_t)(g.KH * g.KW * g.C);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const uint32_t krow = MCGeom<W, NW>::row(wave, i, lane);
      const uint32_t n = origin + MCGeom<W, NW>::chunk(wave, i, lane) * 8;
      colok[i] = n < Ntot;
      const uint32_t tap = fdiv(g.fC, n);
      const uint32_t ci = n - tap * (uint32_t)g.C;
      const uint32_t kh = fdiv(g.fKW, tap), kw = tap - kh * (uint32_t)g.KW;
      th[i] = (int)kh - g.pad;
      tw[i] = (int)kw - g.pad_w;
      const uint32_t k = (uint32_t)kt0 * BK + krow;
      kk[i] = k;
      const uint32_t img = fdiv(g.fHoWo, k), r = k - img * HoWo;
      const uint32_t ho = fdiv(g.fWo, r), wo = r - ho * (uint32_t)g.Wo;
      hs[i] = (int)ho * g.stride;
      ws[i] = (int)wo * g.stride_w;
      off[i] = ((img * (uint32_t)g.H + (uint32_t)hs[i]) * (uint32_t)g.W + (uint32_t)ws[i]) * (uint32_t)g.C +
               (kh * (uint32_t)g.W + kw) * (uint32_t)g.C + ci;
    }
  }
  __device__ void prep(int) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const bool ok = colok[i] & (kk[i] < K) & ((unsigned)(hs[i] + th[i]) < (unsigned)H) &
                      ((unsigned)(ws[i] + tw[i]) < (unsigned)Wd);
      vcur[i] = ok ? off[i] * (uint32_t)sizeof(T) : kOOB;
      ws[i] += dws;
      const bool c1 = ws[i] >= Wos;
      ws[i] -= c1 ? Wos : 0;
      hs[i] += dhs + (c1 ? s : 0);
      const bool c2 = hs[i] >= Hos;
      hs[i] -= c2 ? Hos : 0;
      off[i] += doff + (c1 ? cw : 0u) + (c2 ? ch : 0u);
      kk[i] += BK;
    }
  }
  __device__ uint32_t voff(int, int i) const { return vcur[i]; }
};

// ---------------------------------------------------------------------------------------------
// Fragment loads from an LDS stage.
template <bool KC, int R>
struct FragLoader;

template <int R>
struct FragLoader<true, R> {  // KC image: ds_read_b128
  __device__ static bf16x8 load(const char* img, uint32_t row0, int ks, int lane) {
    uint32_t row = row0 + (lane & 15);
    uint32_t chunk = ks * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + kc_off(row, chunk));
  }
};

template <int W>
struct FragLoader<false, W> {  // MC image: 2 x ds_read_b64_tr_b16
  __device__ static bf16x8 load(const char* img, uint32_t col0, int ks, int lane) {
    uint32_t g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    uint32_t c = (col0 >> 3) + (p >> 1);
    uint32_t k0 = ks * 32 + 8 * g + q;
    const char* a0 = img + mc_off<W>(k0, c) + 8 * (p & 1);
    const char* a1 = img + mc_off<W>(k0 + 4, c) + 8 * (p & 1);
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a1);
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
};

// ---------------------------------------------------------------------------------------------
// Wait until at most N of this wave's vector-memory operations (the LDS-DMA loads of younger
// stages) are outstanding.  s_waitcnt immediate on gfx9: vmcnt [3:0] + [15:14], expcnt [6:4],
// lgkmcnt [11:8]; the other counters are left at their maxima (no wait).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// Main-loop schedule variants (bit flags of MainLoop's V).
constexpr int kLoopRawBarrier = 1;  // lgkmcnt(0) + s_barrier instead of __syncthreads()
constexpr int kLoopPrio = 2;        // s_setprio(1) around the MFMA block
constexpr int kLoopSpread = 4;      // next stage's LDS-DMA pieces spread between MFMAs
// single-stage tiles: the next k-step's LDS-DMA is issued as soon as every wave holds this
// k-step's fragments in registers (a barrier after the reads), so it flies under this k-step's
// MFMAs instead of after them
constexpr int kLoopEarlyDma = 8;
#ifndef MIPIPE_LOOP_DEFAULT
#define MIPIPE_LOOP_DEFAULT 11
#endif
constexpr int kLoopDefault = MIPIPE_LOOP_DEFAULT;

// Main loop.  Returns accumulators acc[MT][NT] (swapped orientation: lane holds C[m][n..n+3]).
// WM x WN waves (4 or 8), wave tile (BM/WM) x (BN/WN) of 16x16 MFMA tiles.
// NS = LDS stages:
//  1: single buffer, k-steps strictly serial inside the block — the least LDS, so more blocks
//     fit per CU and the overlap comes from neighbouring blocks (short-K, memory-bound GEMMs);
//  2: double buffer, the next k-step's LDS-DMA in flight under this one's MFMAs;
//  3: triple buffer, two k-steps in flight; the wait before each step is a COUNTED vmcnt (the
//     youngest stage keeps flying) so HBM-latency misses overlap two steps of MFMAs.
// Per k-step (NS >= 2): wait own loads of stage k -> barrier (everyone's stage k landed, and
// everyone finished reading stage k-1's buffer) -> issue stage k+NS-1 into that buffer ->
// fragments + MFMAs of stage k.  One barrier per k-step.
template <int BM, int BN, class OpA, class OpB, int NS = 2, int WM = 2, int WN = 2, int V = kLoopDefault>
struct MainLoop {
  static constexpr int NW = WM * WN;
  static constexpr int MT = BM / WM / 16;  // 16-row tiles per wave
  static constexpr int NT = BN / WN / 16;
  static constexpr int A_BYTES = BM * BK * 2;
  static constexpr int B_BYTES = BN * BK * 2;
  static constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  static constexpr int LDS_BYTES = NS * STAGE_BYTES;
  static constexpr int LOADS = OpA::NI + OpB::NI;  // LDS-DMA instructions per wave per stage
  static constexpr int MFMAS = 2 * MT * NT;        // per wave per k-step
  static constexpr bool RAW_BARRIER = (V & kLoopRawBarrier) != 0;
  static constexpr bool PRIO = (V & kLoopPrio) != 0;
  static constexpr bool SPREAD = (V & kLoopSpread) != 0;
  static_assert(OpA::NI * 8 * NW == BM && OpB::NI * 8 * NW == BN, "policy wave count");
  static_assert(NS >= 1 && NS <= 3, "1..3 LDS stages");

  // one LDS-DMA instruction (piece p of LOADS) of stage kt
  template <bool CHECK = true>
  __device__ static void piece(char* buf, OpA& a, OpB& b, int kt, int wave, int p) {
    if (p < OpA::NI) dma16<CHECK>(a, kt, p, buf + (wave * OpA::NI + p) * 1024);
    else dma16<CHECK>(b, kt, p - OpA::NI, buf + A_BYTES + (wave * OpB::NI + p - OpA::NI) * 1024);
  }

  __device__ static void stage(char* buf, OpA& a, OpB& b, int kt, int wave) {
    a.prep(kt);  // per-k-step wave-uniform address state (filter tap ...), computed once
    b.prep(kt);
    if (is_tail(a, kt) || is_tail(b, kt)) {  // wave-uniform branch: at most one k-step
#pragma unroll
      for (int p = 0; p < LOADS; ++p) piece<true>(buf, a, b, kt, wave, p);
      tail_block_end();
    } else {
#pragma unroll
      for (int p = 0; p < LOADS; ++p) piece<false>(buf, a, b, kt, wave, p);
    }
  }

  // Block barrier.  RAW: this wave's LDS reads retired + s_barrier, WITHOUT the vmcnt(0) a
  // __syncthreads() fence adds (which would drain LDS-DMA stages meant to stay in flight).
  __device__ static void barrier() {
    if constexpr (RAW_BARRIER) {
      __builtin_amdgcn_s_waitcnt((7 << 4) | (0 << 8) | 15 | (3 << 14));  // lgkmcnt(0) only
      __builtin_amdgcn_s_barrier();
    } else {
      __syncthreads();
    }
  }

  // Fragments + MFMAs of one stage.  With SPREAD, the next stage's LOADS LDS-DMA pieces
  // (nbuf != nullptr) are issued between MFMA groups instead of in one burst before them.
  // FIRST: the k-step that starts the accumulation — its first MFMA of each tile takes C = 0
  // (an inline constant) instead of 64 zeroed accumulator registers
  // folded-BN operands (HasXform): the landed images of k-step kt transformed in place by the
  // whole block (every thread's chunks), between the "stage landed" barrier and the fragment
  // reads (the caller's next barrier orders the writes)
  __device__ static void xform_pass(char* buf, const OpA& a, const OpB& b, int kt) {
    if constexpr (HasXform<OpA>::value) a.xform_lds(buf, kt, (int)threadIdx.x, NW * 64);
    if constexpr (HasXform<OpB>::value) b.xform_lds(buf + A_BYTES, kt, (int)threadIdx.x, NW * 64);
  }
  static constexpr bool XF = HasXform<OpA>::value || HasXform<OpB>::value;

  template <bool FIRST = false>
  __device__ static void compute(const char* cbuf, f32x4 (&acc)[MT][NT], uint32_t arow0,
                                 uint32_t bcol0, int lane, char* nbuf, OpA& a, OpB& b, int nkt,
                                 int wave, int kt) {
    const char* aimg = cbuf;
    const char* bimg = cbuf + A_BYTES;
    // both k-substeps' fragments are requested up front, so the second substep's LDS reads
    // are in flight under the first substep's MFMAs (only a counted lgkmcnt before each)
    bf16x8 af[2][MT], bfr[2][NT];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
        af[ks][i] = FragLoader<OpA::KC, BM>::load(aimg, arow0 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < NT; ++j)
        bfr[ks][j] = FragLoader<OpB::KC, BN>::load(bimg, bcol0 + j * 16, ks, lane);
    }
    if constexpr (SPREAD) {
      if (nbuf != nullptr) {
        a.prep(nkt);
        b.prep(nkt);
      }
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              bfr[ks][j], af[ks][i], (FIRST && ks == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j],
              0, 0, 0);
          if constexpr (SPREAD) {
            constexpr int STEP = MFMAS / LOADS > 0 ? MFMAS / LOADS : 1;
            const int idx = (ks * MT + i) * NT + j;  // compile-time after unrolling
            if (idx % STEP == STEP - 1 && idx / STEP < LOADS && nbuf != nullptr)
              piece(nbuf, a, b, nkt, wave, idx / STEP);
          }
        }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  }

  // NS == 1 with kLoopEarlyDma: fragments of k-step kt -> barrier (the single buffer is free)
  // -> LDS-DMA of kt+1 -> MFMAs of kt
  template <bool FIRST>
  __device__ static void compute_then_refill(char* smem, f32x4 (&acc)[MT][NT], uint32_t arow0,
                                             uint32_t bcol0, int lane, OpA& a, OpB& b, int kt_next,
                                             int kt1, int wave) {
    const char* aimg = smem;
    const char* bimg = smem + A_BYTES;
    bf16x8 af[2][MT], bfr[2][NT];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
        af[ks][i] = FragLoader<OpA::KC, BM>::load(aimg, arow0 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < NT; ++j)
        bfr[ks][j] = FragLoader<OpB::KC, BN>::load(bimg, bcol0 + j * 16, ks, lane);
    }
    barrier();  // this wave's reads retired (lgkmcnt 0) and every other wave's: buffer free
    if (kt_next < kt1) stage(smem, a, b, kt_next, wave);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              bfr[ks][j], af[ks][i], (FIRST && ks == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j],
              0, 0, 0);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  }

  __device__ static void run(char* smem, OpA& a, OpB& b, int kt0, int kt1,
                             f32x4 (&acc)[MT][NT], int wave, int lane) {
    if (kt0 >= kt1) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      return;
    }
    const int wr = wave / WN, wc = wave % WN;
    const uint32_t arow0 = wr * (BM / WM), bcol0 = wc * (BN / WN);
    if constexpr (HasXform<OpB>::value) b.xform_setup((int)threadIdx.x);
    if constexpr (NS == 1 && (V & kLoopEarlyDma) != 0) {
      stage(smem, a, b, kt0, wave);
      for (int kt = kt0; kt < kt1; ++kt) {
        wait_vmcnt<0>();
        barrier();  // every wave's pieces of stage kt landed
        if constexpr (XF) {
          xform_pass(smem, a, b, kt);
          barrier();
        }
        if (kt == kt0) compute_then_refill<true>(smem, acc, arow0, bcol0, lane, a, b, kt + 1, kt1, wave);
        else compute_then_refill<false>(smem, acc, arow0, bcol0, lane, a, b, kt + 1, kt1, wave);
      }
    } else if constexpr (NS == 1) {
      for (int kt = kt0; kt < kt1; ++kt) {
        if (kt > kt0) __syncthreads();  // every wave is done reading the single buffer
        stage(smem, a, b, kt, wave);
        wait_vmcnt<0>();
        __syncthreads();
        if constexpr (XF) {
          xform_pass(smem, a, b, kt);
          __syncthreads();
        }
        if (kt == kt0) compute<true>(smem, acc, arow0, bcol0, lane, nullptr, a, b, 0, wave, kt);
        else compute(smem, acc, arow0, bcol0, lane, nullptr, a, b, 0, wave, kt);
      }
    } else {
#pragma unroll
      for (int s = 0; s < NS - 1; ++s)
        if (kt0 + s < kt1) stage(smem + s * STAGE_BYTES, a, b, kt0 + s, wave);
      int cur = 0;                // buffer of stage kt
      int nxt = NS - 1;           // buffer the stage kt + NS - 1 goes to
      for (int kt = kt0; kt < kt1; ++kt) {
        if constexpr (NS == 3) {
          if (kt + 1 < kt1) wait_vmcnt<LOADS>();  // stage kt+1 may stay in flight
          else wait_vmcnt<0>();
        } else {
          wait_vmcnt<0>();
        }
        barrier();
        if constexpr (XF) {
          xform_pass(smem + cur * STAGE_BYTES, a, b, kt);
          barrier();
        }
        const bool more = kt + NS - 1 < kt1;
        char* nb = more ? smem + nxt * STAGE_BYTES : nullptr;
        if constexpr (!SPREAD) {
          if (more) stage(nb, a, b, kt + NS - 1, wave);
          nb = nullptr;
        }
        if (kt == kt0)
          compute<true>(smem + cur * STAGE_BYTES, acc, arow0, bcol0, lane, nb, a, b,
                        kt + NS - 1, wave, kt);
        else
          compute(smem + cur * STAGE_BYTES, acc, arow0, bcol0, lane, nb, a, b, kt + NS - 1,
                  wave, kt);
        cur = cur + 1 == NS ? 0 : cur + 1;
        nxt = nxt + 1 == NS ? 0 : nxt + 1;
      }
    }
    // the epilogue reuses the stage buffers (statistics partials, output staging): every wave
    // must be done reading them
    __syncthreads();
  }
};

// fp32-operand main loop ("split-bf16x3", the reference-precision path).  Operands are fp32
// in memory; each lane's 8-element chunk (the same chunk the bf16 policies hand to glds) is read
// into registers one k-step ahead and split exactly into three bf16 parts
//   v = v0 + v1 + v2,  v0 = rn(v), v1 = rn(v - v0), v2 = rn(v - v0 - v1)
// (3 x 8 significant bits = fp32's 24), written as three bf16 LDS images in exactly the bf16
// layouts, so the fragment loaders are unchanged.  Each 16x16x32 tile takes 6 MFMAs — every
// partial product down to 2^-16 relative, smallest first:
//   a0*b2 + a1*b1 + a2*b0,  a0*b1 + a1*b0,  a0*b0
// bf16 x bf16 products are exact in the fp32 accumulator, so the result carries fp32-class
// error (~1e-7 relative; measured against float64 in tests/test_fp32_gpu.py) at 1/6 of the bf16
// MFMA rate — still ~2.6x the v_mfma_f32_16x16x4_f32 peak.  (A two-part split would lose 8 bits
// per operand: ~1e-5 errors, enough to flip near-zero ReLU decisions the float64 model makes.)
// STAGES = 1: one LDS stage; the register prefetch of step k+1 overlaps global latency with
// step k's MFMAs, and the split + store of k+1 waits behind a barrier for every wave to finish
// reading step k (two barriers per k-step, the split VALU never beside the MFMAs).
// STAGES = 2 (tiles with BM + BN <= 192: 144 KB of images, one block per CU): two image sets;
// registers hold steps k+1 and k+2, and the split + store of step k+1 into the OTHER stage
// follows step k's MFMAs in the same basic block (independent: the scheduler interleaves the
// split VALU with the MFMAs), one barrier per k-step.
template <int BM, int BN, class OpA, class OpB, int WM = 2, int WN = 2, int STAGES = 1>
struct MainLoopF32 {
  static_assert(!HasXform<OpA>::value && !HasXform<OpB>::value, "folded BN: bf16 loops only");
  static_assert(STAGES == 1 || STAGES == 2, "fp32 loop stages");
  static constexpr int MT = BM / WM / 16;
  static constexpr int NT = BN / WN / 16;
  static constexpr int PARTS = 3;
  static constexpr int A_BYTES = BM * BK * 2;
  static constexpr int B_BYTES = BN * BK * 2;
  static constexpr int IMG_BYTES = A_BYTES + B_BYTES;      // one part's image (A | B)
  static constexpr int STAGE_BYTES = PARTS * IMG_BYTES;    // part 0 | part 1 | part 2
  static constexpr int LDS_BYTES = STAGES * STAGE_BYTES;
  struct Regs {
    float4 a[OpA::NI][2];
    float4 b[OpB::NI][2];
  };

  __device__ static void load(Regs& r, OpA& a, OpB& b, int kt) {
    a.prep(kt);
    b.prep(kt);
#pragma unroll
    for (int i = 0; i < OpA::NI; ++i) {
      const float4* p = reinterpret_cast<const float4*>(a.src(kt, i));
      r.a[i][0] = p[0];
      r.a[i][1] = p[1];
    }
#pragma unroll
    for (int i = 0; i < OpB::NI; ++i) {
      const float4* p = reinterpret_cast<const float4*>(b.src(kt, i));
      r.b[i][0] = p[0];
      r.b[i][1] = p[1];
    }
  }

  __device__ static void split_store(char* dst, const float4 (&v)[2]) {
    const float f[8] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
    bf16x8 p0, p1, p2;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const __bf16 h = f2bf(f[q]);
      const float r1 = f[q] - bf2f(h);
      const __bf16 m = f2bf(r1);
      p0[q] = h;
      p1[q] = m;
      p2[q] = f2bf(r1 - bf2f(m));
    }
    *reinterpret_cast<bf16x8*>(dst) = p0;
    *reinterpret_cast<bf16x8*>(dst + IMG_BYTES) = p1;
    *reinterpret_cast<bf16x8*>(dst + 2 * IMG_BYTES) = p2;
  }

  // lane-linear destinations, the same bytes a glds16 of this chunk would have written
  __device__ static void store(char* smem, const Regs& r, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < OpA::NI; ++i)
      split_store(smem + (wave * OpA::NI + i) * 1024 + lane * 16, r.a[i]);
#pragma unroll
    for (int i = 0; i < OpB::NI; ++i)
      split_store(smem + A_BYTES + (wave * OpB::NI + i) * 1024 + lane * 16, r.b[i]);
  }

  // fragments + the 6 MFMAs per 16x16x32 tile of the stage at `img` (both k-substeps)
  __device__ static void mfmas(const char* img, f32x4 (&acc)[MT][NT], uint32_t arow0,
                               uint32_t bcol0, int lane) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[PARTS][MT], bfr[PARTS][NT];
#pragma unroll
      for (int p = 0; p < PARTS; ++p) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
          af[p][i] = FragLoader<OpA::KC, BM>::load(img + p * IMG_BYTES, arow0 + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < NT; ++j)
          bfr[p][j] = FragLoader<OpB::KC, BN>::load(img + p * IMG_BYTES + A_BYTES,
                                                    bcol0 + j * 16, ks, lane);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          f32x4 c = acc[i][j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[2][j], af[0][i], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[1][j], af[1][i], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[0][j], af[2][i], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[1][j], af[0][i], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[0][j], af[1][i], c, 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[0][j], af[0][i], c, 0, 0, 0);
        }
    }
  }

  // STAGES = 2, step k (stage CUR): registers r[CUR] held step k (already in LDS) and take step
  // k+2 now; step k's MFMAs; then step k+1 (registers r[1-CUR], loaded one step ago) is split
  // into the other stage; one barrier.
  template <int CUR>
  __device__ static void step2(char* smem, Regs (&r)[2], OpA& a, OpB& b, int kt, int kt1,
                               f32x4 (&acc)[MT][NT], uint32_t arow0, uint32_t bcol0, int wave,
                               int lane) {
    if (kt + 2 < kt1) load(r[CUR], a, b, kt + 2);
    mfmas(smem + CUR * STAGE_BYTES, acc, arow0, bcol0, lane);
    if (kt + 1 < kt1) store(smem + (1 - CUR) * STAGE_BYTES, r[1 - CUR], wave, lane);
    __syncthreads();  // stage 1-CUR written; every wave done reading stage CUR
  }

  __device__ static void run(char* smem, OpA& a, OpB& b, int kt0, int kt1,
                             f32x4 (&acc)[MT][NT], int wave, int lane) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (kt0 >= kt1) return;
    const int wr = wave / WN, wc = wave % WN;
    const uint32_t arow0 = wr * (BM / WM), bcol0 = wc * (BN / WN);
    if constexpr (STAGES == 2) {
      Regs r[2];
      load(r[0], a, b, kt0);
      if (kt0 + 1 < kt1) load(r[1], a, b, kt0 + 1);
      store(smem, r[0], wave, lane);
      __syncthreads();
      for (int kt = kt0; kt < kt1; kt += 2) {  // unrolled by two: the register sets stay static
        step2<0>(smem, r, a, b, kt, kt1, acc, arow0, bcol0, wave, lane);
        if (kt + 1 < kt1) step2<1>(smem, r, a, b, kt + 1, kt1, acc, arow0, bcol0, wave, lane);
      }
      return;  // (the last step's barrier: every wave is done reading before the epilogue)
    }
    Regs r;
    load(r, a, b, kt0);
    store(smem, r, wave, lane);
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) load(r, a, b, kt + 1);  // in flight under this step's MFMAs
      mfmas(smem, acc, arow0, bcol0, lane);
      if (more) {
        __syncthreads();  // every wave is done reading this step's images
        store(smem, r, wave, lane);
        __syncthreads();
      }
    }
    __syncthreads();  // the epilogue reuses the images
  }
};

// Two fp32 image stages (-DMIPIPE_F32_TWO_STAGE; tiles with BM + BN <= 192) measured SLOWER on
// the reference config: 291k vs 339k img/s, the 128x64 forwards 1,173 vs 883 us per step — one
// block per CU interleaving split VALU and MFMAs inside each wave loses to two single-stage
// blocks per CU interleaving them across blocks (profiles/r6_f32_two_stage_negative.txt).
#ifdef MIPIPE_F32_TWO_STAGE
constexpr bool kF32TwoStage = true;
#else
constexpr bool kF32TwoStage = false;
#endif
template <int BM, int BN>
constexpr int f32_stages() { return (kF32TwoStage && BM + BN <= 192) ? 2 : 1; }

// Selects the main loop for the operand element type.
template <class T, int BM, int BN, class OpA, class OpB, int NS = 2, int WM = 2, int WN = 2,
          int V = kLoopDefault>
struct MainLoopFor {
  typedef MainLoop<BM, BN, OpA, OpB, NS, WM, WN, V> type;
  static constexpr int LDS_BYTES = NS * (BM + BN) * BK * 2;
};
template <int BM, int BN, class OpA, class OpB, int NS, int WM, int WN, int V>
struct MainLoopFor<float, BM, BN, OpA, OpB, NS, WM, WN, V> {
  typedef MainLoopF32<BM, BN, OpA, OpB, WM, WN, f32_stages<BM, BN>()> type;
  static constexpr int LDS_BYTES = type::LDS_BYTES;
};

// Row/col of acc element: lane holds C[m][n + e], e = 0..3, for tile (i, j):
//   m = block_m0 + wr*(BM/2) + i*16 + (lane & 15)
//   n = block_n0 + wc*(BN/2) + j*16 + (lane >> 4)*4

}  // namespace gk
}  // namespace mipipe
