// The ResNet stem (7x7/2 conv -> BatchNorm -> ReLU -> 3x3/2 max-pool) fused around a conv that is
// computed twice in the forward instead of being written and re-read between passes.
//
// The unfused stem writes y (411 MB at b256), reads it for BN-apply + pool, reads it twice in the
// backward (BN-backward reduce and apply) and writes + reads the 411 MB conv gradient for the
// weight-grad.  The conv itself is 92 GFLOP (packed K = 224) ≈ 40 us of MFMA time, so:
//
//   stem_stats  : conv -> per-channel Σ(y-shift), Σ(y-shift)² (no y store)             [1x conv]
//   stem_pool   : conv -> y (stored for the backward) and z = relu(bn(y)) pooled
//                 3x3/2 in registers + an LDS ring -> pooled output + argmax            [1x conv]
//   backward    : pool_bn_bwd_reduce (pool.hip) -> Σg, Σg·x̂; then stem_bwd_wgrad: g routed
//                 from the pooled gradient, dy = A·g + B·y + C kept in LDS, dW += dyᵀ·im2col(x)
//                 (the BN-apply and the weight-grad in one pass: dy never reaches HBM)
//
// Measured alternatives (profiles/r3_stem_fused_*.txt): recomputing the conv in the backward
// as well (gather- or scatter-routed g) was VALU/latency-bound at 285-550 us per pass — the
// per-pixel routing costs more than reading y back.
//
// Input: the packed stem image xp [N][229][115][8] bf16 (stem_pack: 2 horizontally adjacent
// padded pixels x 4 channels per 16-byte super-pixel) and packed weights [64][7 kh][4 kwp][8]
// bf16; y[n][ho][wo][co] = Σ xp[n][2ho+kh][wo+kwp][c] w[co][kh][kwp][c].  A band = 4 conv rows of
// one image, one per wave; the rows it needs are 13 CONTIGUOUS xp rows (23,920 B), staged into
// LDS by linear LDS-DMA.  A k-step (kh) takes the 4 kwp taps: a lane's 8 k-values are one
// super-pixel = one ds_read_b128, so no im2col address math exists.  Numerics match the unfused
// path: y, z and dy are rounded to bf16 where it stores them.
#include "conv_common.hpp"

namespace mipipe {
namespace stem {

using gk::mc_off;
using gk::mc_swz;
using gk::wait_vmcnt;

constexpr int kWo = 112;                 // conv output width (7 pixel blocks of 16)
constexpr int kPB = 7;
constexpr int kCo = 64;                  // 4 channel blocks of 16
constexpr int kWsp = 115;                // packed input width
constexpr int kRowB = kWsp * 16;         // 1840 B per packed input row
constexpr int kRB = 4;                   // conv rows per band (one per wave)
constexpr int kBandRows = 2 * kRB + 5;   // 13 packed input rows per band
constexpr int kPatchValid = kBandRows * kRowB;  // 23,920 B
constexpr int kPatchB = 24 * 1024;
constexpr int kWStride = 464;            // LDS weight row: 448 B + 16 B pad (conflict-free b128)
constexpr int kWB = kCo * kWStride;      // 29,696 B
constexpr int kHp = 56, kWp = 56;        // pooled output (3x3 / 2 / pad 1)

struct Geo {
  const __bf16* xp;   // [N][Hp][115][8]
  const __bf16* w;    // [64][224]
  int N, Ho, Hp;      // conv rows per image, packed input rows per image
  uint32_t xp_bytes;  // N * Hp * 1840
};

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ bf16x8 ld128(uint32_t a) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  static_assert(N >= 0 && N <= 15, "lgkmcnt range");
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// weights -> LDS [64][464 B] (plain loads, once per block)
__device__ __forceinline__ void load_weights(char* wl, const __bf16* w, int tid, int nthreads) {
  for (int c = tid; c < kCo * 28; c += nthreads) {
    const int co = c / 28, ch = c - co * 28;
    const uint4 v = *reinterpret_cast<const uint4*>(w + co * 224 + ch * 8);
    *reinterpret_cast<uint4*>(wl + co * kWStride + ch * 16) = v;
  }
}

// stage band (n, conv rows ho0..ho0+3) of xp: 24 x 1 KiB linear LDS-DMA, 6 per wave (4 waves)
// Buffer descriptor over [base, base + bytes): LDS-DMA loads past the end return zeros (the
// range check replaces per-lane zero-page selects), offsets are 32-bit VGPRs.  Built from
// wave-uniform values only.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void buf_lds16(__amdgpu_buffer_rsrc_t r, char* lds_wave_base,
                                          uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds_wave_base, 16, voff, 0, 0, 0);
}

// stage band (n, conv rows ho0..ho0+3) of xp: 24 x 1 KiB linear LDS-DMA, 6 per wave (4 waves).
// The 13 rows are 23,920 B; the rest of the 24 KiB is never read.
__device__ __forceinline__ void stage_patch(char* pb, const Geo& g, int n, int ho0, int wave,
                                            int lane) {
  const auto r = buf_rsrc(g.xp, g.xp_bytes);
  const uint32_t v = (uint32_t)((n * g.Hp + 2 * ho0) * kRowB + wave * 6 * 1024 + lane * 16);
#pragma unroll
  for (int i = 0; i < 6; ++i) buf_lds16(r, pb + (wave * 6 + i) * 1024, v + i * 1024);
}

// One conv row (band row `r`) for this wave: acc[i][j] = C[px = 16i + (lane&15)][co = 16j +
// 4(lane>>4) + q].  7 k-steps (kh); the reads of step kh+1 are in flight under step kh's MFMAs.
__device__ __forceinline__ void conv_row(uint32_t patch, uint32_t wl, int r, int lane,
                                         f32x4 (&acc)[kPB][4]) {
#pragma unroll
  for (int i = 0; i < kPB; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int m = lane & 15, g = lane >> 4;
  // A: super-pixel (row 2r+kh, col px+kwp), kwp = g;  B: weight row co, chunk kh*4 + g
  const uint32_t abase = patch + (uint32_t)(((2 * r) * kWsp + m + g) * 16);
  const uint32_t bbase = wl + (uint32_t)(m * kWStride + g * 16);
  bf16x8 a[2][kPB], b[2][4];
  auto issue = [&](int kh, int s) {
#pragma unroll
    for (int j = 0; j < 4; ++j) b[s][j] = ld128(bbase + j * 16 * kWStride + kh * 64);
#pragma unroll
    for (int i = 0; i < kPB; ++i) a[s][i] = ld128(abase + (kh * kWsp + 16 * i) * 16);
  };
  issue(0, 0);
#pragma unroll
  for (int kh = 0; kh < 7; ++kh) {
    const int s = kh & 1;
    if (kh + 1 < 7) {
      issue(kh + 1, s ^ 1);
      wait_lgkm<11>();  // this step's 11 reads landed, the next step's 11 in flight
    } else {
      wait_lgkm<0>();
    }
#pragma unroll
    for (int i = 0; i < kPB; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[s][j], a[s][i], acc[i][j], 0, 0, 0);
  }
}

__device__ __forceinline__ float bfr(float v) { return bf2f(f2bf(v)); }

// ------------------------------------------------------------------------ F1: batch statistics
// Σ(y - shift), Σ(y - shift)² per channel of the bf16-rounded conv output (the conv epilogue's
// contract, epilogue.hpp): per-lane sums over the block's bands, DPP row sums, a fixed-order sum
// of the 4 waves, then one atomic per channel into replica row blockIdx % R (or, deterministic,
// a plain store of this block's partial row).
__global__ __launch_bounds__(256, 1) void stem_stats_kernel(Geo g, const float* __restrict__ shift,
                                                             float* __restrict__ ssum,
                                                             float* __restrict__ ssq, int R,
                                                             int det) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kPatchB + kWB];
  char* wl = smem + 2 * kPatchB;
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int bands_per_img = g.Ho / kRB, nb = g.N * bands_per_img;
  float sh[4][4], s[4][4], ss[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      sh[j][q] = shift[16 * j + 4 * (lane >> 4) + q];
      s[j][q] = ss[j][q] = 0.f;
    }
  load_weights(wl, g.w, tid, 256);
  int b = blockIdx.x;
  if (b < nb) stage_patch(smem, g, b / bands_per_img, (b % bands_per_img) * kRB, wave, lane);
  int cur = 0;
  for (; b < nb; b += gridDim.x) {
    const int nxt = b + (int)gridDim.x;
    wait_vmcnt<0>();
    __syncthreads();  // every wave's stage of `cur` landed; the other buffer is free
    if (nxt < nb)
      stage_patch(smem + (cur ^ 1) * kPatchB, g, nxt / bands_per_img, (nxt % bands_per_img) * kRB,
                  wave, lane);
    f32x4 acc[kPB][4];
    conv_row(lds_u32(smem + cur * kPatchB), lds_u32(wl), wave, lane, acc);
#pragma unroll
    for (int i = 0; i < kPB; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float d = bfr(acc[i][j][q]) - sh[j][q];
          s[j][q] += d;
          ss[j][q] += d * d;
        }
    cur ^= 1;
  }
  // lanes of one DPP row hold the same 4 channels (16 pixels each)
  __syncthreads();  // the stage buffers are reused for the wave partials
  float* red = reinterpret_cast<float*>(smem);  // [4 waves][2][64]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float a = row16_sum(s[j][q]), c = row16_sum(ss[j][q]);
      if ((lane & 15) == 0) {
        const int co = 16 * j + 4 * (lane >> 4) + q;
        red[(wave * 2 + 0) * kCo + co] = a;
        red[(wave * 2 + 1) * kCo + co] = c;
      }
    }
  __syncthreads();
  if (tid < 2 * kCo) {
    const int arr = tid / kCo, co = tid % kCo;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += red[(w * 2 + arr) * kCo + co];
    float* base = arr == 0 ? ssum : ssq;
    if (det) base[(long)blockIdx.x * kCo + co] = v;
    else atomicAdd(base + (long)(blockIdx.x % R) * kCo + co, v);
  }
}

// ------------------------------------------------------------------------ shared helpers
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(2))) short s16x2;

// lgkmcnt(0) + s_barrier without the vmcnt(0) a __syncthreads() fence adds: LDS-DMA prefetches
// and global loads / stores stay in flight across it.  The "memory" clobber keeps the compiler
// from moving LDS accesses across.
__device__ __forceinline__ void lds_barrier_raw() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// LDS accesses inside the band loops are inline asm: the compiler would make every LDS access
// it sees wait for all LDS-DMA prefetches in flight (vmcnt(0)), serialising the prefetch.
__device__ __forceinline__ void st32(uint32_t a, uint32_t x) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(x) : "memory");
}
__device__ __forceinline__ void st64(uint32_t a, uint32_t x, uint32_t y) {
  const u32x2 v = {x, y};
  asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void st128(uint32_t a, u32x4 v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t ld32(uint32_t a) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ uint32_t ld16(uint32_t a) {
  uint32_t v;
  asm volatile("ds_read_u16 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ void st16(uint32_t a, uint32_t x) {
  asm volatile("ds_write_b16 %0, %1" ::"v"(a), "v"(x) : "memory");
}
__device__ __forceinline__ u32x2 ld64(uint32_t a) {
  u32x2 v;
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ u32x4 ldk128(uint32_t a) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ s16x4 tr_read(uint32_t a) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ bf16x8 join(s16x4 lo, s16x4 hi) {
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t umax3(uint32_t a, uint32_t b, uint32_t c) {
  return max(max(a, b), c);
}
// ReLU on a packed bf16 pair: signed 16-bit max with 0 (negative values and -0 become +0)
__device__ __forceinline__ uint32_t relu_pk(uint32_t v) {
  s16x2 t = __builtin_bit_cast(s16x2, v);
  t = __builtin_elementwise_max(t, (s16x2){0, 0});
  return __builtin_bit_cast(uint32_t, t);
}

// ------------------------------------------------------------------------ F2: BN + ReLU + pool
// One block per image (28 bands).  Each wave turns its conv row into z = bf16(relu(bf16(y)*scale
// + bias)) and pools it HORIZONTALLY in registers on 32-bit keys (z bits << 16 | 15 - kw): a
// window's columns 2wo-1, 2wo, 2wo+1 are lanes m-1, m, m+1 of a DPP row (row_ror / row_shl; the
// m = 0 left neighbour comes from the previous pixel block), and one unsigned max3 picks the
// largest z with the smallest kw — non-negative bf16 bit patterns order like their values.  The
// 56-wide key rows go to an LDS ring of 5 rows; after a barrier the block pools VERTICALLY (key -
// 3*kh turns the code into 15 - tap): pooled rows 2b and 2b+1 take conv rows 4b-1 .. 4b+3 (row
// 4b-1 kept from band b-1).  First maximum in row-major tap order wins, as in pool_bn_fwd
// (pool.hip).  idx = kh*3 + kw, or 0xFF where the output is not > 0 (the backward's ReLU mask,
// folded in so the backward never reads the output).
constexpr int kKeyPix = 272;             // LDS bytes per h-pooled pixel: 64 keys + 16 B pad
constexpr int kKeyRow = kWp * kKeyPix;   // 15,232 B per ring row
__global__ __launch_bounds__(256, 1) void stem_pool_kernel(Geo g, const float* __restrict__ scale,
                                                            const float* __restrict__ bias,
                                                            __bf16* __restrict__ out,
                                                            uint8_t* __restrict__ idx,
                                                            __bf16* __restrict__ yout, bool nt) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kPatchB + kWB + 5 * kKeyRow];
  char* wl = smem + 2 * kPatchB;
  char* ring = wl + kWB;
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int m = lane & 15, grp = lane >> 4;
  const int n = blockIdx.x;
  const int nb = g.Ho / kRB, Hpo = g.Ho / 2;
  float sc[4][4], bi[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      sc[j][q] = scale[16 * j + 4 * grp + q];
      bi[j][q] = bias[16 * j + 4 * grp + q];
    }
  load_weights(wl, g.w, tid, 256);
  __syncthreads();  // weights and the per-lane vectors are resident before any LDS-DMA is issued
  stage_patch(smem, g, n, 0, wave, lane);
  for (int b = 0; b < nb; ++b) {
    const int cur = b & 1;
    // patch b landed: only band b-1's stores (issued after it: 28 of y unless eval, then 8 pool
    // stores on waves 0-1 and 6 on waves 2-3) may still be in flight
    if (b == 0) wait_vmcnt<0>();
    else if (yout != nullptr) {
      if (wave < 2) wait_vmcnt<36>();
      else wait_vmcnt<34>();
    } else {
      if (wave < 2) wait_vmcnt<8>();
      else wait_vmcnt<6>();
    }
    lds_barrier_raw();  // every wave's patch stage landed; band b-1's ring reads are done
    if (b + 1 < nb) stage_patch(smem + (cur ^ 1) * kPatchB, g, n, (b + 1) * kRB, wave, lane);
    f32x4 acc[kPB][4];
    conv_row(lds_u32(smem + cur * kPatchB), lds_u32(wl), wave, lane, acc);
    const int row = b * kRB + wave;
    if (yout != nullptr) {  // y (bf16) for the backward's BN reduction and BN-apply
      __bf16* yr = yout + (((long)n * g.Ho + row) * kWo + m) * kCo + 4 * grp;
#pragma unroll
      for (int i = 0; i < kPB; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
        {
          typedef __attribute__((ext_vector_type(2))) unsigned int u32v2;
          const u32v2 v = {pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3])};
          // y is read only by the backward: streaming stores when g_nt_store & 16
          if (nt) __builtin_nontemporal_store(v, reinterpret_cast<u32v2*>(yr + 16 * i * kCo + 16 * j));
          else *reinterpret_cast<u32v2*>(yr + 16 * i * kCo + 16 * j) = v;
        }
    }
    // even lanes m hold output column wo = 8i + m/2 after the horizontal max
    const uint32_t kb = lds_u32(ring + (row % 5) * kKeyRow) + (m >> 1) * kKeyPix + 16 * grp;
    uint32_t rprev[4][4];
#pragma unroll
    for (int i = 0; i < kPB; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t kc[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t yb = pack2(acc[i][j][2 * h], acc[i][j][2 * h + 1]);  // bf16(y) pair
          const float v0 = fmaf(__uint_as_float(yb << 16), sc[j][2 * h], bi[j][2 * h]);
          const float v1 = fmaf(__uint_as_float(yb & 0xffff0000u), sc[j][2 * h + 1], bi[j][2 * h + 1]);
          const uint32_t zb = relu_pk(pack2(v0, v1));
          kc[2 * h] = (zb << 16) | 14u;
          kc[2 * h + 1] = (zb & 0xffff0000u) | 14u;
        }
        u32x4 best;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t r = dpp_u<0x121>(kc[q]) + 1u;  // row_ror:1 -> lane m-1, code 15 (kw 0)
          uint32_t left = r;
          if (m == 0) left = i == 0 ? 0u : rprev[j][q];  // column -1 is padding: key 0 loses
          rprev[j][q] = r;
          const uint32_t right = dpp_u<0x101>(kc[q]) - 1u;  // row_shl:1 -> lane m+1, code 13
          best[q] = umax3(left, kc[q], right);
        }
        if ((m & 1) == 0) st128(kb + i * 8 * kKeyPix + 64 * j, best);
      }
    }
    lds_barrier_raw();  // the band's h-pooled key rows are in the ring
    // vertical pool: task = (pooled row 2b + pr, wo, 8 channels); 896 tasks, 3.5 per thread
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k == 3 && wave >= 2) break;  // wave-uniform: tasks 768..895 on waves 0, 1
      const int t = tid + 256 * k;
      const int pr = t / (kWp * 8), rem = t - pr * (kWp * 8);
      const int wo = rem >> 3, c8 = rem & 7;
      const int po = 2 * b + pr;
      uint32_t best[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
      u32x4 kv[3][2];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int hr = max(2 * po - 1 + kh, 0);  // row -1 (padding) is masked below
        const uint32_t a = lds_u32(ring + (hr % 5) * kKeyRow) + wo * kKeyPix + c8 * 32;
        kv[kh][0] = ldk128(a);
        kv[kh][1] = ldk128(a + 16);
      }
      wait_lgkm<0>();
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        if (2 * po - 1 + kh < 0) continue;
#pragma unroll
        for (int q = 0; q < 8; ++q) best[q] = max(best[q], kv[kh][q >> 2][q & 3] - 3u * kh);
      }
      uint32_t ov[4], tp[2] = {0u, 0u};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint32_t zb = best[q] >> 16;
        // ReLU mask: no gradient where the output is not > 0 (zero, or NaN as in pool.hip)
        const uint32_t tap = (zb == 0u || zb > 0x7f80u) ? 0xffu : 15u - (best[q] & 15u);
        tp[q >> 2] |= tap << (8 * (q & 3));
      }
#pragma unroll
      for (int h = 0; h < 4; ++h) ov[h] = (best[2 * h] >> 16) | (best[2 * h + 1] & 0xffff0000u);
      const long o = (((long)n * Hpo + po) * kWp + wo) * kCo + c8 * 8;
      *reinterpret_cast<uint4*>(out + o) = make_uint4(ov[0], ov[1], ov[2], ov[3]);
      *reinterpret_cast<uint2*>(idx + o) = make_uint2(tp[0], tp[1]);
    }
  }
}

// ------------------------------------------------------------------------ backward
// The BN-backward statistics (Σg, Σg·x̂) come from pool_bn_bwd_reduce (pool.hip) over y, dp and
// the argmax; this kernel fuses the rest: the BN-apply dy = A·g + B·y + C (pool_bn_bwd_apply's
// contract, dy never stored) and the stem weight-gradient dW = Σ dy ⊗ im2col(x).
//
// g at conv pixel (h, w), channels co..co+3: the pooled windows (a, b) covering it (1 or 2 per
// axis) whose tap is this pixel, in pool_grad_quad's order (rows, then columns).  The band's
// three pooled rows 2b..2b+2 (dp and idx) are staged into LDS by LDS-DMA with an XOR swizzle of
// 16-byte chunks chosen so the reads below (8 windows x 4 channel groups per 16-lane row) hit
// distinct banks:
//   dp  row [56 wo][128 B]: chunk ^ ((wo >> 1) & 3) << 1        (3 rows = 21,504 B)
//   idx row [56 wo][64 B] : chunk ^ ((wo >> 2) & 1)             (3 rows = 10,752 B, + 512 pad)
struct PoolGrad {
  const __bf16* dp;
  const uint8_t* idx;
  int Hpo;
};
constexpr int kDpRow = kWp * 128, kIxRow = kWp * 64;
constexpr int kPoolStage = 32 * 1024;  // 21 KiB dp + 11 KiB idx: 32 LDS-DMA loads, 8 per wave

// stage pooled rows 2b .. 2b+2 of image n (rows past the image read as zeros: dp = 0): this
// wave's loads u = 8*wave + k, 0..20 dp, 21..31 idx (the last one half padding)
__device__ __forceinline__ void stage_pooled(char* buf, const PoolGrad& pg, int n, int b, int wave,
                                             int lane) {
  const auto rd = buf_rsrc(reinterpret_cast<const char*>(pg.dp) + (long)n * pg.Hpo * kDpRow,
                           (uint32_t)(pg.Hpo * kDpRow));
  const auto ri = buf_rsrc(pg.idx + (long)n * pg.Hpo * kIxRow, (uint32_t)(pg.Hpo * kIxRow));
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int u = wave * 8 + k;  // wave-uniform
    if (u < 21) {
      const uint32_t p = (uint32_t)(u * 1024 + lane * 16);
      const uint32_t r3 = p / kDpRow, q = p - r3 * kDpRow;
      const uint32_t wo = q >> 7, ch = ((q >> 4) & 7) ^ (((wo >> 1) & 3) << 1);
      buf_lds16(rd, buf + u * 1024, (uint32_t)((2 * b + r3) * kDpRow) + wo * 128 + ch * 16);
    } else {
      const uint32_t p = (uint32_t)((u - 21) * 1024 + lane * 16);
      const uint32_t r3 = p / kIxRow, q = p - r3 * kIxRow;
      const uint32_t wo = q >> 6, ch = ((q >> 4) & 3) ^ ((wo >> 2) & 1);
      buf_lds16(ri, buf + u * 1024, (uint32_t)((2 * b + r3) * kIxRow) + wo * 64 + ch * 16);
    }
  }
}

// Per-lane offsets of the windows (b0 = w >> 1, b1 = (w + 1) >> 1) inside a staged pooled row,
// for pixel block i = 0 (block i adds i*1024 / i*512) and channel block j.
struct RouteOffs {
  uint32_t d0[4], d1[4], x0[4], x1[4];
  __device__ void init(int lane) {
    const int m = lane & 15, g = lane >> 4;
    const int c0 = m >> 1, c1 = (m + 1) >> 1;
    const int s0 = (m >> 2) & 3, s1 = ((m + 1) >> 2) & 3;
    const int t0 = (m >> 3) & 1, t1 = ((m + 1) >> 3) & 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      d0[j] = c0 * 128 + ((2 * (j ^ s0) + (g >> 1)) << 4) + 8 * (g & 1);
      d1[j] = c1 * 128 + ((2 * (j ^ s1) + (g >> 1)) << 4) + 8 * (g & 1);
      x0[j] = c0 * 64 + ((j ^ t0) << 4) + 4 * g;
      x1[j] = c1 * 64 + ((j ^ t1) << 4) + 4 * g;
    }
  }
};

// Route the pooled gradient to this wave's conv row (band row wr, parity HODD) and hand each
// (i, j) fragment's 4 channel sums to f(i, j, gq).  The reads of fragment u+1 are in flight while
// fragment u is consumed.
// NDP: staged dp rows (the idx rows follow them); [I0, I1): this wave's pixel blocks (f gets the
// block's index relative to I0 first)
template <bool HODD, int NDP = 3, int I0 = 0, int I1 = kPB, class F>
__device__ __forceinline__ void route_row(uint32_t pst, const RouteOffs& ro, int wr, int lane,
                                          F&& f) {
  const int m = lane & 15;
  const uint32_t dpr0 = pst + (wr >> 1) * kDpRow, dpr1 = pst + ((wr + 1) >> 1) * kDpRow;
  const uint32_t ixr0 = pst + NDP * kDpRow + (wr >> 1) * kIxRow;
  const uint32_t ixr1 = pst + NDP * kDpRow + ((wr + 1) >> 1) * kIxRow;
  const uint32_t wodd = m & 1;
  const uint32_t t00 = 3 * (HODD ? 2 : 1) + wodd + 1, t01 = 3 * (HODD ? 2 : 1);
  const uint32_t t10 = wodd + 1, t11 = 0;
  constexpr int NW = HODD ? 4 : 2;  // windows per pixel: (a0,b0), (a0,b1) [, (a1,b0), (a1,b1)]
  struct Blk {
    u32x2 d[NW];
    uint32_t x[NW];
  };
  auto load = [&](Blk& k, int u) {
    const int i = u >> 2, j = u & 3;
    k.d[0] = ld64(dpr0 + i * 1024 + ro.d0[j]);
    k.x[0] = ld32(ixr0 + i * 512 + ro.x0[j]);
    k.d[1] = ld64(dpr0 + i * 1024 + ro.d1[j]);
    k.x[1] = ld32(ixr0 + i * 512 + ro.x1[j]);
    if constexpr (HODD) {
      k.d[2] = ld64(dpr1 + i * 1024 + ro.d0[j]);
      k.x[2] = ld32(ixr1 + i * 512 + ro.x0[j]);
      k.d[3] = ld64(dpr1 + i * 1024 + ro.d1[j]);
      k.x[3] = ld32(ixr1 + i * 512 + ro.x1[j]);
    }
  };
  auto add = [](float (&gq)[4], u32x2 d, uint32_t ix, uint32_t tap, bool on) {
    const float dv[4] = {__uint_as_float(d[0] << 16), __uint_as_float(d[0] & 0xffff0000u),
                         __uint_as_float(d[1] << 16), __uint_as_float(d[1] & 0xffff0000u)};
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (on && ((ix >> (8 * q)) & 0xffu) == tap) gq[q] += dv[q];
  };
  Blk blk[2];
  load(blk[0], 4 * I0);
#pragma unroll
  for (int u = 4 * I0; u < 4 * I1; ++u) {
    if (u + 1 < 4 * I1) {
      load(blk[(u + 1) & 1], u + 1);
      wait_lgkm<2 * NW>();  // fragment u's reads landed, u+1's in flight
    } else {
      wait_lgkm<0>();
    }
    const Blk& k = blk[u & 1];
    const int i = u >> 2;
    // odd pixels take the right window too; pixel 111's right window is outside the image
    const bool on1 = wodd && !(i == kPB - 1 && m == 15);
    float gq[4] = {0.f, 0.f, 0.f, 0.f};
    add(gq, k.d[0], k.x[0], t00, true);
    add(gq, k.d[1], k.x[1], t01, on1);
    if constexpr (HODD) {
      add(gq, k.d[2], k.x[2], t10, true);
      add(gq, k.d[3], k.x[3], t11, on1);
    }
    f(i - I0, i, u & 3, gq);
  }
}

// byte address of this lane's 4 channels (16j + 4grp ..) of band pixel k in the MC image
__device__ __forceinline__ uint32_t img_off(uint32_t k, int j, int grp) {
  return mc_off<64>(k, (uint32_t)(2 * j + (grp >> 1))) + 8 * (grp & 1);
}

// g of band bb (conv rows 4bb..4bb+3) by SCATTER: every pooled (row, col, channel) of the three
// staged pooled rows adds its gradient to its argmax pixel, if that pixel is in the band, in the
// bf16 g image (zeroed before).  Windows of pooled rows / columns of equal parity are disjoint,
// so four parity phases (barrier between) need no atomics and sum each pixel in a fixed order.
// ~1/4 of the gather's VALU: one visit per pooled element instead of up to four window tests
// per conv pixel and channel (but not faster end to end: see stem_bwd_wgrad).
__device__ __forceinline__ void scatter_band(uint32_t pst, uint32_t img, int bb, int tid) {
  const int hb = 4 * bb;
#pragma unroll 1
  for (int phase = 0; phase < 4; ++phase) {
    const int pr = phase >> 1, pc = phase & 1;
    const int count = (pr == 0 ? 2 : 1) * 28 * 16;  // (staged rows) x (cols of parity pc) x quads
#pragma unroll 1
    for (int t = tid; t < count; t += 256) {
      const int ri = t / (28 * 16), rem = t - ri * (28 * 16);
      const int wo = 2 * (rem >> 4) + pc, cq = rem & 15;
      const int r3 = pr == 0 ? 2 * ri : 1;  // staged pooled row (pooled row 2bb + r3)
      const int po = 2 * bb + r3;
      const uint32_t adp = pst + (uint32_t)(r3 * kDpRow + wo * 128) +
                           ((uint32_t)((cq >> 1) ^ (((wo >> 1) & 3) << 1)) << 4) + (cq & 1) * 8;
      const uint32_t aix = pst + (uint32_t)(3 * kDpRow + r3 * kIxRow + wo * 64) +
                           ((uint32_t)((cq >> 2) ^ ((wo >> 2) & 1)) << 4) + (cq & 3) * 4;
      const u32x2 d = ld64(adp);
      const uint32_t x = ld32(aix);
      wait_lgkm<0>();
      uint32_t addr[4], old[4];
      bool ok[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int tap = (int)((x >> (8 * q)) & 0xffu);
        const int th = (tap * 11) >> 5;  // tap / 3 for tap < 9
        const int h = 2 * po - 1 + th, w = 2 * wo - 1 + (tap - 3 * th);
        ok[q] = tap < 9 && h >= hb && h < hb + 4 && w >= 0 && w < kWo;
        const int ch = 4 * cq + q;
        const uint32_t k = (uint32_t)((h - hb) * kWo + w);
        addr[q] = img + img_off(ok[q] ? k : 0u, ch >> 4, (ch >> 2) & 3) + 2 * (ch & 3);
        old[q] = 0u;
        if (ok[q]) old[q] = ld16(addr[q]);
      }
      wait_lgkm<0>();
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float dv = __uint_as_float((q & 1) ? (d[q >> 1] & 0xffff0000u) : (d[q >> 1] << 16));
        const float v = __uint_as_float(old[q] << 16) + dv;
        if (ok[q]) st16(addr[q], (uint32_t)__builtin_bit_cast(unsigned short, f2bf(v)));
      }
    }
    lds_barrier_raw();
  }
}

// Per band (4 conv rows of one image, one per wave): y of the wave's row arrives in registers
// (loaded one band ahead), g is routed from the staged pooled rows, dy = bf16(A·g + B·y + C) goes
// into an MC image [448 band pixels][64 co]; then dW[co][k] += Σ_px dy[px][co] · X[px][k] over the
// band's 448 pixels: A = dy (transposed reads of the image), B = the packed input patch
// (transposed reads: a 16-column block of k is two taps x 8 channels, each lane supplying its own
// tap's pixel address).  Wave w owns k-column blocks w, w+4, w+8, w+12 (< 14) for all 64
// channels.  Partial dW per block -> workspace slice blockIdx.x (fixed-order sum afterwards).
constexpr int kImg = 4 * kWo * 128;  // band image: 448 px x 64 co bf16 (57,344 B)
template <bool SCATTER>  // g by scatter_band (opt-in) or by the per-pixel gather route_row
__global__ __launch_bounds__(256, 1) void stem_bwd_wgrad_kernel(
    Geo g, PoolGrad pg, const __bf16* __restrict__ y, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ sum_g, const float* __restrict__ sum_gx, float inv_n,
    float* __restrict__ ws, bool nty) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kPatchB + kPoolStage + kImg + 3 * kCo * 4];
  char* pst = smem + 2 * kPatchB;
  char* gim = pst + kPoolStage;
  float* abc = reinterpret_cast<float*>(gim + kImg);  // [3][64]: A, B, C of dy = A·g + B·y + C
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int bands_per_img = g.Ho / kRB, nb = g.N * bands_per_img;
  if (tid < kCo) {  // dy = A*g + B*y + C per channel (pool_bn_bwd_apply / bn.hip)
    const int c = tid;
    const float is = invstd[c], a = gamma[c] * is;
    const float k1 = sum_g[c] * inv_n, k2 = sum_gx[c] * inv_n;
    abc[c] = a;
    abc[kCo + c] = -a * is * k2;
    abc[2 * kCo + c] = -a * k1 + a * is * k2 * mean[c];
  }
  constexpr int NKB = 4;  // k-column blocks per wave (the 14 blocks dealt round-robin)
  f32x4 wacc[4][NKB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < NKB; ++t) wacc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // y of this wave's conv row of band bnd: 7 x 4 fragments of 4 channels (8 B per lane each)
  u32x2 yv[kPB][4];
  auto load_y = [&](int bnd) {
    const int n = bnd / bands_per_img, h = (bnd % bands_per_img) * kRB + wave;
    const __bf16* yr = y + (((long)n * g.Ho + h) * kWo + (lane & 15)) * kCo + 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < kPB; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        yv[i][j] = nty ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(yr + 16 * i * kCo + 16 * j))
                       : *reinterpret_cast<const u32x2*>(yr + 16 * i * kCo + 16 * j);
  };
  __syncthreads();
  int b = blockIdx.x;
  if (b < nb) {
    load_y(b);
    stage_patch(smem, g, b / bands_per_img, (b % bands_per_img) * kRB, wave, lane);
    stage_pooled(pst, pg, b / bands_per_img, b % bands_per_img, wave, lane);
  }
  int cur = 0;
  const uint32_t img = lds_u32(gim);
  for (; b < nb; b += gridDim.x) {
    // per-lane offsets are rebuilt from an opaque copy of the lane id each band, so the compiler
    // cannot hoist them all out of the loop (register pressure)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int grp = ln >> 4, qq = (ln & 15) >> 2, p = ln & 3;
    const int nxt = b + (int)gridDim.x;
    wait_vmcnt<0>();
    lds_barrier_raw();  // y, patch and pooled rows of band b landed; band b - grid's reads done
    u32x2 yc[kPB][4];
#pragma unroll
    for (int i = 0; i < kPB; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) yc[i][j] = yv[i][j];
    if (nxt < nb) {  // next band's y and patch stream in under this band's work
      load_y(nxt);
      stage_patch(smem + (cur ^ 1) * kPatchB, g, nxt / bands_per_img, (nxt % bands_per_img) * kRB,
                  wave, ln);
    }
    const uint32_t patch = lds_u32(smem + cur * kPatchB);
    {
      u32x4 A[4], Bc[4], Cc[4];  // asm reads: a C++ LDS read would wait for the prefetches
      const uint32_t ab = lds_u32(abc) + 16 * grp;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        A[j] = ldk128(ab + 64 * j);
        Bc[j] = ldk128(ab + 4 * kCo + 64 * j);
        Cc[j] = ldk128(ab + 8 * kCo + 64 * j);
      }
      wait_lgkm<0>();
      const uint32_t k0 = (uint32_t)(wave * kWo + (ln & 15));
      auto mkdy = [&](int, int i, int j, const float (&gq)[4]) {
        const float a4[4] = {__uint_as_float(A[j][0]), __uint_as_float(A[j][1]),
                             __uint_as_float(A[j][2]), __uint_as_float(A[j][3])};
        const float b4[4] = {__uint_as_float(Bc[j][0]), __uint_as_float(Bc[j][1]),
                             __uint_as_float(Bc[j][2]), __uint_as_float(Bc[j][3])};
        const float c4[4] = {__uint_as_float(Cc[j][0]), __uint_as_float(Cc[j][1]),
                             __uint_as_float(Cc[j][2]), __uint_as_float(Cc[j][3])};
        const float yq[4] = {__uint_as_float(yc[i][j][0] << 16), __uint_as_float(yc[i][j][0] & 0xffff0000u),
                             __uint_as_float(yc[i][j][1] << 16), __uint_as_float(yc[i][j][1] & 0xffff0000u)};
        float d[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = a4[q] * bfr(gq[q]) + b4[q] * yq[q] + c4[q];
        st64(img + img_off(k0 + 16 * i, j, grp), pack2(d[0], d[1]), pack2(d[2], d[3]));
      };
      if constexpr (SCATTER) {
#pragma unroll 1
        for (int c = tid; c < kImg / 16; c += 256) st128(img + 16 * c, u32x4{0u, 0u, 0u, 0u});
        lds_barrier_raw();
        scatter_band(lds_u32(pst), img, b % bands_per_img, tid);
        // dy = A·g + B·y + C in place: each lane rewrites exactly the 8 bytes it reads
#pragma unroll
        for (int i = 0; i < kPB; ++i) {
          u32x2 gv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) gv[j] = ld64(img + img_off(k0 + 16 * i, j, grp));
          wait_lgkm<0>();
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float gq[4] = {__uint_as_float(gv[j][0] << 16),
                                 __uint_as_float(gv[j][0] & 0xffff0000u),
                                 __uint_as_float(gv[j][1] << 16),
                                 __uint_as_float(gv[j][1] & 0xffff0000u)};
            mkdy(i, i, j, gq);
          }
        }
      } else {
        RouteOffs ro;
        ro.init(ln);
        if (wave & 1) route_row<true>(lds_u32(pst), ro, wave, ln, mkdy);
        else route_row<false>(lds_u32(pst), ro, wave, ln, mkdy);
      }
    }
    lds_barrier_raw();  // the band's dy image is complete; every wave is done with the pooled rows
    if (nxt < nb) stage_pooled(pst, pg, nxt / bands_per_img, nxt % bands_per_img, wave, ln);
    {
      // dy image transposed reads: row k0 = ks*32 + 8grp + qq (swizzle independent of ks)
      uint32_t dyr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        dyr[i] = img + mc_off<64>((uint32_t)(8 * grp + qq), (uint32_t)(2 * i + (p >> 1))) + 8 * (p & 1);
      uint32_t toff[NKB];
#pragma unroll
      for (int t = 0; t < NKB; ++t) {
        const int kb = wave + 4 * t;
        const int tap = 2 * (kb < 14 ? kb : 0) + (p >> 1);
        toff[t] = (uint32_t)(((tap >> 2) * kWsp + (tap & 3)) * 16 + 8 * (p & 1));
      }
      // A (dy) and B (x) fragments of k-step ks; A of ks+1 is in flight under ks's MFMAs and B
      // of ks+1 is issued right after (at most 15 LDS reads outstanding)
      auto issue_a = [&](bf16x8 (&af)[4], int ks) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i] = join(tr_read(dyr[i] + ks * 32 * 128), tr_read(dyr[i] + ks * 32 * 128 + 4 * 128));
      };
      auto issue_b = [&](bf16x8 (&bf)[NKB], int ks) {
        const int K0 = ks * 32 + 8 * grp + qq, K1 = K0 + 4;
        const int r0 = K0 / kWo, w0 = K0 - r0 * kWo;
        const int r1 = K1 / kWo, w1 = K1 - r1 * kWo;
        const uint32_t pb0 = patch + (uint32_t)(((2 * r0) * kWsp + w0) * 16);
        const uint32_t pb1 = patch + (uint32_t)(((2 * r1) * kWsp + w1) * 16);
#pragma unroll
        for (int t = 0; t < NKB; ++t) bf[t] = join(tr_read(pb0 + toff[t]), tr_read(pb1 + toff[t]));
      };
      bf16x8 af[2][4], bfv[2][NKB];
      issue_a(af[0], 0);
      issue_b(bfv[0], 0);
#pragma unroll 2
      for (int ks = 0; ks < 14; ++ks) {
        const int s = ks & 1;
        if (ks + 1 < 14) {
          issue_a(af[s ^ 1], ks + 1);
          wait_lgkm<8>();  // A and B of ks landed
          issue_b(bfv[s ^ 1], ks + 1);
        } else {
          wait_lgkm<0>();
        }
#pragma unroll
        for (int t = 0; t < NKB; ++t) {
          if (wave + 4 * t >= 14) continue;  // wave-uniform
#pragma unroll
          for (int i = 0; i < 4; ++i)
            wacc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfv[s][t], af[s][i], wacc[i][t], 0, 0, 0);
        }
      }
      wait_lgkm<0>();
    }
    lds_barrier_raw();  // every wave is done with the image and the patch
    cur ^= 1;
  }
  // partial dW -> ws[blockIdx.x][64][224]: lane holds C[co = 16i + (lane&15)][k = 16kb + 4(lane>>4) + q]
  float* o = ws + (long)blockIdx.x * (kCo * 224);
#pragma unroll
  for (int t = 0; t < NKB; ++t) {
    const int kb = wave + 4 * t;
    if (kb >= 14) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = 16 * i + (lane & 15);
      *reinterpret_cast<float4*>(o + co * 224 + 16 * kb + 4 * (lane >> 4)) =
          make_float4(wacc[i][t][0], wacc[i][t][1], wacc[i][t][2], wacc[i][t][3]);
    }
  }
}


// ---- half bands: 2 conv rows per band, TWO blocks per CU -------------------------------------
// The 4-row kernel above holds 138 KB of LDS and runs one wave per SIMD, so a band's VALU routing
// and its weight-grad MFMAs never overlap (469 us for ResNet-50 b256).  A half band (conv rows
// 2t, 2t+1 of one image) needs 9 packed input rows (16.6 KB), 2 pooled rows (21 KB) and a 224-px
// dy image (28 KB): 73 KB, so two blocks share a CU and one's routing runs beside the other's
// MFMAs.  Waves: band row wr = wave >> 1, pixel blocks [0, 4) (even waves) or [4, 7) (odd).
// Single LDS buffers, each refilled right after its last read in the band: pooled rows after
// the routing, the patch after the MFMAs; y (registers) one band ahead.
constexpr int kRBh = 2;                    // conv rows per half band
constexpr int kPatchBH = 20 * 1024;        // 9 x 1840 = 16,560 B of packed rows (5 loads per wave)
constexpr int kPoolStageH = 24 * 1024;     // 2 dp rows (14 KiB) + 2 idx rows (7 KiB), 6 per wave
constexpr int kImgH = kRBh * kWo * 128;    // 224 px x 64 co bf16

__device__ __forceinline__ void stage_patch_half(char* pb, const Geo& g, int n, int ho0, int wave,
                                                 int lane) {
  const auto r = buf_rsrc(g.xp, g.xp_bytes);
  const uint32_t v = (uint32_t)((n * g.Hp + 2 * ho0) * kRowB + wave * 5 * 1024 + lane * 16);
#pragma unroll
  for (int i = 0; i < 5; ++i) buf_lds16(r, pb + (wave * 5 + i) * 1024, v + i * 1024);
}

// pooled rows t, t+1 of image n (dp: loads 0..13, idx: 14..20; rows past the image read zeros)
__device__ __forceinline__ void stage_pooled_half(char* buf, const PoolGrad& pg, int n, int t,
                                                  int wave, int lane) {
  const auto rd = buf_rsrc(reinterpret_cast<const char*>(pg.dp) + (long)n * pg.Hpo * kDpRow,
                           (uint32_t)(pg.Hpo * kDpRow));
  const auto ri = buf_rsrc(pg.idx + (long)n * pg.Hpo * kIxRow, (uint32_t)(pg.Hpo * kIxRow));
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int u = wave * 6 + k;  // wave-uniform
    if (u < 14) {
      const uint32_t p = (uint32_t)(u * 1024 + lane * 16);
      const uint32_t r2 = p / kDpRow, q = p - r2 * kDpRow;
      const uint32_t wo = q >> 7, ch = ((q >> 4) & 7) ^ (((wo >> 1) & 3) << 1);
      buf_lds16(rd, buf + u * 1024, (uint32_t)((t + r2) * kDpRow) + wo * 128 + ch * 16);
    } else if (u < 21) {
      const uint32_t p = (uint32_t)((u - 14) * 1024 + lane * 16);
      const uint32_t r2 = p / kIxRow, q = p - r2 * kIxRow;
      const uint32_t wo = q >> 6, ch = ((q >> 4) & 3) ^ ((wo >> 2) & 1);
      buf_lds16(ri, buf + u * 1024, (uint32_t)((t + r2) * kIxRow) + wo * 64 + ch * 16);
    }
  }
}

__global__ __launch_bounds__(256, 2) void stem_bwd_wgrad_half_kernel(
    Geo g, PoolGrad pg, const __bf16* __restrict__ y, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ sum_g, const float* __restrict__ sum_gx, float inv_n,
    float* __restrict__ ws, bool nty) {
  __shared__ __attribute__((aligned(16))) char smem[kPatchBH + kPoolStageH + kImgH + 3 * kCo * 4];
  char* pst = smem + kPatchBH;
  char* gim = pst + kPoolStageH;
  float* abc = reinterpret_cast<float*>(gim + kImgH);
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int wr = wave >> 1, hp = wave & 1;  // band row, pixel-block half
  const int hb_per_img = g.Ho / kRBh, nb = g.N * hb_per_img;
  if (tid < kCo) {
    const int c = tid;
    const float is = invstd[c], a = gamma[c] * is;
    const float k1 = sum_g[c] * inv_n, k2 = sum_gx[c] * inv_n;
    abc[c] = a;
    abc[kCo + c] = -a * is * k2;
    abc[2 * kCo + c] = -a * k1 + a * is * k2 * mean[c];
  }
  constexpr int NKB = 4;
  f32x4 wacc[4][NKB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < NKB; ++t) wacc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // y of this wave's half row: 4 pixel blocks (the odd half's 4th re-reads block 6: every wave
  // issues the same 16 loads)
  u32x2 yv[4][4];
  auto load_y = [&](int bnd) {
    const int n = bnd / hb_per_img, h = (bnd % hb_per_img) * kRBh + wr;
    const __bf16* yr = y + (((long)n * g.Ho + h) * kWo + (lane & 15)) * kCo + 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ig = min(4 * hp + i, kPB - 1);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        yv[i][j] = nty ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(yr + 16 * ig * kCo + 16 * j))
                       : *reinterpret_cast<const u32x2*>(yr + 16 * ig * kCo + 16 * j);
    }
  };
  __syncthreads();
  int b = blockIdx.x;
  // issue order per band, kept by the loop: y (16 loads), pooled rows (<= 6), patch (5) — so
  // the routing waits for y and the pooled rows only (vmcnt 5: the patch may still fly) and the
  // MFMAs for the patch (vmcnt 16: only the next band's y, issued after it, may still fly)
  if (b < nb) {
    load_y(b);
    stage_pooled_half(pst, pg, b / hb_per_img, b % hb_per_img, wave, lane);
    stage_patch_half(smem, g, b / hb_per_img, (b % hb_per_img) * kRBh, wave, lane);
  }
  const uint32_t img = lds_u32(gim);
  for (; b < nb; b += gridDim.x) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int grp = ln >> 4, qq = (ln & 15) >> 2, p = ln & 3;
    const int nxt = b + (int)gridDim.x;
    wait_vmcnt<5>();
    lds_barrier_raw();  // y and pooled rows of band b landed (every wave's)
    u32x2 yc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) yc[i][j] = yv[i][j];
    if (nxt < nb) load_y(nxt);
    const uint32_t patch = lds_u32(smem);
    {
      u32x4 A[4], Bc[4], Cc[4];
      const uint32_t ab = lds_u32(abc) + 16 * grp;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        A[j] = ldk128(ab + 64 * j);
        Bc[j] = ldk128(ab + 4 * kCo + 64 * j);
        Cc[j] = ldk128(ab + 8 * kCo + 64 * j);
      }
      wait_lgkm<0>();
      const uint32_t k0 = (uint32_t)(wr * kWo + (ln & 15));
      auto mkdy = [&](int il, int i, int j, const float (&gq)[4]) {
        const float a4[4] = {__uint_as_float(A[j][0]), __uint_as_float(A[j][1]),
                             __uint_as_float(A[j][2]), __uint_as_float(A[j][3])};
        const float b4[4] = {__uint_as_float(Bc[j][0]), __uint_as_float(Bc[j][1]),
                             __uint_as_float(Bc[j][2]), __uint_as_float(Bc[j][3])};
        const float c4[4] = {__uint_as_float(Cc[j][0]), __uint_as_float(Cc[j][1]),
                             __uint_as_float(Cc[j][2]), __uint_as_float(Cc[j][3])};
        const float yq[4] = {__uint_as_float(yc[il][j][0] << 16), __uint_as_float(yc[il][j][0] & 0xffff0000u),
                             __uint_as_float(yc[il][j][1] << 16), __uint_as_float(yc[il][j][1] & 0xffff0000u)};
        float d[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = a4[q] * bfr(gq[q]) + b4[q] * yq[q] + c4[q];
        st64(img + img_off(k0 + 16 * i, j, grp), pack2(d[0], d[1]), pack2(d[2], d[3]));
      };
      RouteOffs ro;
      ro.init(ln);
      if (wr == 0) {
        if (hp == 0) route_row<false, 2, 0, 4>(lds_u32(pst), ro, 0, ln, mkdy);
        else route_row<false, 2, 4, kPB>(lds_u32(pst), ro, 0, ln, mkdy);
      } else {
        if (hp == 0) route_row<true, 2, 0, 4>(lds_u32(pst), ro, 1, ln, mkdy);
        else route_row<true, 2, 4, kPB>(lds_u32(pst), ro, 1, ln, mkdy);
      }
    }
    if (nxt < nb) wait_vmcnt<16>();
    else wait_vmcnt<0>();
    lds_barrier_raw();  // dy image complete, pooled rows consumed, band b's patch landed
    if (nxt < nb) stage_pooled_half(pst, pg, nxt / hb_per_img, nxt % hb_per_img, wave, ln);
    {
      uint32_t dyr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        dyr[i] = img + mc_off<64>((uint32_t)(8 * grp + qq), (uint32_t)(2 * i + (p >> 1))) + 8 * (p & 1);
      uint32_t toff[NKB];
#pragma unroll
      for (int t = 0; t < NKB; ++t) {
        const int kb = wave + 4 * t;
        const int tap = 2 * (kb < 14 ? kb : 0) + (p >> 1);
        toff[t] = (uint32_t)(((tap >> 2) * kWsp + (tap & 3)) * 16 + 8 * (p & 1));
      }
      auto issue_a = [&](bf16x8 (&af)[4], int ks) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i] = join(tr_read(dyr[i] + ks * 32 * 128), tr_read(dyr[i] + ks * 32 * 128 + 4 * 128));
      };
      auto issue_b = [&](bf16x8 (&bf)[NKB], int ks) {
        const int K0 = ks * 32 + 8 * grp + qq, K1 = K0 + 4;
        const int r0 = K0 / kWo, w0 = K0 - r0 * kWo;
        const int r1 = K1 / kWo, w1 = K1 - r1 * kWo;
        const uint32_t pb0 = patch + (uint32_t)(((2 * r0) * kWsp + w0) * 16);
        const uint32_t pb1 = patch + (uint32_t)(((2 * r1) * kWsp + w1) * 16);
#pragma unroll
        for (int t = 0; t < NKB; ++t) bf[t] = join(tr_read(pb0 + toff[t]), tr_read(pb1 + toff[t]));
      };
      constexpr int KS = kRBh * kWo / 32;  // 7 k-steps of 32 band pixels
      bf16x8 af[2][4], bfv[2][NKB];
      issue_a(af[0], 0);
      issue_b(bfv[0], 0);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int s = ks & 1;
        if (ks + 1 < KS) {
          issue_a(af[s ^ 1], ks + 1);
          wait_lgkm<8>();
          issue_b(bfv[s ^ 1], ks + 1);
        } else {
          wait_lgkm<0>();
        }
#pragma unroll
        for (int t = 0; t < NKB; ++t) {
          if (wave + 4 * t >= 14) continue;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            wacc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfv[s][t], af[s][i], wacc[i][t], 0, 0, 0);
        }
      }
      wait_lgkm<0>();
    }
    lds_barrier_raw();  // every wave is done with the image and the patch
    if (nxt < nb) stage_patch_half(smem, g, nxt / hb_per_img, (nxt % hb_per_img) * kRBh, wave, ln);
  }
  float* o = ws + (long)blockIdx.x * (kCo * 224);
#pragma unroll
  for (int t = 0; t < NKB; ++t) {
    const int kb = wave + 4 * t;
    if (kb >= 14) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = 16 * i + (lane & 15);
      *reinterpret_cast<float4*>(o + co * 224 + 16 * kb + 4 * (lane >> 4)) =
          make_float4(wacc[i][t][0], wacc[i][t][1], wacc[i][t][2], wacc[i][t][3]);
    }
  }
}

}  // namespace stem

// ------------------------------------------------------------------------------------ host
bool stem_fused_supported(int N, int Ho, int Wo, int Hp, int Wsp, int Co, int Hpool, int Wpool) {
  return Wo == stem::kWo && Wsp == stem::kWsp && Co == stem::kCo && Ho % stem::kRB == 0 &&
         (long)N * Hp * stem::kRowB < (1l << 31) && (long)N * Hpool * stem::kWp * stem::kCo * 2 < (1l << 31) &&
         Hp >= 2 * (Ho - 1) + 7 && Hpool == Ho / 2 && Wpool == stem::kWp && Ho % 2 == 0 && N > 0;
}

static stem::Geo stem_geo(const void* xp, const void* w, int N, int Ho, int Hp) {
  stem::Geo g;
  g.xp_bytes = (uint32_t)((long)N * Hp * stem::kRowB);
  g.xp = (const __bf16*)xp;
  g.w = (const __bf16*)w;
  g.N = N;
  g.Ho = Ho;
  g.Hp = Hp;
  return g;
}

int stem_stats_blocks(int N, int Ho) {
  return std::min(N * (Ho / stem::kRB), 256);
}

void stem_fwd_stats(const void* xp, const void* w, int N, int Ho, int Hp, const float* shift,
                    float* ssum, float* ssq, int R, int det_rows, hipStream_t st) {
  const int G = det_rows > 0 ? det_rows : stem_stats_blocks(N, Ho);
  hipLaunchKernelGGL(stem::stem_stats_kernel, dim3(G), dim3(256), 0, st, stem_geo(xp, w, N, Ho, Hp),
                     shift, ssum, ssq, R, det_rows > 0 ? 1 : 0);
}

void stem_fwd_pool(const void* xp, const void* w, int N, int Ho, int Hp, const float* scale,
                   const float* bias, void* out, uint8_t* idx, void* y, hipStream_t st) {
  hipLaunchKernelGGL(stem::stem_pool_kernel, dim3(N), dim3(256), 0, st, stem_geo(xp, w, N, Ho, Hp),
                     scale, bias, (__bf16*)out, idx, (__bf16*)y, (g_nt_store & 16) != 0);
}

// MIPIPE_STEM_HALF=0: the 4-row-band kernel (one block per CU) instead of the half-band one
static bool stem_half() {
  static const bool on = [] {
    const char* v = getenv("MIPIPE_STEM_HALF");
    return v == nullptr || atoi(v) != 0;
  }();
  return on;
}

int stem_wgrad_blocks(int N, int Ho) {
  return stem_half() ? std::min(N * (Ho / stem::kRBh), 512) : std::min(N * (Ho / stem::kRB), 256);
}

void stem_bwd_wgrad(const void* xp, const void* y, int N, int Ho, int Hp, const void* dp,
                    const uint8_t* idx, const float* mean, const float* invstd, const float* gamma,
                    const float* sum_g, const float* sum_gx, long count, float* ws, float* dw,
                    hipStream_t st) {
  stem::PoolGrad pg{(const __bf16*)dp, idx, Ho / 2};
  const int G = stem_wgrad_blocks(N, Ho);
  // MIPIPE_STEM_SCATTER=1: g by scatter_band.  Measured equal to the gather (ResNet-50 step
  // 20.949 vs 20.942 ms, same box, alternating; profiles/r4_stem_scatter_ab.txt): a quarter of
  // the routing VALU, but five more barriers and dependent LDS round trips per band at one wave
  // per SIMD.  Off by default.
  static const bool scatter = [] {
    const char* v = getenv("MIPIPE_STEM_SCATTER");
    return v != nullptr && atoi(v) != 0;
  }();
  if (stem_half())
    hipLaunchKernelGGL(stem::stem_bwd_wgrad_half_kernel, dim3(G), dim3(256), 0, st,
                       stem_geo(xp, nullptr, N, Ho, Hp), pg, (const __bf16*)y, mean, invstd, gamma,
                       sum_g, sum_gx, 1.f / (float)count, ws, (g_nt_store & 512) != 0);
  else if (scatter)
    hipLaunchKernelGGL(stem::stem_bwd_wgrad_kernel<true>, dim3(G), dim3(256), 0, st,
                       stem_geo(xp, nullptr, N, Ho, Hp), pg, (const __bf16*)y, mean, invstd, gamma,
                       sum_g, sum_gx, 1.f / (float)count, ws, (g_nt_store & 512) != 0);
  else
    hipLaunchKernelGGL(stem::stem_bwd_wgrad_kernel<false>, dim3(G), dim3(256), 0, st,
                       stem_geo(xp, nullptr, N, Ho, Hp), pg, (const __bf16*)y, mean, invstd, gamma,
                       sum_g, sum_gx, 1.f / (float)count, ws, (g_nt_store & 512) != 0);
  splitk_sum(ws, G, (long)stem::kCo * 224, dw, st);
}

}  // namespace mipipe
