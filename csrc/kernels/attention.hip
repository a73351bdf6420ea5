// Fused multi-head self-attention for gfx950 (BERT-base: head_dim 64), forward + backward.
//
// Layout (no transposes anywhere): the QKV projection's output is consumed in place,
//   qkv [B*S][3*H*64] bf16 (row = token; columns q | k | v, head-major inside each),
//   o   [B*S][H*64]   bf16 (feeds the output projection GEMM directly),
//   dqkv[B*S][3*H*64] bf16 (feeds the QKV GEMM's backward directly),
//   lse [B][H][S] fp32 (natural log), mask [B][S] fp32 additive key bias (optional).
//
// Forward (flash style, online softmax, one pass over K/V): a block = 4 waves x 32 queries of
// one (batch, head).  Scores are computed SWAPPED, X = K·Qᵀ on mfma_f32_32x32x16_bf16, so a
// lane owns one query column and 16 of its keys in registers: the row max / sum need a single
// cross-half shuffle, the rescale is lane-local, and X converted to bf16 is directly the B
// operand of Oᵀ += Vᵀ·P (guide §3 "An accumulator tile as the next MFMA's operand"); Vᵀ comes
// from the row-major V tile by ds_read_b64_tr_b16 (T10).  K/V tiles (64 keys) are double-
// buffered in LDS through global_load_lds with a source-side XOR swizzle that makes both the
// ds_read_b128 row reads and the transposed reads conflict-free.
//
// Backward: a block = 4 waves x 32 keys of one (batch, head); each wave keeps its K/V slice in
// registers and dKᵀ/dVᵀ accumulators, streams 32-query tiles of Q/dO (+ lse, delta) through
// LDS, recomputes P, forms dS = P∘(dP − δ) and issues dVᵀ += dOᵀ·P, dKᵀ += Qᵀ·dS with the same
// accumulator-as-operand trick; dQ = dS·K goes through an LDS dSᵀ image and fp32 atomics.
//
// Attention-probability dropout uses a counter-based hash of (seed, b, h, q, k), recomputed in
// the backward pass (no mask tensor).
//
// Replaces torch.nn.MultiheadAttention / HF BertSelfAttention's matmul-softmax-matmul chain
// (SURVEY.md §2.5 "BASELINE config 4": softmax-attention flash-style fwd/bwd, head_dim 64).
#include "common.hpp"
#include "launchers.hpp"

namespace mipipe {
namespace attn {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) short s16x8;
constexpr int D = 64;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// 128-byte rows of 8 16-B chunks; chunk position XOR f(row) with f a bijection on every
// aligned 16 rows (row reads: conflict-free) that flips bit 2 between rows 4k and 4k+2
// (transposed reads of 4 aligned rows x 64 B: conflict-free).
__device__ __forceinline__ uint32_t swz(uint32_t r) { return (((r >> 1) & 1u) << 2) | ((r >> 2) & 3u); }
__device__ __forceinline__ uint32_t off(uint32_t r, uint32_t chunk) {
  return r * 128u + ((chunk ^ swz(r)) << 4);
}

__device__ __forceinline__ void glds16(const void* src, char* dst_wave_base) {
  __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)dst_wave_base, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* src, char* dst_wave_base) {
  __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)dst_wave_base, 4, 0, 0);
}

__device__ __forceinline__ bf16x8 ld_row(const char* img, uint32_t row, uint32_t chunk) {
  return *reinterpret_cast<const bf16x8*>(img + off(row, chunk));
}

// A operand of mfma_32x32x16 holding Tᵀ for a row-major [rows][64] tile T, with the k (row)
// order of an accumulator used as the B operand: element j of lane half h <-> tile row
// r0 + 8(j>>2) + 4h + (j&3); the lane's column is c0 + (lane & 31).
__device__ __forceinline__ bf16x8 ld_tr(const char* img, uint32_t r0, uint32_t c0, int lane) {
  const uint32_t hl = lane >> 5, li = lane & 15, q = li >> 2, p = li & 3;
  const uint32_t col = c0 + 16 * ((lane >> 4) & 1) + 4 * p;
  const uint32_t row = r0 + 4 * hl + q;
  const char* a0 = img + off(row, col >> 3) + 8 * (p & 1);
  const char* a1 = img + off(row + 8, col >> 3) + 8 * (p & 1);
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a0);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a1);
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 pack_acc(const f32x16& x, int s) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (__bf16)x[8 * s + j];
  return v;
}

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// counter-based dropout hash (murmur3 finaliser on two mixed words)
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ bool keep_elem(uint32_t seed, uint32_t row_id, uint32_t key, uint32_t thr) {
  return mix32(mix32(seed ^ (row_id * 0x9e3779b1u)) ^ (key * 0x85ebca77u + 0x27d4eb2fu)) >= thr;
}

// reg i of a 32x32 accumulator <-> row (i&3) + 8(i>>2) + 4h
__device__ __forceinline__ int acc_row(int i, int hl) { return (i & 3) + 8 * (i >> 2) + 4 * hl; }

struct FwdArgs {
  const __bf16* qkv;
  __bf16* o;
  float* lse;
  const float* mask;
  int B, S, H;
  float scale_log2;
  float p_drop;
  uint32_t drop_thr;
  uint32_t seed;
  const uint32_t* seed_dev;  // device step counter mixed into the seed (hipGraph replays), or null
};

// effective dropout seed: host seed, or host seed mixed with the device step counter (read once
// per wave through the scalar cache; the counter is advanced by a kernel before the forward)
__device__ __forceinline__ uint32_t eff_seed(uint32_t seed, const uint32_t* dev) {
  if (dev == nullptr) return seed;
  // agent-scope relaxed load: served by L2 (sc1), never by a scalar / L1 line that kernels
  // replayed back to back from a hipGraph might not have invalidated since the counter was bumped
  const uint32_t c = __hip_atomic_load(dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return mix32(seed ^ (c * 0x9e3779b1u + 0x632be5abu));
}

constexpr int kFwdTile = 16384;  // K (8 KB) + V (8 KB) for 64 keys
constexpr int kMaxS = 2048;

// NW waves per block (32 queries each): 4 (default) or 2 (see attn_waves()).
template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_fwd_kernel(FwdArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kFwdTile + kMaxS * 4];
  constexpr int QB = 32 * NW;  // queries per block
  const int S = a.S, H = a.H;
  const long ld = 3l * H * D, ldo = (long)H * D;
  const int nqt = (S + QB - 1) / QB;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);  // a head's q-tiles share an XCD's L2
  const int qt = bid % nqt, bh = bid / nqt, h = bh % H, b = bh / H;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5, r = lane & 31;
  const __bf16* qb = a.qkv + (long)b * S * ld + h * D;
  const __bf16* kb = qb + (long)H * D;
  const __bf16* vb = kb + (long)H * D;
  const int nkt = (S + 63) / 64;
  const uint32_t dseed = a.p_drop > 0.f ? eff_seed(a.seed, a.seed_dev) : a.seed;
  float* maskl = reinterpret_cast<float*>(smem + 2 * kFwdTile);
  for (int i = tid; i < nkt * 64; i += 64 * NW)
    maskl[i] = i < S ? (a.mask ? a.mask[(long)b * S + i] * kLog2e : 0.f) : -INFINITY;
  const int q = qt * QB + wave * 32 + r;
  const int qc = min(q, S - 1);
  bf16x8 qf[4];
#pragma unroll
  for (int st = 0; st < 4; ++st)
    qf[st] = *reinterpret_cast<const bf16x8*>(qb + (long)qc * ld + 16 * st + 8 * hl);

  auto stage = [&](char* buf, int k0) {  // 64 keys x 8 chunks of K and of V
#pragma unroll
    for (int i = 0; i < 8 / NW; ++i) {
      const int t = (i * NW + wave) * 64 + lane;
      const int row = t >> 3, pos = t & 7;
      const int chunk = pos ^ swz(row);
      const long key = min(k0 + row, S - 1);
      glds16(kb + key * ld + chunk * 8, buf + (i * NW + wave) * 1024);
      glds16(vb + key * ld + chunk * 8, buf + 8192 + (i * NW + wave) * 1024);
    }
  };

  stage(smem, 0);
  f32x16 o0 = zero16(), o1 = zero16();
  float m = -INFINITY, l = 0.f;
  const float inv_keep = a.p_drop > 0.f ? 1.f / (1.f - a.p_drop) : 1.f;
  const uint32_t row_id = ((uint32_t)(b * H + h)) * (uint32_t)S + (uint32_t)qc;
  for (int kt = 0; kt < nkt; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const char* cur = smem + (kt & 1) * kFwdTile;
    if (kt + 1 < nkt) stage(smem + ((kt + 1) & 1) * kFwdTile, (kt + 1) * 64);
    f32x16 s[2];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      s[sub] = zero16();
#pragma unroll
      for (int st = 0; st < 4; ++st)
        s[sub] = mfma32(ld_row(cur, sub * 32 + r, 2 * st + hl), qf[st], s[sub]);
    }
    float mt = -INFINITY;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float v = s[sub][i] * a.scale_log2 + maskl[kt * 64 + sub * 32 + acc_row(i, hl)];
        s[sub][i] = v;
        mt = fmaxf(mt, v);
      }
    mt = fmaxf(mt, __shfl_xor(mt, 32));
    const float mn = fmaxf(m, mt);
    const float mu = mn == -INFINITY ? 0.f : mn;
    const float alpha = exp2f(m - mu);
    float ls = 0.f;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = exp2f(s[sub][i] - mu);
        ls += p;
        if (a.p_drop > 0.f) {
          const uint32_t key = kt * 64 + sub * 32 + acc_row(i, hl);
          p = keep_elem(dseed, row_id, key, a.drop_thr) ? p * inv_keep : 0.f;
        }
        s[sub][i] = p;
      }
    l = l * alpha + ls;
    m = mn;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      o0[i] *= alpha;
      o1[i] *= alpha;
    }
    const char* vimg = cur + 8192;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 pf = pack_acc(s[sub], ks);
        o0 = mfma32(ld_tr(vimg, sub * 32 + 16 * ks, 0, lane), pf, o0);
        o1 = mfma32(ld_tr(vimg, sub * 32 + 16 * ks, 32, lane), pf, o1);
      }
  }
  l += __shfl_xor(l, 32);
  const float inv_l = l > 0.f ? 1.f / l : 0.f;
  if (hl == 0 && q < S) a.lse[((long)b * H + h) * S + q] = l > 0.f ? (m + __log2f(l)) * kLn2 : -INFINITY;
  // stage Oᵀ -> O rows through LDS (pitch 136 B) and store 8-byte row pieces
  __syncthreads();
  char* ow = smem + wave * (32 * 136);
#pragma unroll
  for (int ig = 0; ig < 4; ++ig) {
    const int d0 = 8 * ig + 4 * hl;
    uint2 v0 = make_uint2(pack2(o0[4 * ig] * inv_l, o0[4 * ig + 1] * inv_l),
                          pack2(o0[4 * ig + 2] * inv_l, o0[4 * ig + 3] * inv_l));
    uint2 v1 = make_uint2(pack2(o1[4 * ig] * inv_l, o1[4 * ig + 1] * inv_l),
                          pack2(o1[4 * ig + 2] * inv_l, o1[4 * ig + 3] * inv_l));
    *reinterpret_cast<uint2*>(ow + r * 136 + 2 * d0) = v0;
    *reinterpret_cast<uint2*>(ow + r * 136 + 2 * (32 + d0)) = v1;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int row = it * 4 + (lane >> 4), piece = lane & 15;
    const int qq = qt * QB + wave * 32 + row;
    if (qq < S) {
      uint2 v = *reinterpret_cast<const uint2*>(ow + row * 136 + piece * 8);
      *reinterpret_cast<uint2*>(a.o + ((long)b * S + qq) * ldo + h * D + piece * 4) = v;
    }
  }
}

// δ[b,h,q] = Σ_d dO·O  (one thread per (token, head)); also zeroes that (token, head)'s 64
// fp32 dQ accumulators (the backward kernel adds into them) — no separate memset
// δ[b][h][q] = Σ_d dO·O over the head's 64 values, and the fp32 dQ accumulator zeroed.  Eight
// lanes per (token, head) — one 16-byte chunk each, summed across the 8 lanes with xor shuffles
// (fixed order) — so loads and stores are contiguous across a wave and the grid has 8x the
// blocks of a thread-per-row mapping (192 blocks at BERT-base 32x128: under one per CU).
__global__ __launch_bounds__(256) void attn_delta_kernel(const __bf16* __restrict__ dout,
                                                         const __bf16* __restrict__ o,
                                                         float* __restrict__ delta,
                                                         float* __restrict__ dq_acc, int B, int S,
                                                         int H, bool zero_dq) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long row = gid >> 3;  // (token, head); rows * 8 is a multiple of 8: groups stay whole
  const int c = (int)(gid & 7);
  if (row >= (long)B * S * H) return;
  const int h = (int)(row % H);
  const long tok = row / H;
  const int b = (int)(tok / S), q = (int)(tok % S);
  const long off = tok * H * D + h * D + c * 8;
  float x[8], y[8];
  unpack8(*reinterpret_cast<const uint4*>(dout + off), x);
  unpack8(*reinterpret_cast<const uint4*>(o + off), y);
  float acc = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) acc += x[e] * y[e];
  acc += __shfl_xor(acc, 1);
  acc += __shfl_xor(acc, 2);
  acc += __shfl_xor(acc, 4);
  if (c == 0) delta[((long)b * H + h) * S + q] = acc;
  if (!zero_dq) return;
  float4* dq = reinterpret_cast<float4*>(dq_acc + off);
  dq[0] = make_float4(0.f, 0.f, 0.f, 0.f);
  dq[1] = make_float4(0.f, 0.f, 0.f, 0.f);
}

struct BwdArgs {
  const __bf16* qkv;
  const __bf16* dout;
  const float* lse;    // [B][H][S]
  const float* delta;  // [B][H][S]
  const float* mask;
  float* dq_acc;       // [B*S][H*64] fp32, zeroed; det: [nkb][B*S][H*64] slabs, written
  __bf16* dqkv;
  int det;             // deterministic mode: each key block STORES its dQ part in its own slab
  int direct;          // one key block per (b, h): its dQ tiles are complete -> bf16 into dqkv
  int B, S, H;
  float scale, scale_log2;
  float p_drop;
  uint32_t drop_thr;
  uint32_t seed;
  const uint32_t* seed_dev;
};

// LDS: K tile (KB keys) | 2 x {Q 4 KB, dO 4 KB, lse 128 B, delta 128 B} | dSᵀ [KB][32] bf16
constexpr int kQStage = 8192 + 256;

// NW waves per block (32 keys each; 4 by default, as in the forward)
template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_bwd_kernel(BwdArgs a) {
  constexpr int KB = 32 * NW;  // keys per block
  constexpr int kKT = KB * 128;
  constexpr int kDsOff = kKT + 2 * kQStage;
  constexpr int kDqOff = kDsOff + KB * 64;  // direct mode: finished dQ tile [32 q][64 d] bf16
  __shared__ __attribute__((aligned(16))) char smem[kDqOff + 32 * 128];
  const int S = a.S, H = a.H;
  const long ld = 3l * H * D, ldq = (long)H * D;
  const int nkb = (S + KB - 1) / KB;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int kbk = bid % nkb, bh = bid / nkb, h = bh % H, b = bh / H;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5, r = lane & 31;
  const __bf16* qb = a.qkv + (long)b * S * ld + h * D;
  const __bf16* kb = qb + (long)H * D;
  const __bf16* vb = kb + (long)H * D;
  const __bf16* dob = a.dout + (long)b * S * ldq + h * D;
  const uint32_t dseed = a.p_drop > 0.f ? eff_seed(a.seed, a.seed_dev) : a.seed;
  const float* lseb = a.lse + ((long)b * H + h) * S;
  const float* delb = a.delta + ((long)b * H + h) * S;
  const int key = kbk * KB + wave * 32 + r;
  const int kc = min(key, S - 1);
  // this lane's key: K and V rows as B operands, its mask bias
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    kf[st] = *reinterpret_cast<const bf16x8*>(kb + (long)kc * ld + 16 * st + 8 * hl);
    vf[st] = *reinterpret_cast<const bf16x8*>(vb + (long)kc * ld + 16 * st + 8 * hl);
  }
  const float mk = key < S ? (a.mask ? a.mask[(long)b * S + key] * kLog2e : 0.f) : -INFINITY;
  // K tile [KB keys][64] for the dQ product (4 glds per thread)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = (i * NW + wave) * 64 + lane;
    const int row = t >> 3, pos = t & 7;
    const long kk = min(kbk * KB + row, S - 1);
    glds16(kb + kk * ld + ((pos ^ swz(row)) * 8), smem + (i * NW + wave) * 1024);
  }
  const int nqt = (S + 31) / 32;
  auto stage = [&](char* buf, int q0) {
#pragma unroll
    for (int i = 0; i < 4 / NW; ++i) {  // 256 chunks of 16 B per 32x64 tile
      const int t = (i * NW + wave) * 64 + lane;
      const int row = t >> 3, pos = t & 7;
      const long qq = min(q0 + row, S - 1);
      glds16(qb + qq * ld + ((pos ^ swz(row)) * 8), buf + (i * NW + wave) * 1024);
      glds16(dob + qq * ldq + ((pos ^ swz(row)) * 8), buf + 4096 + (i * NW + wave) * 1024);
    }
    if (wave == 0) {
      const int qi = min(q0 + (lane & 31), S - 1);
      glds4(lane < 32 ? lseb + qi : delb + qi, buf + 8192);
    }
  };
  stage(smem + kKT, 0);
  f32x16 dk0 = zero16(), dk1 = zero16(), dv0 = zero16(), dv1 = zero16();
  const float inv_keep = a.p_drop > 0.f ? 1.f / (1.f - a.p_drop) : 1.f;
  char* dsT = smem + kDsOff;
  // direct mode: the finished 32 x 64 bf16 dQ tile of q tile t, 256 chunks of 16 B, from LDS to
  // dqkv.  Tile t is written to LDS in iteration t and stored after the next barrier (the top of
  // iteration t + 1, or after the loop); every wave reads it before the mid-iteration barrier
  // that precedes the next rewrite.
  auto store_dq = [&](int t) {
#pragma unroll
    for (int c = tid; c < 256; c += 64 * NW) {
      const int row = c >> 3, qg = t * 32 + row;
      const uint4 v = *reinterpret_cast<const uint4*>(smem + kDqOff + 16 * c);
      if (qg < S)
        *reinterpret_cast<uint4*>(a.dqkv + ((long)b * S + qg) * ld + h * D + 8 * (c & 7)) = v;
    }
  };
  for (int it = 0; it < nqt; ++it) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const char* cur = smem + kKT + (it & 1) * kQStage;
    if (it + 1 < nqt) stage(smem + kKT + ((it + 1) & 1) * kQStage, (it + 1) * 32);
    if (a.direct && it > 0) store_dq(it - 1);
    const float* lsel = reinterpret_cast<const float*>(cur + 8192);
    const float* dell = lsel + 32;
    // X = S[q][key] (rows q, lane = key) and dP = dO·Vᵀ in the same layout
    f32x16 s = zero16(), dp = zero16();
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      s = mfma32(ld_row(cur, r, 2 * st + hl), kf[st], s);
      dp = mfma32(ld_row(cur + 4096, r, 2 * st + hl), vf[st], dp);
    }
    f32x16 pd, ds;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qi = acc_row(i, hl);
      const float p = exp2f(s[i] * a.scale_log2 + mk - lsel[qi] * kLog2e);
      float pdrop = p, dpv = dp[i];
      if (a.p_drop > 0.f) {
        const uint32_t row_id = ((uint32_t)(b * H + h)) * (uint32_t)S + (uint32_t)min(it * 32 + qi, S - 1);
        const bool kp = keep_elem(dseed, row_id, (uint32_t)key, a.drop_thr);
        pdrop = kp ? p * inv_keep : 0.f;
        dpv = kp ? dpv * inv_keep : 0.f;
      }
      const bool valid = (it * 32 + qi) < S;
      pd[i] = valid ? pdrop : 0.f;
      ds[i] = valid ? p * (dpv - dell[qi]) * a.scale : 0.f;
    }
    // dVᵀ += dOᵀ·P,  dKᵀ += Qᵀ·dS
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pf = pack_acc(pd, ks), sf = pack_acc(ds, ks);
      dv0 = mfma32(ld_tr(cur + 4096, 16 * ks, 0, lane), pf, dv0);
      dv1 = mfma32(ld_tr(cur + 4096, 16 * ks, 32, lane), pf, dv1);
      dk0 = mfma32(ld_tr(cur, 16 * ks, 0, lane), sf, dk0);
      dk1 = mfma32(ld_tr(cur, 16 * ks, 32, lane), sf, dk1);
    }
    // dSᵀ image [key 128][q 32] (64-B rows): lane writes 4 consecutive q per 8-byte store
    const int krow = wave * 32 + r;
#pragma unroll
    for (int ig = 0; ig < 4; ++ig) {
      const int q0 = 8 * ig + 4 * hl;
      *reinterpret_cast<uint2*>(dsT + krow * 64 + q0 * 2) =
          make_uint2(pack2(ds[4 * ig], ds[4 * ig + 1]), pack2(ds[4 * ig + 2], ds[4 * ig + 3]));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // raw barrier: keeps the next tile's glds in flight
    asm volatile("" ::: "memory");
    // dQ[32 q][64 d] += dS[q][KB keys]·K[keys][d]: wave -> q rows 16(w&1), d cols
    // (128/NW)(w>>1) in DT 16-column MFMA tiles
    {
      constexpr int DT = 128 / NW / 16;
      const int qr0 = 16 * (wave & 1), dc0 = (128 / NW) * (wave >> 1);
      const int g = lane >> 4, li = lane & 15, qq = li >> 2, p = li & 3;
      f32x4 cacc[DT];
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) cacc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NW; ++ks) {
        const int k0 = ks * 32 + 8 * g + qq;
        // A = dS[q][key]: transposed read of dSᵀ rows k0, k0+4, columns qr0 + 4p..
        const char* a0 = dsT + k0 * 64 + (qr0 + 4 * p) * 2;
        s16x4 alo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a0);
        s16x4 ahi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0 + 4 * 64));
        s16x8 av = {alo[0], alo[1], alo[2], alo[3], ahi[0], ahi[1], ahi[2], ahi[3]};
        const bf16x8 af = __builtin_bit_cast(bf16x8, av);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int col = dc0 + 16 * dt + 4 * p;
          const char* b0 = smem + off(k0, col >> 3) + 8 * (p & 1);
          const char* b1 = smem + off(k0 + 4, col >> 3) + 8 * (p & 1);
          s16x4 blo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)b0);
          s16x4 bhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)b1);
          s16x8 bv = {blo[0], blo[1], blo[2], blo[3], bhi[0], bhi[1], bhi[2], bhi[3]};
          const bf16x8 bfr = __builtin_bit_cast(bf16x8, bv);
          cacc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, cacc[dt], 0, 0, 0);
        }
      }
      // C: col = lane&15 (d), row = 4(lane>>4) + i (q)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qg = it * 32 + qr0 + 4 * g + i;
        if (qg < S) {
          float* dst = a.dq_acc + ((long)b * S + qg) * ldq + h * D + dc0 + li;
          if (a.direct) {
            // the block holds every key of (b, h): this is the finished dQ value -> LDS tile,
            // stored to dqkv below as whole 16-byte chunks
            __bf16* dql = reinterpret_cast<__bf16*>(smem + kDqOff) + (qr0 + 4 * g + i) * D + dc0 + li;
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) dql[16 * dt] = f2bf(cacc[dt][i]);
          } else if (a.det) {
            // deterministic: this key block's slab; every (q, d) of it is written exactly once
            // (one q tile per iteration), and attn_dq_store_kernel sums the slabs in key order
            dst += (long)kbk * a.B * S * ldq;
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) dst[16 * dt] = cacc[dt][i];
          } else {
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) atomicAdd(dst + 16 * dt, cacc[dt][i]);
          }
        }
      }
    }
  }
  if (a.direct) {  // the last q tile's dQ
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    store_dq(nqt - 1);
  }
  // dKᵀ / dVᵀ: lane = key column, regs = d rows -> 8-byte stores into dqkv's k / v columns
  if (key < S) {
    __bf16* dkp = a.dqkv + ((long)b * S + key) * ld + (long)H * D + h * D;
    __bf16* dvp = dkp + (long)H * D;
#pragma unroll
    for (int ig = 0; ig < 4; ++ig) {
      const int d0 = 8 * ig + 4 * hl;
      *reinterpret_cast<uint2*>(dkp + d0) =
          make_uint2(pack2(dk0[4 * ig], dk0[4 * ig + 1]), pack2(dk0[4 * ig + 2], dk0[4 * ig + 3]));
      *reinterpret_cast<uint2*>(dkp + 32 + d0) =
          make_uint2(pack2(dk1[4 * ig], dk1[4 * ig + 1]), pack2(dk1[4 * ig + 2], dk1[4 * ig + 3]));
      *reinterpret_cast<uint2*>(dvp + d0) =
          make_uint2(pack2(dv0[4 * ig], dv0[4 * ig + 1]), pack2(dv0[4 * ig + 2], dv0[4 * ig + 3]));
      *reinterpret_cast<uint2*>(dvp + 32 + d0) =
          make_uint2(pack2(dv1[4 * ig], dv1[4 * ig + 1]), pack2(dv1[4 * ig + 2], dv1[4 * ig + 3]));
    }
  }
}

// dq (fp32 accumulator, or `slabs` per-key-block slabs summed in key-block order) -> bf16 q
// columns of dqkv
__global__ __launch_bounds__(256) void attn_dq_store_kernel(const float* __restrict__ acc,
                                                            __bf16* __restrict__ dqkv, long T,
                                                            int HD, int slabs) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // one 8-element chunk each
  const long per_row = HD / 8;
  if (i >= T * per_row) return;
  const long t = i / per_row, c = i % per_row;
  float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int sl = 0; sl < slabs; ++sl) {
    const float4* src = reinterpret_cast<const float4*>(acc + ((long)sl * T + t) * HD + c * 8);
    const float4 x = src[0], y = src[1];
    f[0] += x.x; f[1] += x.y; f[2] += x.z; f[3] += x.w;
    f[4] += y.x; f[5] += y.y; f[6] += y.z; f[7] += y.w;
  }
  *reinterpret_cast<uint4*>(dqkv + t * 3l * HD + c * 8) = pack8(f);
}

}  // namespace attn

int g_attn_waves = 0;  // 0: default (4); 2 / 4: forced (tests, A/B)

// waves (32 rows each) per attention block.  4 by default: measured on BERT-base 8x512, the
// 2-wave blocks (twice the grid, even spread over the CUs) run the step 7 % slower — sharing
// each staged K/V (fwd) / Q-dO (bwd) tile across 4 waves matters more than occupancy
// (tools/r2/bench_attn_waves.py).
static int attn_waves(int B, int S, int H) {
  (void)B; (void)S; (void)H;
  return g_attn_waves == 2 ? 2 : 4;
}

static uint32_t drop_threshold(float p) {
  double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
}

void attention_fwd(const void* qkv, const float* mask, void* o, float* lse, int B, int S, int H,
                   float scale, float p_drop, uint32_t seed, hipStream_t st,
                   const uint32_t* seed_dev) {
  attn::FwdArgs a{(const __bf16*)qkv, (__bf16*)o, lse, mask, B, S, H, scale * attn::kLog2e,
                  p_drop, drop_threshold(p_drop), seed, seed_dev};
  if (attn_waves(B, S, H) == 2)
    hipLaunchKernelGGL(attn::attn_fwd_kernel<2>, dim3(B * H * ((S + 63) / 64)), dim3(128), 0, st, a);
  else
    hipLaunchKernelGGL(attn::attn_fwd_kernel<4>, dim3(B * H * ((S + 127) / 128)), dim3(256), 0, st, a);
}

// S within one backward key block: every dQ tile is finished inside its block and stored as bf16
// directly (no fp32 accumulator to zero, no atomics, no dq_store pass)
bool attention_dq_direct(int S) { return S <= (attn_waves(1, S, 1) == 2 ? 64 : 128); }

int attention_dq_slabs(int S) {
  if (attention_dq_direct(S)) return 0;
  if (!g_deterministic) return 1;
  const int kb = attn_waves(1, S, 1) == 2 ? 64 : 128;  // keys per backward block
  return (S + kb - 1) / kb;
}

void attention_bwd(const void* dout, const void* qkv, const void* o, const float* lse,
                   const float* mask, void* dqkv, float* delta, float* dq_acc, int B, int S,
                   int H, float scale, float p_drop, uint32_t seed, hipStream_t st,
                   const uint32_t* seed_dev) {
  const long rows = (long)B * S * H;
  // deterministic mode with several key blocks per (b, h): per-key-block dQ slabs summed in a
  // fixed order instead of fp32 atomics (one key block: its single add is already exact)
  const bool direct = attention_dq_direct(S);
  const int slabs = attention_dq_slabs(S);
  const int det = slabs > 1 ? 1 : 0;
  hipLaunchKernelGGL(attn::attn_delta_kernel, dim3((rows * 8 + 255) / 256), dim3(256), 0, st,
                     (const __bf16*)dout, (const __bf16*)o, delta, dq_acc, B, S, H, !direct);
  attn::BwdArgs a{(const __bf16*)qkv, (const __bf16*)dout, lse, delta, mask, dq_acc,
                  (__bf16*)dqkv, det, direct ? 1 : 0, B, S, H, scale, scale * attn::kLog2e,
                  p_drop, drop_threshold(p_drop), seed, seed_dev};
  if (attn_waves(B, S, H) == 2)
    hipLaunchKernelGGL(attn::attn_bwd_kernel<2>, dim3(B * H * ((S + 63) / 64)), dim3(128), 0, st, a);
  else
    hipLaunchKernelGGL(attn::attn_bwd_kernel<4>, dim3(B * H * ((S + 127) / 128)), dim3(256), 0, st, a);
  if (direct) return;
  const long chunks = (long)B * S * H * attn::D / 8;
  hipLaunchKernelGGL(attn::attn_dq_store_kernel, dim3((chunks + 255) / 256), dim3(256), 0, st,
                     dq_acc, (__bf16*)dqkv, (long)B * S, H * attn::D, det ? slabs : 1);
}

}  // namespace mipipe
