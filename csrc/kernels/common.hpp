// Shared device helpers for mipipe's gfx950 (MI355X / CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include <algorithm>

namespace mipipe {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

constexpr int kWave = 64;  // CDNA wavefront width

__device__ __forceinline__ float bf2f(__bf16 v) { return (float)v; }
__device__ __forceinline__ __bf16 f2bf(float v) { return (__bf16)v; }

__device__ __forceinline__ float bf16_bits_to_f(uint16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}

// 8 consecutive fp32 (16-B aligned) as two 16-B loads.
__device__ __forceinline__ void ld_f32x8(const float* p, float* f) {
  const float4 a = reinterpret_cast<const float4*>(p)[0];
  const float4 b = reinterpret_cast<const float4*>(p)[1];
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
  f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

// Unpack 8 bf16 held in a uint4 to floats.
__device__ __forceinline__ void unpack8(const uint4& u, float* f) {
  f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
  f[4] = __uint_as_float(u.z << 16); f[5] = __uint_as_float(u.z & 0xffff0000u);
  f[6] = __uint_as_float(u.w << 16); f[7] = __uint_as_float(u.w & 0xffff0000u);
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  bf16x2 v = {(__bf16)a, (__bf16)b};
  return *reinterpret_cast<uint32_t*>(&v);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

// scalar element <-> fp32 for kernels templated on the activation dtype
__device__ __forceinline__ float to_f32(__bf16 v) { return (float)v; }
__device__ __forceinline__ float to_f32(float v) { return v; }
template <class T>
__device__ __forceinline__ T from_f32(float v) { return (T)v; }

// 8-channel vector I/O for both activation dtypes: bf16 = one 16-B access, fp32 = two.  Kernels
// templated on the element type T (bf16 mixed precision / fp32 reference precision) use these.
__device__ __forceinline__ void load8(const __bf16* p, float* f) {
  unpack8(*reinterpret_cast<const uint4*>(p), f);
}
__device__ __forceinline__ void load8(const float* p, float* f) {
  const float4 a = reinterpret_cast<const float4*>(p)[0];
  const float4 b = reinterpret_cast<const float4*>(p)[1];
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
  f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
__device__ __forceinline__ void store8(__bf16* p, const float* f) {
  *reinterpret_cast<uint4*>(p) = pack8(f);
}
__device__ __forceinline__ void store8(float* p, const float* f) {
  reinterpret_cast<float4*>(p)[0] = make_float4(f[0], f[1], f[2], f[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(f[4], f[5], f[6], f[7]);
}
// GELU (erf form, BERT's) of one value: the gelu_fwd kernel's and the GEMM epilogue's formula
__device__ __forceinline__ float gelu_erf(float v) {
  return 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
}
// store8 with an optional non-temporal (streaming) hint: activations written once and read by a
// later kernel, larger than the caches (g_nt_store)
typedef __attribute__((ext_vector_type(4))) unsigned int u32v4;
__device__ __forceinline__ void store8(__bf16* p, const float* f, bool nt) {
  const uint4 v = pack8(f);
  if (nt) __builtin_nontemporal_store(u32v4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32v4*>(p));
  else *reinterpret_cast<uint4*>(p) = v;
}
__device__ __forceinline__ void store8(float* p, const float* f, bool) { store8(p, f); }
// 8 raw elements of T held in registers (prefetched before they are needed).
template <class T>
struct Raw8 {
  uint4 v[sizeof(T) / 2];
};
template <class T>
__device__ __forceinline__ Raw8<T> ld_raw8(const T* p) {
  Raw8<T> r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 2); ++i) r.v[i] = reinterpret_cast<const uint4*>(p)[i];
  return r;
}
// ld_raw8 with an optional non-temporal (streaming) hint
template <class T>
__device__ __forceinline__ Raw8<T> ld_raw8(const T* p, bool nt) {
  if (!nt) return ld_raw8(p);
  typedef __attribute__((ext_vector_type(4))) unsigned int u4;
  Raw8<T> r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 2); ++i) {
    const u4 v = __builtin_nontemporal_load(reinterpret_cast<const u4*>(p) + i);
    r.v[i] = make_uint4(v.x, v.y, v.z, v.w);
  }
  return r;
}
__device__ __forceinline__ void unpack_raw(const Raw8<__bf16>& r, float* f) { unpack8(r.v[0], f); }
__device__ __forceinline__ void unpack_raw(const Raw8<float>& r, float* f) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    f[4 * i + 0] = __uint_as_float(r.v[i].x);
    f[4 * i + 1] = __uint_as_float(r.v[i].y);
    f[4 * i + 2] = __uint_as_float(r.v[i].z);
    f[4 * i + 3] = __uint_as_float(r.v[i].w);
  }
}

// Value as the tensor stores it (rounds to bf16 for bf16 tensors): statistics fused into a
// producing kernel must see the stored value, not the fp32 accumulator.
template <class T>
__device__ __forceinline__ float as_stored(float v) {
  if constexpr (std::is_same<T, float>::value) return v;
  else return bf2f(f2bf(v));
}

// DPP lane move within 16-lane rows (VALU only; no LDS crossbar like ds_bpermute).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, false));
}
// Sum over each 16-lane DPP row (lanes 16r .. 16r+15); every lane of the row gets the total.
// quad_perm [1,0,3,2] (xor 1), [2,3,0,1] (xor 2), then row_ror 4 and row_ror 8.
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x124>(v);
  v += dpp_f<0x128>(v);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Whole-wave sum without the LDS crossbar (each __shfl_xor step above is a ds_bpermute round
// trip): DPP within each 16-lane row, then the four row totals read lane by lane (v_readlane)
// and added in a fixed order; every lane gets the total.  All 64 lanes must be active.
__device__ __forceinline__ float wave_sum_dpp(float v) {
  const int b = __builtin_bit_cast(int, row16_sum(v));
  return (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16))) +
         (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48)));
}

// 4 bf16 held in a uint2 <-> floats (the 8-byte twins of unpack8 / pack8)
__device__ __forceinline__ void unpack4(const uint2& u, float* f) {
  f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
}
__device__ __forceinline__ uint2 pack4(const float* f) {
  return make_uint2(pack2(f[0], f[1]), pack2(f[2], f[3]));
}
__device__ __forceinline__ void unpackv(const uint4& u, float* f) { unpack8(u, f); }
__device__ __forceinline__ void unpackv(const uint2& u, float* f) { unpack4(u, f); }
template <class VT>
__device__ __forceinline__ VT packv(const float* f);
template <>
__device__ __forceinline__ uint4 packv<uint4>(const float* f) { return pack8(f); }
template <>
__device__ __forceinline__ uint2 packv<uint2>(const float* f) { return pack4(f); }

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// Fast unsigned division by a runtime constant (Granlund-Montgomery): with l = ceil(log2 d) and
// m = floor(2^32 (2^l - d) / d) + 1, n / d = (umulhi(n, m) + n) >> l, the sum taken in 64 bits.
// Exact for every 32-bit n and every d >= 1 (d = 1: l = 0, m = 1 -> n), so no d == 1 branch:
// the per-k-step operand preps run it on wave-uniform (SGPR) indices, and a branch or a VALU
// clamp there cost SALU issue slots in every conv main loop.
struct FastDiv {
  uint32_t d, m, s;
  __host__ __device__ FastDiv() : d(1), m(1), s(0) {}
  __host__ __device__ explicit FastDiv(uint32_t div) : d(div) {
    s = 0;
    while ((1ull << s) < div) ++s;
    m = (uint32_t)((((1ull << 32) * ((1ull << s) - div)) / div) + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    const uint32_t t = __umulhi(n, m);
    return (uint32_t)(((uint64_t)t + n) >> s);
  }
};

__device__ __forceinline__ uint32_t fdiv(const FastDiv& f, uint32_t n) { return f.div(n); }

// XCD-aware bijective remap of a linear workgroup id (guide §5 "XCD swizzle must be
// bijective"): consecutive logical tiles land on the same XCD (shared L2).
__device__ __forceinline__ uint32_t xcd_remap(uint32_t wg, uint32_t nwg) {
  constexpr uint32_t NX = 8;
  if (nwg < NX) return wg;
  uint32_t q = nwg / NX, r = nwg % NX;
  uint32_t x = wg % NX, l = wg / NX;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + l;
}

}  // namespace mipipe
