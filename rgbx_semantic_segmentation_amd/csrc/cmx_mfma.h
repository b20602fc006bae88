// 32x32 MFMA tile traits shared by the attention-shaped kernels.
//
// One wave computes a 32x32 fp32 tile D += A(32xK) * B(Kx32).  Lane l = (r = l & 31,
// h = l >> 5) supplies A[r][E*h + j] and B[E*h + j][r] for j < E per instruction:
//   bf16: v_mfma_f32_32x32x16_bf16, KI = 16 k per instruction, E = 8 elements per lane
//   f16 : v_mfma_f32_32x32x16_f16 , the same shape and rate
//   fp32: v_mfma_f32_32x32x2_f32  , KI = 2,                    E = 1 (exact fp32)
// Accumulator register i of lane (col = l & 31, h) holds row accrow(i, h).
// An accumulator X (rows = k) can feed the next MFMA as its B operand with no data
// movement: k-step s uses registers E*s .. E*s+E-1 and element j of lane half h then
// stands for row accrow(E*s + j, h) of X, so the A operand must supply that same k.
#pragma once
#include "cmx_common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int accrow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

template <typename T> struct MF;

template <> struct MF<float> {
  static constexpr int KI = 2, E = 1;
  typedef float frag;
  __device__ static __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
  // E contiguous elements starting at p
  __device__ static __forceinline__ frag load(const float* p) { return *p; }
  __device__ static __forceinline__ frag from_acc(const f32x16& acc, int s) { return acc[s]; }
};

template <> struct MF<bf16> {
  static constexpr int KI = 16, E = 8;
  typedef bf16x8 frag;
  __device__ static __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ frag load(const bf16* p) {
    return __builtin_bit_cast(frag, *reinterpret_cast<const uint4*>(p));
  }
  // two groups of 4 contiguous elements (k-permuted operand from a transposed image)
  __device__ static __forceinline__ frag load2x4(const bf16* p0, const bf16* p1) {
    uint2 a = *reinterpret_cast<const uint2*>(p0);
    uint2 b = *reinterpret_cast<const uint2*>(p1);
    return __builtin_bit_cast(frag, make_uint4(a.x, a.y, b.x, b.y));
  }
  __device__ static __forceinline__ frag from_acc(const f32x16& acc, int s) {
    u16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = from_f32<bf16>(acc[8 * s + j]).x;
    return __builtin_bit_cast(frag, v);
  }
};

template <> struct MF<f16> {
  static constexpr int KI = 16, E = 8;
  typedef f16x8 frag;
  __device__ static __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ frag load(const f16* p) {
    return __builtin_bit_cast(frag, *reinterpret_cast<const uint4*>(p));
  }
  __device__ static __forceinline__ frag load2x4(const f16* p0, const f16* p1) {
    uint2 a = *reinterpret_cast<const uint2*>(p0);
    uint2 b = *reinterpret_cast<const uint2*>(p1);
    return __builtin_bit_cast(frag, make_uint4(a.x, a.y, b.x, b.y));
  }
  __device__ static __forceinline__ frag from_acc(const f32x16& acc, int s) {
    u16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = from_f32<f16>(acc[8 * s + j]).x;
    return __builtin_bit_cast(frag, v);
  }
};

// an 8-element fragment from raw 16-byte bits (16-bit storage types)
template <typename T> __device__ __forceinline__ typename MF<T>::frag frag_bits(uint4 u) {
  return __builtin_bit_cast(typename MF<T>::frag, u);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// zero fragment
template <typename T> __device__ __forceinline__ typename MF<T>::frag zfrag();
template <> __device__ __forceinline__ float zfrag<float>() { return 0.f; }
template <> __device__ __forceinline__ bf16x8 zfrag<bf16>() {
  return __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
}
template <> __device__ __forceinline__ f16x8 zfrag<f16>() {
  return __builtin_bit_cast(f16x8, make_uint4(0, 0, 0, 0));
}
