// Shared helpers for the CMX gfx950 kernels (C-ABI library libcmx_hip.so).
//
// Storage types: float (fp32 parity mode) and bf16 (performance mode); every kernel
// accumulates in fp32.  dtype codes on the C-ABI: 0 = fp32, 1 = bf16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include "../../include/cmx_hip.h"  // compiler-checks every definition against the ABI header

#define CMX_ABI_VERSION 1

enum cmx_status {
  CMX_OK = 0,
  CMX_ERR_SHAPE = -1,
  CMX_ERR_DTYPE = -2,
  CMX_ERR_LAUNCH = -3,
  CMX_ERR_ARG = -4,
};

// ---------------------------------------------------------------- error reporting
void cmx_set_error(const char* fmt, ...);
int cmx_check_launch(const char* what);

#define CMX_REQUIRE(cond, code, ...)   \
  do {                                 \
    if (!(cond)) {                     \
      cmx_set_error(__VA_ARGS__);      \
      return (code);                   \
    }                                  \
  } while (0)

// ---------------------------------------------------------------- bf16
struct bf16 {
  uint16_t x;
};

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16 v) {
  return __uint_as_float(((uint32_t)v.x) << 16);
}
template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float v) {
  // round-to-nearest-even; NaN kept NaN
  uint32_t u = __float_as_uint(v);
  bf16 r;
  if ((u & 0x7fffffffu) > 0x7f800000u) {
    r.x = (uint16_t)((u >> 16) | 0x40);
  } else {
    r.x = (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
  }
  return r;
}

// 16-byte vectors: VEC<float> = 4 elements, VEC<bf16> = 8 elements.
template <typename T> struct VecT;
template <> struct VecT<float> { static constexpr int N = 4; typedef float4 raw; };
template <> struct VecT<bf16> { static constexpr int N = 8; typedef uint4 raw; };

template <typename T>
__device__ __forceinline__ void load_vec(const T* p, float* out) {
  if constexpr (sizeof(T) == 4) {
    float4 v = *reinterpret_cast<const float4*>(p);
    out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
  } else {
    uint4 v = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      out[2 * i] = __uint_as_float(w[i] << 16);
      out[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
}

template <typename T>
__device__ __forceinline__ void store_vec(T* p, const float* in) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(in[0], in[1], in[2], in[3]);
  } else {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bf16 a = from_f32<bf16>(in[2 * i]);
      bf16 b = from_f32<bf16>(in[2 * i + 1]);
      w[i] = (uint32_t)a.x | ((uint32_t)b.x << 16);
    }
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// sum across a power-of-two group of `width` lanes (width <= 64)
__device__ __forceinline__ float group_sum(float v, int width) {
  for (int o = width >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// activation codes shared by several kernels
enum { ACT_NONE = 0, ACT_GELU = 1, ACT_RELU = 2, ACT_SIGMOID = 3 };

__device__ __forceinline__ float act_fwd(float z, int act) {
  if (act == ACT_GELU) return gelu_erf(z);
  if (act == ACT_RELU) return z > 0.f ? z : 0.f;
  if (act == ACT_SIGMOID) return 1.f / (1.f + __expf(-z));
  return z;
}
// derivative w.r.t. the pre-activation z
__device__ __forceinline__ float act_grad(float z, int act) {
  if (act == ACT_GELU) return gelu_erf_grad(z);
  if (act == ACT_RELU) return z > 0.f ? 1.f : 0.f;
  if (act == ACT_SIGMOID) { float s = 1.f / (1.f + __expf(-z)); return s * (1.f - s); }
  return 1.f;
}

static inline unsigned cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }

// dtype dispatch helper for launch wrappers
#define CMX_DISPATCH(dtype, T, ...)                                   \
  do {                                                                \
    if ((dtype) == 0) { typedef float T; __VA_ARGS__; }               \
    else if ((dtype) == 1) { typedef bf16 T; __VA_ARGS__; }           \
    else { cmx_set_error("unsupported dtype %d", (int)(dtype)); return CMX_ERR_DTYPE; } \
  } while (0)

// ws (G, nblk, W) -> out (G, W); defined in layernorm.hip, shared by all two-stage reductions
int cmx_reduce_partials(const float* ws, float* out, int G, int nblk, int W, int accumulate,
                        float alpha, hipStream_t s);
// ws (nblk, stride) columns [0, W) -> out (W)
int cmx_reduce_partials_strided(const float* ws, float* out, int nblk, int W, int stride, int accumulate,
                                hipStream_t s);
