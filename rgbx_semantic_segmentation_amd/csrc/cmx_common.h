// Shared helpers for the CMX gfx950 kernels (C-ABI library libcmx_hip.so).
//
// Storage types: float (fp32 parity mode), bf16 (performance mode) and f16 (IEEE half:
// the reference's AMP / config-5 dtype); every kernel accumulates in fp32.  dtype codes on
// the C-ABI: 0 = fp32, 1 = bf16, 2 = fp16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <type_traits>
#include "../../include/cmx_hip.h"  // compiler-checks every definition against the ABI header
                                     // (and defines CMX_ABI_VERSION)

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
// launch-policy knob NAME: a stable reference, initialised from CMX_NAME or `def` (abi.cpp)
int& cmx_knob(const char* name, int def);

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
// fp32 -> bf16 with gfx950's v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN stays NaN)
typedef float cmx_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 cmx_bf2 __attribute__((ext_vector_type(2)));
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float v) {
  bf16 r;
  r.x = __builtin_bit_cast(uint16_t, (__bf16)v);
  return r;
}
// two fp32 -> packed bf16 pair (lo = a), one instruction
__device__ __forceinline__ uint32_t pack2_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((cmx_f2){a, b}, cmx_bf2));
}

// ---------------------------------------------------------------- f16 (IEEE half)
struct f16 {
  uint16_t x;
};
typedef _Float16 cmx_h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float to_f32(f16 v) { return (float)__builtin_bit_cast(_Float16, v.x); }
// fp32 -> fp16 round-to-nearest-even (v_cvt_f16_f32), overflow -> inf like a cast in torch
template <> __device__ __forceinline__ f16 from_f32<f16>(float v) {
  f16 r;
  r.x = __builtin_bit_cast(uint16_t, (_Float16)v);
  return r;
}
__device__ __forceinline__ uint32_t pack2_f16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((cmx_f2){a, b}, cmx_h2));
}

// 16-bit storage types (bf16, f16) share every 2-byte code path; these convert a packed pair.
template <typename T> constexpr bool is_h16 = std::is_same<T, bf16>::value || std::is_same<T, f16>::value;
template <typename T> __device__ __forceinline__ uint32_t pack2(float a, float b) {
  if constexpr (std::is_same<T, bf16>::value) return pack2_bf16(a, b);
  else return pack2_f16(a, b);
}
template <typename T> __device__ __forceinline__ cmx_f2 unpack2(uint32_t u) {
  if constexpr (std::is_same<T, bf16>::value) {
    return (cmx_f2){__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
  } else {
    return __builtin_convertvector(__builtin_bit_cast(cmx_h2, u), cmx_f2);
  }
}
// the stored 16-bit pattern of 1.0 (a constant MFMA operand)
template <typename T> constexpr uint16_t one_bits = std::is_same<T, bf16>::value ? 0x3f80 : 0x3c00;

// 16-byte vectors: VEC<float> = 4 elements, VEC<bf16 / f16> = 8 elements.
template <typename T> struct VecT;
template <> struct VecT<float> { static constexpr int N = 4; typedef float4 raw; };
template <> struct VecT<bf16> { static constexpr int N = 8; typedef uint4 raw; };
template <> struct VecT<f16> { static constexpr int N = 8; typedef uint4 raw; };

// one 16-B vector as loaded (raw) and its fp32 values: a raw load can be issued well before
// its values are wanted (across a barrier or a prologue loop, which the compiler does not move
// the unpacking past, so a load_vec there waits for its data on the spot)
template <typename T>
__device__ __forceinline__ typename VecT<T>::raw load_raw(const T* p) {
  return *reinterpret_cast<const typename VecT<T>::raw*>(p);
}
template <typename T>
__device__ __forceinline__ void unpack_raw(const typename VecT<T>::raw& v, float* out) {
  if constexpr (sizeof(T) == 4) {
    out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
  } else {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const cmx_f2 f = unpack2<T>(w[i]);
      out[2 * i] = f.x;
      out[2 * i + 1] = f.y;
    }
  }
}
template <typename T>
__device__ __forceinline__ void load_vec(const T* p, float* out) {
  unpack_raw<T>(load_raw<T>(p), out);
}

// load_vec of p[off] when ok, zeros otherwise -- as an UNCONDITIONAL load of a clamped offset
// (`safe`: any in-bounds one) and a select.  A load inside `if (ok) ... else zero` makes the
// compiler wait for it at the branch's join, so loads meant to be in flight together (several
// rows per lane) became one round trip each.
template <typename T>
__device__ __forceinline__ void load_vec_if(const T* p, long off, long safe, bool ok, float* out) {
  constexpr int N = VecT<T>::N;
  load_vec<T>(p + (ok ? off : safe), out);
#pragma unroll
  for (int j = 0; j < N; ++j) out[j] = ok ? out[j] : 0.f;
}

template <typename T>
__device__ __forceinline__ void store_vec(T* p, const float* in) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(in[0], in[1], in[2], in[3]);
  } else {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[i] = pack2<T>(in[2 * i], in[2 * i + 1]);
    }
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// ---------------------------------------------------------------- in-kernel partial folds
// A kernel whose blocks each produce a partial result can fold the partials in the LAST block
// to arrive instead of a second launch.  The 8 XCDs have separate L2s, so the partials are
// written with agent-scope stores (global_store ... sc1: through to the device-coherent level)
// and read back with agent-scope loads (sc1: not served from a stale L2 line); each block
// drains its stores (s_waitcnt 0) before taking a ticket with a relaxed device atomic.  No
// release / acquire fence: at agent scope those write back / invalidate the whole L2 per block
// (AdamW measured 891 us with one per block).  The ticket counter is reset by the last block,
// so a graph replay or the next launch finds it at zero; a ticket array is owned by one kernel
// family and its launches are stream-ordered.
__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_agent(const int* p) {
  return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// true in every thread of the block that arrives last of `total` blocks sharing `ticket`
__device__ __forceinline__ bool last_arrival(unsigned* ticket, unsigned total) {
  __shared__ int s_last;
  __builtin_amdgcn_s_waitcnt(0);                // this thread's partial stores have completed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == total - 1;
    if (prev == total - 1) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return s_last != 0;
}

// ---------------------------------------------------------------- cross-lane exchange
// v of lane (lane ^ O), O a power of two < 64, on the VALU instead of the LDS crossbar
// (__shfl_xor is a ds_bpermute: an address, an LDS-pipe round trip and an lgkmcnt wait per
// step): DPP quad permutes for O = 1, 2, DPP row rotates for O = 4, 8 (a 16-lane row rotated by
// 8 is lane ^ 8; by 4 / 12 selected on lane bit 2 is lane ^ 4), gfx950's v_permlane16_swap /
// v_permlane32_swap for O = 16, 32 (the swap hands each half its partner row / half, one select
// per lane).  Exact xor semantics: reductions built on it add in the same order as the
// __shfl_xor butterflies they replace and give the same bits.  Every lane of the group must be
// active (all callers reduce in uniform control flow or over whole row groups).
template <int O>
__device__ __forceinline__ float xor_lane(float v) {
  const int x = __builtin_bit_cast(int, v);
  if constexpr (O == 1) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(x, x, 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
  } else if constexpr (O == 2) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(x, x, 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
  } else if constexpr (O == 4) {
    const int a = __builtin_amdgcn_update_dpp(x, x, 0x124, 0xF, 0xF, false);                      // row_ror 4
    const int b = __builtin_amdgcn_update_dpp(x, x, 0x12C, 0xF, 0xF, false);                      // row_ror 12
    return __builtin_bit_cast(float, (__lane_id() & 4) ? a : b);
  } else if constexpr (O == 8) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(x, x, 0x128, 0xF, 0xF, false));  // row_ror 8
  } else if constexpr (O == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
    return __builtin_bit_cast(float, (__lane_id() & 16) ? r[0] : r[1]);
  } else {
    static_assert(O == 32, "xor_lane: O in 1 .. 32");
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)x, false, false);
    return __builtin_bit_cast(float, (__lane_id() & 32) ? r[0] : r[1]);
  }
}
// the same for an offset known only after inlining (folds to one case when it is a constant)
__device__ __forceinline__ float xor_lane(float v, int o) {
  switch (o) {
    case 1: return xor_lane<1>(v);
    case 2: return xor_lane<2>(v);
    case 4: return xor_lane<4>(v);
    case 8: return xor_lane<8>(v);
    case 16: return xor_lane<16>(v);
    case 32: return xor_lane<32>(v);
    default: return __shfl_xor(v, o, 64);
  }
}

// ---------------------------------------------------------------- reductions
// sum across a power-of-two group of `width` lanes (width <= 64): the butterfly from the widest
// offset down, as the __shfl_xor loop this replaced (same bits)
__device__ __forceinline__ float group_sum(float v, int width) {
  if (width > 32) v += xor_lane<32>(v);
  if (width > 16) v += xor_lane<16>(v);
  if (width > 8) v += xor_lane<8>(v);
  if (width > 4) v += xor_lane<4>(v);
  if (width > 2) v += xor_lane<2>(v);
  if (width > 1) v += xor_lane<1>(v);
  return v;
}
__device__ __forceinline__ float wave_sum(float v) { return group_sum(v, 64); }

// Branch-free fp32 erf: x * P(x^2) / Q(x^2) on x clamped to [-4, 4] (the rational minimax
// form used by Eigen's fast float erf); max |error| 4.2e-7 against libm erf on [-6, 6]
// (checked in tests/test_oracle_kats.py::test_fast_erf_table).  ocml's erff branches on the
// argument range and divides; this is 12 FMAs + 1 v_rcp_f32, which matters in the
// HBM/VALU-balanced DWConv+GELU stencil.
__device__ __forceinline__ float cmx_erf(float x) {
  x = fminf(fmaxf(x, -4.f), 4.f);
  const float x2 = x * x;
  float p = -2.72614225801306e-10f;
  p = fmaf(p, x2, 2.77068142495902e-08f);
  p = fmaf(p, x2, -2.10102402082508e-06f);
  p = fmaf(p, x2, -5.69250639462346e-05f);
  p = fmaf(p, x2, -7.34990630326855e-04f);
  p = fmaf(p, x2, -2.95459980854025e-03f);
  p = fmaf(p, x2, -1.60960333262415e-02f);
  float q = -1.45660718464996e-05f;
  q = fmaf(q, x2, -2.13374055278905e-04f);
  q = fmaf(q, x2, -1.68282697438203e-03f);
  q = fmaf(q, x2, -7.37332916720468e-03f);
  q = fmaf(q, x2, -1.42647390514189e-02f);
  return x * p * __builtin_amdgcn_rcpf(q);
}
__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.f + cmx_erf(x * 0.70710678118654752f));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.f + cmx_erf(x * 0.70710678118654752f));
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

// ---------------------------------------------------------------- packed (2 x fp32) math
// ext_vector_type(2) arithmetic lowers to v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two
// fp32 lanes per VALU op, used by the VALU-heavy stencil kernels (DWConv + GELU).
__device__ __forceinline__ cmx_f2 pk_fma(cmx_f2 a, cmx_f2 b, cmx_f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ cmx_f2 pk_splat(float v) { return (cmx_f2){v, v}; }

__device__ __forceinline__ cmx_f2 cmx_erf2(cmx_f2 x) {
  x.x = fminf(fmaxf(x.x, -4.f), 4.f);
  x.y = fminf(fmaxf(x.y, -4.f), 4.f);
  const cmx_f2 x2 = x * x;
  cmx_f2 p = pk_splat(-2.72614225801306e-10f);
  p = pk_fma(p, x2, pk_splat(2.77068142495902e-08f));
  p = pk_fma(p, x2, pk_splat(-2.10102402082508e-06f));
  p = pk_fma(p, x2, pk_splat(-5.69250639462346e-05f));
  p = pk_fma(p, x2, pk_splat(-7.34990630326855e-04f));
  p = pk_fma(p, x2, pk_splat(-2.95459980854025e-03f));
  p = pk_fma(p, x2, pk_splat(-1.60960333262415e-02f));
  cmx_f2 q = pk_splat(-1.45660718464996e-05f);
  q = pk_fma(q, x2, pk_splat(-2.13374055278905e-04f));
  q = pk_fma(q, x2, pk_splat(-1.68282697438203e-03f));
  q = pk_fma(q, x2, pk_splat(-7.37332916720468e-03f));
  q = pk_fma(q, x2, pk_splat(-1.42647390514189e-02f));
  const cmx_f2 r = {__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)};
  return x * p * r;
}

// compile-time activation on a pair (ACT_* codes below)
template <int ACT>
__device__ __forceinline__ cmx_f2 act2_fwd(cmx_f2 z) {
  if constexpr (ACT == 1) {            // GELU (erf)
    const cmx_f2 e = cmx_erf2(z * pk_splat(0.70710678118654752f));
    return pk_splat(0.5f) * z * (pk_splat(1.f) + e);
  } else if constexpr (ACT == 2) {     // ReLU
    return (cmx_f2){z.x > 0.f ? z.x : 0.f, z.y > 0.f ? z.y : 0.f};
  } else if constexpr (ACT == 3) {     // sigmoid
    return (cmx_f2){1.f / (1.f + __expf(-z.x)), 1.f / (1.f + __expf(-z.y))};
  } else {
    return z;
  }
}
template <int ACT>
__device__ __forceinline__ cmx_f2 act2_grad(cmx_f2 z) {
  if constexpr (ACT == 1) {
    const cmx_f2 cdf = pk_splat(0.5f) * (pk_splat(1.f) + cmx_erf2(z * pk_splat(0.70710678118654752f)));
    const cmx_f2 pdf = pk_splat(0.39894228040143268f) *
                       (cmx_f2){__expf(-0.5f * z.x * z.x), __expf(-0.5f * z.y * z.y)};
    return pk_fma(z, pdf, cdf);
  } else if constexpr (ACT == 2) {
    return (cmx_f2){z.x > 0.f ? 1.f : 0.f, z.y > 0.f ? 1.f : 0.f};
  } else if constexpr (ACT == 3) {
    const float sx = 1.f / (1.f + __expf(-z.x)), sy = 1.f / (1.f + __expf(-z.y));
    return (cmx_f2){sx * (1.f - sx), sy * (1.f - sy)};
  } else {
    return pk_splat(1.f);
  }
}

// runtime activation code -> compile-time template argument
#define CMX_ACT_DISPATCH(act, A, ...)                                            \
  do {                                                                          \
    switch (act) {                                                              \
      case 0: { constexpr int A = 0; __VA_ARGS__; break; }                      \
      case 1: { constexpr int A = 1; __VA_ARGS__; break; }                      \
      case 2: { constexpr int A = 2; __VA_ARGS__; break; }                      \
      case 3: { constexpr int A = 3; __VA_ARGS__; break; }                      \
      default: cmx_set_error("unsupported activation %d", (int)(act)); return CMX_ERR_ARG; \
    }                                                                           \
  } while (0)

// bilinear source index of F.interpolate(align_corners=False), PyTorch's rule:
//   src = max(0, (dst + 0.5) * in/out - 0.5); i0 = floor(src); i1 = min(i0 + 1, in - 1)
// (scale = (float)in / out, as PyTorch forms it); weights l0 = 1 - (src - i0), l1 = src - i0
__device__ __forceinline__ void cmx_bilin_src(int dst, float scale, int in, int& i0, int& i1, float& l0, float& l1) {
  float s = (dst + 0.5f) * scale - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = s - (float)i0;
  l0 = 1.f - l1;
}

static inline unsigned cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }

// dtype dispatch helper for launch wrappers
#define CMX_DISPATCH(dtype, T, ...)                                   \
  do {                                                                \
    if ((dtype) == 0) { typedef float T; __VA_ARGS__; }               \
    else if ((dtype) == 1) { typedef bf16 T; __VA_ARGS__; }           \
    else if ((dtype) == 2) { typedef f16 T; __VA_ARGS__; }            \
    else { cmx_set_error("unsupported dtype %d", (int)(dtype)); return CMX_ERR_DTYPE; } \
  } while (0)

// ws (G, nblk, W) -> out (G, W); defined in layernorm.hip, shared by all two-stage reductions
int cmx_reduce_partials(const float* ws, float* out, int G, int nblk, int W, int accumulate,
                        float alpha, hipStream_t s);
// ws (nblk, stride) columns [0, W) -> out (W)
int cmx_reduce_partials_strided(const float* ws, float* out, int nblk, int W, int stride, int accumulate,
                                hipStream_t s);
