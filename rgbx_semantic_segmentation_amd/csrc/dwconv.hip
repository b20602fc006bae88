// Depthwise 3x3 (pad 1, stride 1) convolution + bias + activation on token-major NHWC.
//
// Replaces  DWConv.forward + act  of Mix-FFN (dual_segformer.py:27-33, 67-71:
//   x.permute(0,2,1).reshape(B,C,H,W) -> Conv2d(C,C,3,1,1,groups=C) -> flatten/transpose -> GELU)
// and the DW3x3 + ReLU of ChannelEmbed (net_utils.py:315-318).  No NCHW round trip: the
// channel dim is contiguous.
//
// Images: NI = G*B images of H x W x C; image n belongs to group n / imgs_per_group (the
// RGB and X streams carry separate weights).  w: (G, C, 9) fp32, b: (G, C) fp32.
// Thread mapping: a thread owns ONE quad of 4 channels for its whole life (its 36 weights
// and 4 biases live in registers) and walks a strided set of pixels of one group; lanes of
// a wave are consecutive quads, so every 3x3 neighbour load is a coalesced 8-byte (bf16) /
// 16-byte (fp32) row segment.  HBM-bound: read h once (+L1/L2 halo re-reads), write once.
#include "cmx_common.h"

namespace {
constexpr int DW_THREADS_PER_GROUP = 32768;   // quads x pixel slots per group

template <typename T>
__device__ __forceinline__ void ld4(const T* p, float* v) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  } else {
    const uint2 a = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(a.x << 16); v[1] = __uint_as_float(a.x & 0xffff0000u);
    v[2] = __uint_as_float(a.y << 16); v[3] = __uint_as_float(a.y & 0xffff0000u);
  }
}

template <typename T>
__device__ __forceinline__ void st4(T* p, const float* v) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    const uint32_t a = (uint32_t)from_f32<bf16>(v[0]).x | ((uint32_t)from_f32<bf16>(v[1]).x << 16);
    const uint32_t b = (uint32_t)from_f32<bf16>(v[2]).x | ((uint32_t)from_f32<bf16>(v[3]).x << 16);
    *reinterpret_cast<uint2*>(p) = make_uint2(a, b);
  }
}

__device__ __forceinline__ void load_w36(const float* wg, float (&w)[4][9]) {
  // the 4 channels' 9 taps are 36 contiguous floats (c0 % 4 == 0 -> 16-byte aligned)
  const float4* p = reinterpret_cast<const float4*>(wg);
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const float4 a = p[i];
    const float f[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) w[(4 * i + u) / 9][(4 * i + u) % 9] = f[u];
  }
}

int slots_for(int CQ) {
  int p = DW_THREADS_PER_GROUP / CQ;
  return p < 1 ? 1 : p;
}

// forward (flip = 0) or transposed conv of the backward (flip = 1, no bias, no act)
template <typename T>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const T* __restrict__ h, const float* __restrict__ w,
                                                     const float* __restrict__ b, T* __restrict__ out, int ipg, int H,
                                                     int W, int C, int act, int flip, int P) {
  const int CQ = C / 4;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= CQ * P) return;
  const int g = blockIdx.y;
  const int q = t % CQ, slot = t / CQ;
  const int c0 = q * 4;
  float wr[4][9], bias[4];
  load_w36(w + ((long)g * C + c0) * 9, wr);
#pragma unroll
  for (int u = 0; u < 4; ++u) bias[u] = b ? b[(long)g * C + c0 + u] : 0.f;
  const long gpix = (long)ipg * H * W;
  const T* base = h + (long)g * gpix * C + c0;
  T* obase = out + (long)g * gpix * C + c0;
  for (int p = slot; p < (int)gpix; p += P) {
    const int x = p % W;
    const int y = (p / W) % H;
    const int img = p / (W * H);
    const T* ib = base + img * H * W * C;
    float acc[4] = {bias[0], bias[1], bias[2], bias[3]};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int yy = y + i - 1;
      if (yy < 0 || yy >= H) continue;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int xx = x + j - 1;
        if (xx < 0 || xx >= W) continue;
        float v[4];
        ld4<T>(ib + ((long)yy * W + xx) * C, v);
        const int tap = flip ? 8 - (i * 3 + j) : i * 3 + j;
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] += wr[u][tap] * v[u];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = act_fwd(acc[u], act);
    st4<T>(obase + p * C, acc);
  }
}

// dz = da * act'(z) with z recomputed; per-thread partial dW (9 taps) / db for the thread's
// quad go to ws[(g, slot)][c][10] (reduced afterwards over the P slots).
template <typename T>
__global__ __launch_bounds__(256) void dw_bwd_dz_kernel(const T* __restrict__ da, const T* __restrict__ h,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        T* __restrict__ dz, float* __restrict__ ws, int ipg, int H,
                                                        int W, int C, int act, int P) {
  const int CQ = C / 4;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= CQ * P) return;
  const int g = blockIdx.y;
  const int q = t % CQ, slot = t / CQ;
  const int c0 = q * 4;
  float wr[4][9], bias[4], aw[4][9], ab[4];
  load_w36(w + ((long)g * C + c0) * 9, wr);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    bias[u] = b ? b[(long)g * C + c0 + u] : 0.f;
    ab[u] = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) aw[u][k] = 0.f;
  }
  const long gpix = (long)ipg * H * W;
  const T* base = h + (long)g * gpix * C + c0;
  for (int p = slot; p < (int)gpix; p += P) {
    const int x = p % W;
    const int y = (p / W) % H;
    const int img = p / (W * H);
    const T* ib = base + img * H * W * C;
    float hv[9][4];
    float z[4] = {bias[0], bias[1], bias[2], bias[3]};
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
        ld4<T>(ib + ((long)yy * W + xx) * C, hv[k]);
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) hv[k][u] = 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) z[u] += wr[u][k] * hv[k][u];
    }
    const long pofs = ((long)g * gpix + p) * C + c0;
    float d[4];
    ld4<T>(da + pofs, d);
#pragma unroll
    for (int u = 0; u < 4; ++u) d[u] *= act_grad(z[u], act);
    st4<T>(dz + pofs, d);
    // accumulate with the value as stored (bf16-rounded) so dW matches the dz used for dh
    float dq[4];
    if constexpr (sizeof(T) == 2) {
      ld4<T>(dz + pofs, dq);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) dq[u] = d[u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      ab[u] += dq[u];
#pragma unroll
      for (int k = 0; k < 9; ++k) aw[u][k] += dq[u] * hv[k][u];
    }
  }
  float* o = ws + ((long)g * P + slot) * C * 10 + (long)c0 * 10;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
#pragma unroll
    for (int k = 0; k < 9; ++k) o[u * 10 + k] = aw[u][k];
    o[u * 10 + 9] = ab[u];
  }
}

// tmp (G, C, 10) -> dw (G, C, 9), db (G, C)
__global__ void dw_scatter_kernel(const float* __restrict__ tmp, float* __restrict__ dw, float* __restrict__ db, int G,
                                  int C, int accumulate) {
  const long total = (long)G * C * 10;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)total; i += gridDim.x * blockDim.x) {
    const int k = i % 10;
    const int gc = i / 10;
    const float s = tmp[i];
    float* o = k < 9 ? &dw[gc * 9 + k] : (db ? &db[gc] : nullptr);
    if (o) *o = accumulate ? *o + s : s;
  }
}
}  // namespace

extern "C" {

int cmx_dwconv3x3_fwd(const void* h, const float* w, const float* b, void* out, int NI, int imgs_per_group, int H,
                      int W, int C, int act, int dtype, hipStream_t s) {
  CMX_REQUIRE(C % 4 == 0 && NI % imgs_per_group == 0, CMX_ERR_SHAPE, "dwconv_fwd: C=%d", C);
  const int G = NI / imgs_per_group;
  const int P = slots_for(C / 4);
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(dw_fwd_kernel<T>, dim3(cdiv((long)(C / 4) * P, 256), G), dim3(256), 0, s, (const T*)h, w, b,
                       (T*)out, imgs_per_group, H, W, C, act, 0, P);
  });
  return cmx_check_launch("dwconv_fwd");
}

size_t cmx_dwconv3x3_bwd_workspace(int NI, int imgs_per_group, int H, int W, int C) {
  const int G = NI / imgs_per_group;
  const int P = slots_for(C / 4);
  return ((size_t)G * P * C * 10 + (size_t)G * C * 10) * sizeof(float);
}

// da: upstream grad of the activation output; dz (sized like h, dtype) receives
// da * act'(z); dh = conv^T(dz) (may be NULL); dw (G,C,9), db (G,C) fp32 (db may be NULL).
int cmx_dwconv3x3_bwd(const void* da, const void* h, const float* w, const float* b, void* dz, void* dh, float* dw,
                      float* db, float* workspace, int NI, int imgs_per_group, int H, int W, int C, int act,
                      int accumulate, int dtype, hipStream_t s) {
  CMX_REQUIRE(C % 4 == 0 && NI % imgs_per_group == 0, CMX_ERR_SHAPE, "dwconv_bwd: C=%d", C);
  const int G = NI / imgs_per_group;
  const int CQ = C / 4;
  const int P = slots_for(CQ);
  float* tmp = workspace + (size_t)G * P * C * 10;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(dw_bwd_dz_kernel<T>, dim3(cdiv((long)CQ * P, 256), G), dim3(256), 0, s, (const T*)da,
                       (const T*)h, w, b, (T*)dz, workspace, imgs_per_group, H, W, C, act, P);
    if (dh)
      hipLaunchKernelGGL(dw_fwd_kernel<T>, dim3(cdiv((long)CQ * P, 256), G), dim3(256), 0, s, (const T*)dz, w,
                         (const float*)nullptr, (T*)dh, imgs_per_group, H, W, C, (int)ACT_NONE, 1, P);
  });
  int st = cmx_reduce_partials(workspace, tmp, G, P, C * 10, 0, 1.f, s);
  if (st) return st;
  const long tot = (long)G * C * 10;
  hipLaunchKernelGGL(dw_scatter_kernel, dim3(cdiv(tot, 256) < 4096 ? cdiv(tot, 256) : 4096), dim3(256), 0, s, tmp, dw,
                     db, G, C, accumulate);
  return cmx_check_launch("dwconv_bwd");
}

}  // extern "C"
