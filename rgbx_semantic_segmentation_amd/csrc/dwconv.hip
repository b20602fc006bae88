// Depthwise 3x3 (pad 1, stride 1) convolution + bias + activation on token-major NHWC.
//
// Replaces  DWConv.forward + act  of Mix-FFN (dual_segformer.py:27-33, 67-71:
//   x.permute(0,2,1).reshape(B,C,H,W) -> Conv2d(C,C,3,1,1,groups=C) -> flatten/transpose -> GELU)
// and the DW3x3 + ReLU of ChannelEmbed (net_utils.py:315-318).  No NCHW round trip: the
// channel dim is contiguous.
//
// Images: NI = G*B images of H x W x C; image n belongs to group n / imgs_per_group (the
// RGB and X streams carry separate weights).  w: (G, C, 9) fp32, b: (G, C) fp32.
//
// Thread mapping (HBM/VALU-balanced stencil): a thread owns ONE quad of 4 channels (two
// packed fp32 pairs, so the taps and the GELU run as v_pk_fma_f32) and a strip of RX x RY
// output pixels.  It keeps a sliding window of 3 input rows (RX + 2 pixels each) in
// registers, so each input row is fetched once per strip ((RY+2)(RX+2) loads for RX*RY
// outputs), and its 36 weights + 4 biases stay in registers.  All loads are straight-line
// (out-of-image taps are predicated to zero, stores predicated), so a strip's loads can be
// in flight together.  Lanes of a wave are consecutive quads: every load / store is a
// coalesced 8-byte (bf16) / 16-byte (fp32) segment of a channel-contiguous NHWC row.
// The activation is a template argument: the GELU kernels carry no dead ReLU/sigmoid code.
#include "cmx_common.h"

namespace {
constexpr int RXF = 4;           // output pixels per strip along x (forward / transposed pass)
constexpr int RXB = 2;           // ... in the dW-accumulating backward pass (register budget)
constexpr int RY = 8;            // output rows per strip
constexpr int DW_BWD_THREADS = 65536;   // target threads per group for the dW-accumulating pass

typedef cmx_f2 Px[2];            // 4 channels as two packed pairs

template <typename T>
__device__ __forceinline__ void ld4(const T* p, Px& v) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = (cmx_f2){a.x, a.y};
    v[1] = (cmx_f2){a.z, a.w};
  } else {
    const uint2 a = *reinterpret_cast<const uint2*>(p);
    v[0] = (cmx_f2){__uint_as_float(a.x << 16), __uint_as_float(a.x & 0xffff0000u)};
    v[1] = (cmx_f2){__uint_as_float(a.y << 16), __uint_as_float(a.y & 0xffff0000u)};
  }
}

template <typename T>
__device__ __forceinline__ void st4(T* p, const Px& v) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0].x, v[0].y, v[1].x, v[1].y);
  } else {
    *reinterpret_cast<uint2*>(p) = make_uint2(pack2_bf16(v[0].x, v[0].y), pack2_bf16(v[1].x, v[1].y));
  }
}

// the pair as it is stored in T (bf16 round-to-nearest-even)
template <typename T>
__device__ __forceinline__ cmx_f2 stored(cmx_f2 v) {
  if constexpr (sizeof(T) == 4) {
    return v;
  } else {
    const uint32_t u = pack2_bf16(v.x, v.y);
    return (cmx_f2){__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
  }
}

// the 4 channels' 9 taps are 36 contiguous floats (c0 % 4 == 0 -> 16-byte aligned);
// w2[pair][tap] = {w[2 pair][tap], w[2 pair + 1][tap]}
__device__ __forceinline__ void load_w36(const float* wg, cmx_f2 (&w2)[2][9]) {
  const float4* p = reinterpret_cast<const float4*>(wg);
  float w[36];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const float4 a = p[i];
    w[4 * i] = a.x; w[4 * i + 1] = a.y; w[4 * i + 2] = a.z; w[4 * i + 3] = a.w;
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    w2[0][k] = (cmx_f2){w[k], w[9 + k]};
    w2[1][k] = (cmx_f2){w[18 + k], w[27 + k]};
  }
}

__device__ __forceinline__ void load_bias(const float* b, Px& bias) {
  if (b) {
    const float4 bb = *reinterpret_cast<const float4*>(b);
    bias[0] = (cmx_f2){bb.x, bb.y};
    bias[1] = (cmx_f2){bb.z, bb.w};
  } else {
    bias[0] = bias[1] = pk_splat(0.f);
  }
}

// input row y, pixels x0-1 .. x0+R of one image (ib already offset to channel c0)
template <typename T, int R>
__device__ __forceinline__ void load_row(const T* ib, int y, int x0, int H, int W, int C, Px (&r)[R + 2]) {
  const bool yok = y >= 0 && y < H;
#pragma unroll
  for (int j = 0; j < R + 2; ++j) {
    const int x = x0 - 1 + j;
    if (yok && x >= 0 && x < W) {
      ld4<T>(ib + (y * W + x) * C, r[j]);
    } else {
      r[j][0] = pk_splat(0.f);
      r[j][1] = pk_splat(0.f);
    }
  }
}

struct Strip {
  int img, x0, y0;
};

template <int R>
__device__ __forceinline__ Strip strip_of(int s, int NXS, int NYS) {
  Strip st;
  st.x0 = (s % NXS) * R;
  const int r = s / NXS;
  st.y0 = (r % NYS) * RY;
  st.img = r / NYS;
  return st;
}

// forward (FLIP = false: cross-correlation + bias + act) or the transposed conv of the
// backward (FLIP = true: taps mirrored, no bias, ACT = 0).  One strip per thread.
template <typename T, bool FLIP, int ACT>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const T* __restrict__ h, const float* __restrict__ w,
                                                     const float* __restrict__ b, T* __restrict__ out, int ipg, int H,
                                                     int W, int C, int NXS, int NYS) {
  const int CQ = C >> 2;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= CQ * NXS * NYS * ipg) return;
  const int g = blockIdx.y;
  const int c0 = (t % CQ) * 4;
  const Strip st = strip_of<RXF>(t / CQ, NXS, NYS);
  cmx_f2 wr[2][9];
  load_w36(w + ((long)g * C + c0) * 9, wr);
  Px bias;
  load_bias(b ? b + g * C + c0 : nullptr, bias);
  const long off = ((long)g * ipg + st.img) * H * W * C + c0;
  const T* ib = h + off;
  T* ob = out + off;
  Px rin[3][RXF + 2];
  load_row<T, RXF>(ib, st.y0 - 1, st.x0, H, W, C, rin[0]);
  load_row<T, RXF>(ib, st.y0, st.x0, H, W, C, rin[1]);
#pragma unroll
  for (int rr = 0; rr < RY; ++rr) {
    const int y = st.y0 + rr;
    load_row<T, RXF>(ib, y + 1, st.x0, H, W, C, rin[(rr + 2) % 3]);
#pragma unroll
    for (int xi = 0; xi < RXF; ++xi) {
      Px acc = {bias[0], bias[1]};
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int tap = FLIP ? 8 - (i * 3 + j) : i * 3 + j;
#pragma unroll
          for (int u = 0; u < 2; ++u) acc[u] = pk_fma(wr[u][tap], rin[(rr + i) % 3][xi + j][u], acc[u]);
        }
      acc[0] = act2_fwd<ACT>(acc[0]);
      acc[1] = act2_fwd<ACT>(acc[1]);
      if (y < H && st.x0 + xi < W) st4<T>(ob + (y * W + st.x0 + xi) * C, acc);
    }
  }
}

// dz = da * act'(z) with z recomputed from h; per-thread partial dW (9 taps) / db of the
// thread's quad over its strips go to ws[(g, slot)][c][10] (reduced afterwards over the P
// slots).  Thread (q, slot) processes strips slot, slot + P, ...
template <typename T, int ACT>
__global__ __launch_bounds__(256) void dw_bwd_dz_kernel(const T* __restrict__ da, const T* __restrict__ h,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        T* __restrict__ dz, float* __restrict__ ws, int ipg, int H,
                                                        int W, int C, int NXS, int NYS, int P) {
  const int CQ = C >> 2;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= CQ * P) return;
  const int g = blockIdx.y;
  const int q = t % CQ, slot = t / CQ;
  const int c0 = q * 4;
  cmx_f2 wr[2][9], aw[2][9];
  Px bias, ab;
  load_w36(w + ((long)g * C + c0) * 9, wr);
  load_bias(b ? b + g * C + c0 : nullptr, bias);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    ab[u] = pk_splat(0.f);
#pragma unroll
    for (int k = 0; k < 9; ++k) aw[u][k] = pk_splat(0.f);
  }
  const int nstrips = NXS * NYS * ipg;
  for (int s = slot; s < nstrips; s += P) {
    const Strip st = strip_of<RXB>(s, NXS, NYS);
    const long off = ((long)g * ipg + st.img) * H * W * C + c0;
    const T* ib = h + off;
    const T* dab = da + off;
    T* dzb = dz + off;
    Px rin[3][RXB + 2];
    load_row<T, RXB>(ib, st.y0 - 1, st.x0, H, W, C, rin[0]);
    load_row<T, RXB>(ib, st.y0, st.x0, H, W, C, rin[1]);
#pragma unroll
    for (int rr = 0; rr < RY; ++rr) {
      const int y = st.y0 + rr;
      load_row<T, RXB>(ib, y + 1, st.x0, H, W, C, rin[(rr + 2) % 3]);
#pragma unroll
      for (int xi = 0; xi < RXB; ++xi) {
        const bool in = y < H && st.x0 + xi < W;
        Px d = {pk_splat(0.f), pk_splat(0.f)};
        if (in) {
          Px z = {bias[0], bias[1]};
#pragma unroll
          for (int k = 0; k < 9; ++k)
#pragma unroll
            for (int u = 0; u < 2; ++u) z[u] = pk_fma(wr[u][k], rin[(rr + k / 3) % 3][xi + k % 3][u], z[u]);
          const int pofs = (y * W + st.x0 + xi) * C;
          ld4<T>(dab + pofs, d);
#pragma unroll
          for (int u = 0; u < 2; ++u) d[u] = d[u] * act2_grad<ACT>(z[u]);
          st4<T>(dzb + pofs, d);
          // accumulate with the value as stored so dW matches the dz used for dh
#pragma unroll
          for (int u = 0; u < 2; ++u) d[u] = stored<T>(d[u]);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          ab[u] += d[u];
#pragma unroll
          for (int k = 0; k < 9; ++k) aw[u][k] = pk_fma(d[u], rin[(rr + k / 3) % 3][xi + k % 3][u], aw[u][k]);
        }
      }
    }
  }
  float* o = ws + ((long)g * P + slot) * C * 10 + (long)c0 * 10;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      o[(2 * u) * 10 + k] = aw[u][k].x;
      o[(2 * u + 1) * 10 + k] = aw[u][k].y;
    }
    o[(2 * u) * 10 + 9] = ab[u].x;
    o[(2 * u + 1) * 10 + 9] = ab[u].y;
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

int bwd_slots(int CQ, int nstrips) {
  int pmax = DW_BWD_THREADS / CQ;
  if (pmax < 1) pmax = 1;
  if (pmax >= nstrips) return nstrips;
  const int per = (nstrips + pmax - 1) / pmax;    // strips per thread, balanced
  return (nstrips + per - 1) / per;
}
}  // namespace

extern "C" {

int cmx_dwconv3x3_fwd(const void* h, const float* w, const float* b, void* out, int NI, int imgs_per_group, int H,
                      int W, int C, int act, int dtype, hipStream_t s) {
  CMX_REQUIRE(C % 4 == 0 && NI % imgs_per_group == 0, CMX_ERR_SHAPE, "dwconv_fwd: C=%d", C);
  CMX_REQUIRE((long)NI * H * W * C < (1L << 31), CMX_ERR_SHAPE, "dwconv_fwd: tensor too large for 32-bit indexing");
  const int G = NI / imgs_per_group;
  const int NXS = cdiv(W, RXF), NYS = cdiv(H, RY);
  const long threads = (long)(C / 4) * NXS * NYS * imgs_per_group;
  CMX_DISPATCH(dtype, T, {
    CMX_ACT_DISPATCH(act, A, {
      hipLaunchKernelGGL((dw_fwd_kernel<T, false, A>), dim3(cdiv(threads, 256), G), dim3(256), 0, s, (const T*)h, w,
                         b, (T*)out, imgs_per_group, H, W, C, NXS, NYS);
    });
  });
  return cmx_check_launch("dwconv_fwd");
}

size_t cmx_dwconv3x3_bwd_workspace(int NI, int imgs_per_group, int H, int W, int C) {
  const int G = NI / imgs_per_group;
  const int P = bwd_slots(C / 4, cdiv(W, RXB) * cdiv(H, RY) * imgs_per_group);
  return ((size_t)G * P * C * 10 + (size_t)G * C * 10) * sizeof(float);
}

// da: upstream grad of the activation output; dz (sized like h, dtype) receives
// da * act'(z); dh = conv^T(dz) (may be NULL); dw (G,C,9), db (G,C) fp32 (db may be NULL).
int cmx_dwconv3x3_bwd(const void* da, const void* h, const float* w, const float* b, void* dz, void* dh, float* dw,
                      float* db, float* workspace, int NI, int imgs_per_group, int H, int W, int C, int act,
                      int accumulate, int dtype, hipStream_t s) {
  CMX_REQUIRE(C % 4 == 0 && NI % imgs_per_group == 0, CMX_ERR_SHAPE, "dwconv_bwd: C=%d", C);
  CMX_REQUIRE((long)NI * H * W * C < (1L << 31), CMX_ERR_SHAPE, "dwconv_bwd: tensor too large for 32-bit indexing");
  const int G = NI / imgs_per_group;
  const int CQ = C / 4;
  const int NXB = cdiv(W, RXB), NXS = cdiv(W, RXF), NYS = cdiv(H, RY);
  const int P = bwd_slots(CQ, NXB * NYS * imgs_per_group);
  float* tmp = workspace + (size_t)G * P * C * 10;
  CMX_DISPATCH(dtype, T, {
    CMX_ACT_DISPATCH(act, A, {
      hipLaunchKernelGGL((dw_bwd_dz_kernel<T, A>), dim3(cdiv((long)CQ * P, 256), G), dim3(256), 0, s, (const T*)da,
                         (const T*)h, w, b, (T*)dz, workspace, imgs_per_group, H, W, C, NXB, NYS, P);
    });
    if (dh) {
      const long threads = (long)CQ * NXS * NYS * imgs_per_group;
      hipLaunchKernelGGL((dw_fwd_kernel<T, true, 0>), dim3(cdiv(threads, 256), G), dim3(256), 0, s, (const T*)dz, w,
                         (const float*)nullptr, (T*)dh, imgs_per_group, H, W, C, NXS, NYS);
    }
  });
  int st = cmx_reduce_partials(workspace, tmp, G, P, C * 10, 0, 1.f, s);
  if (st) return st;
  const long tot = (long)G * C * 10;
  hipLaunchKernelGGL(dw_scatter_kernel, dim3(cdiv(tot, 256) < 4096 ? cdiv(tot, 256) : 4096), dim3(256), 0, s, tmp, dw,
                     db, G, C, accumulate);
  return cmx_check_launch("dwconv_bwd");
}

}  // extern "C"
