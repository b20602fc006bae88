// FFM cross-attention (efficient / linear attention) of CrossAttention.forward
// (net_utils.py:199-214), on the MFMA GEMM:
//   ctx_g = softmax_{dim=-2}( k_g^T v_g * d^-1/2 )      (a d x d matrix per (b, head))
//   out_1 = q_1 @ ctx_2 ,  out_2 = q_2 @ ctx_1         (contexts crossed between modalities)
// q is the raw (ReLU'd) channel_proj half u, k / v the two halves of the kv projection.
//
// The token contractions are batched bf16 MFMA GEMMs over (g, b) = one (C x C) product per image
// and modality (functions.CrossAttentionF):  KV = k^T v (fp32), out = u @ BD^T,  and in the
// backward du = dout @ BD, dBD = u^T dout (fp32), dk = v @ dA^T, dv = k @ dA.  Taking all C x C
// products instead of the heads' d x d diagonal blocks costs heads x the MACs of those blocks --
// at most 2 x 300 x 512 x 512 per image (stage 4) -- and turns the per-head skinny products into
// plain batched GEMMs with K = C.  This file holds the two small kernels in between:
//  ffm_ctx_fwd : the heads' diagonal blocks of KV -> scale, softmax over dim -2 -> ctx (fp32,
//                saved) and the block-diagonal operand BDt of the OTHER modality's out GEMM
//                (BDt[h d + j][h d + i] = ctx[i][j], zeros off the diagonal blocks)
//  ffm_ctx_bwd : dctx (the diagonal blocks of dBD of the consuming modality) -> softmax backward
//                -> dA = scale * ctx * (dctx - colsum(ctx * dctx)) as a block-diagonal operand
// One workgroup per (g, b, head); each writes the d rows of its head in the C x C operand, the
// zeros included, so no memset launch is needed.
#include "cmx_common.h"

namespace {

// rows i of column j split over RG = 256 / D row groups
template <typename T, int D>
__global__ __launch_bounds__(256) void ffm_ctx_fwd_kernel(const float* __restrict__ kv, float* __restrict__ ctx,
                                                          T* __restrict__ bdt, int B, int heads, float scale) {
  constexpr int RG = 256 / D, RPT = D / RG;
  __shared__ float part[2][RG][D];
  const int C = heads * D;
  const int src = blockIdx.x / heads, head = blockIdx.x % heads;     // src = g * B + b
  const int g = src / B, b = src % B;
  const int dst = (1 - g) * B + b;                                   // the modality that consumes it
  const int j = threadIdx.x % D, rg = threadIdx.x / D;
  const float* m = kv + (long)src * C * C + (long)head * D * C + head * D;
  float v[RPT];
  float mx = -INFINITY;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    v[r] = m[(long)(rg * RPT + r) * C + j] * scale;
    mx = fmaxf(mx, v[r]);
  }
  part[0][rg][j] = mx;
  __syncthreads();
  mx = part[0][0][j];
#pragma unroll
  for (int q = 1; q < RG; ++q) mx = fmaxf(mx, part[0][q][j]);
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    v[r] = __expf(v[r] - mx);
    s += v[r];
  }
  part[1][rg][j] = s;
  __syncthreads();
  s = 0.f;
#pragma unroll
  for (int q = 0; q < RG; ++q) s += part[1][q][j];
  const float inv = 1.f / s;
  float* c = ctx + ((long)src * heads + head) * D * D;
  T* o = bdt + (long)dst * C * C;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int i = rg * RPT + r;
    const float p = v[r] * inv;
    c[i * D + j] = p;
    o[(long)(head * D + j) * C + head * D + i] = from_f32<T>(p);
  }
  // the rest of this head's D rows of BDt: zeros
  for (int e = threadIdx.x; e < D * (C - D); e += 256) {
    const int row = e / (C - D), col = e % (C - D);
    const int cc = col < head * D ? col : col + D;
    o[(long)(head * D + row) * C + cc] = from_f32<T>(0.f);
  }
}

// dA[i][j] = scale * P[i][j] * (dP[i][j] - sum_i' P[i'][j] dP[i'][j]); dP = dBD of the consumer
template <typename T, int D>
__global__ __launch_bounds__(256) void ffm_ctx_bwd_kernel(const float* __restrict__ ctx, const float* __restrict__ dbd,
                                                          T* __restrict__ da, int B, int heads, float scale) {
  constexpr int RG = 256 / D, RPT = D / RG;
  __shared__ float part[RG][D];
  const int C = heads * D;
  const int src = blockIdx.x / heads, head = blockIdx.x % heads;
  const int g = src / B, b = src % B;
  const int dst = (1 - g) * B + b;
  const int j = threadIdx.x % D, rg = threadIdx.x / D;
  const float* P = ctx + ((long)src * heads + head) * D * D;
  const float* dP = dbd + (long)dst * C * C + (long)head * D * C + head * D;
  float p[RPT], dp[RPT];
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int i = rg * RPT + r;
    p[r] = P[i * D + j];
    dp[r] = dP[(long)i * C + j];
    s += p[r] * dp[r];
  }
  part[rg][j] = s;
  __syncthreads();
  s = 0.f;
#pragma unroll
  for (int q = 0; q < RG; ++q) s += part[q][j];
  T* o = da + (long)src * C * C;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int i = rg * RPT + r;
    o[(long)(head * D + i) * C + head * D + j] = from_f32<T>(scale * p[r] * (dp[r] - s));
  }
  for (int e = threadIdx.x; e < D * (C - D); e += 256) {
    const int row = e / (C - D), col = e % (C - D);
    const int cc = col < head * D ? col : col + D;
    o[(long)(head * D + row) * C + cc] = from_f32<T>(0.f);
  }
}

#define FFM_D_DISPATCH(D_, ...)                                                   \
  do {                                                                            \
    if ((D_) == 64) { constexpr int DD = 64; __VA_ARGS__; }                       \
    else if ((D_) == 32) { constexpr int DD = 32; __VA_ARGS__; }                  \
    else if ((D_) == 16) { constexpr int DD = 16; __VA_ARGS__; }                  \
    else { cmx_set_error("ffm_ctx: head dim %d (16, 32 or 64)", (D_)); return CMX_ERR_SHAPE; } \
  } while (0)

}  // namespace

extern "C" {

int cmx_ffm_ctx_fwd(const float* kv, float* ctx, void* bdt, int G, int B, int heads, int D, float scale, int dtype,
                    hipStream_t s) {
  CMX_REQUIRE(G == 2 && B > 0 && heads > 0, CMX_ERR_SHAPE, "ffm_ctx_fwd: G=%d B=%d heads=%d", G, B, heads);
  CMX_DISPATCH(dtype, T, {
    FFM_D_DISPATCH(D, hipLaunchKernelGGL((ffm_ctx_fwd_kernel<T, DD>), dim3(G * B * heads), dim3(256), 0, s, kv, ctx,
                                         (T*)bdt, B, heads, scale));
  });
  return cmx_check_launch("ffm_ctx_fwd");
}

int cmx_ffm_ctx_bwd(const float* ctx, const float* dbd, void* da, int G, int B, int heads, int D, float scale, int dtype,
                    hipStream_t s) {
  CMX_REQUIRE(G == 2 && B > 0 && heads > 0, CMX_ERR_SHAPE, "ffm_ctx_bwd: G=%d B=%d heads=%d", G, B, heads);
  CMX_DISPATCH(dtype, T, {
    FFM_D_DISPATCH(D, hipLaunchKernelGGL((ffm_ctx_bwd_kernel<T, DD>), dim3(G * B * heads), dim3(256), 0, s, ctx, dbd,
                                         (T*)da, B, heads, scale));
  });
  return cmx_check_launch("ffm_ctx_bwd");
}

}  // extern "C"
