// FFM cross-attention (efficient / linear attention) of CrossAttention.forward
// (net_utils.py:199-214), on the MFMA GEMM:
//   ctx_g = softmax_{dim=-2}( k_g^T v_g * d^-1/2 )      (a d x d matrix per (b, head))
//   out_1 = q_1 @ ctx_2 ,  out_2 = q_2 @ ctx_1         (contexts crossed between modalities)
// q is the raw (ReLU'd) channel_proj half u, k / v the two halves of the kv projection.
//
// The token contractions are per-head MFMA GEMMs over (g, b, head) (cmx_gemm_h2, a two-level
// batch: the heads are column slices of each token row): KV_h = k_h^T v_h (d x d, fp32),
// out_h = u_h @ ctx_h, and in the backward du_h = dout_h @ ctx_h^T, dctx_h = u_h^T dout_h (fp32),
// dk_h = v_h @ dA_h^T, dv_h = k_h @ dA_h -- exactly the reference's MACs (functions.py
// _cross_attn_fwd / _bwd).  This file holds the two small kernels in between, one workgroup
// per (g, b, head):
//  ffm_ctx_fwd : KV_h -> scale, softmax over dim -2 -> ctx (fp32, saved) and its transpose in the
//                compute dtype, ctxT, filed under the OTHER modality (the GEMM operand of its out)
//  ffm_ctx_bwd : dctx (of the consuming modality) -> softmax backward
//                -> dA = scale * ctx * (dctx - colsum(ctx * dctx)) in the compute dtype
#include "cmx_common.h"

namespace {

// rows i of column j split over RG = 256 / D row groups
// kv, ctx, ctxT: (2 * B, heads, D, D)
template <typename T, int D>
__global__ __launch_bounds__(256) void ffm_ctx_fwd_kernel(const float* __restrict__ kv, float* __restrict__ ctx,
                                                          T* __restrict__ ctxT, int B, int heads, float scale) {
  constexpr int RG = 256 / D, RPT = D / RG;
  __shared__ float part[2][RG][D];
  const int src = blockIdx.x / heads, head = blockIdx.x % heads;     // src = g * B + b
  const int g = src / B, b = src % B;
  const int dst = (1 - g) * B + b;                                   // the modality that consumes it
  const int j = threadIdx.x % D, rg = threadIdx.x / D;
  const float* m = kv + ((long)src * heads + head) * D * D;
  float v[RPT];
  float mx = -INFINITY;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    v[r] = m[(rg * RPT + r) * D + j] * scale;
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
  T* o = ctxT + ((long)dst * heads + head) * D * D;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int i = rg * RPT + r;
    const float p = v[r] * inv;
    c[i * D + j] = p;
    o[j * D + i] = from_f32<T>(p);
  }
}

// dA[i][j] = scale * P[i][j] * (dP[i][j] - sum_i' P[i'][j] dP[i'][j]); dP = dBD of the consumer
// ctx, dctx, da: (2 * B, heads, D, D); dctx is filed under the consuming modality
template <typename T, int D>
__global__ __launch_bounds__(256) void ffm_ctx_bwd_kernel(const float* __restrict__ ctx, const float* __restrict__ dctx,
                                                          T* __restrict__ da, int B, int heads, float scale) {
  constexpr int RG = 256 / D, RPT = D / RG;
  __shared__ float part[RG][D];
  const int src = blockIdx.x / heads, head = blockIdx.x % heads;
  const int g = src / B, b = src % B;
  const int dst = (1 - g) * B + b;
  const int j = threadIdx.x % D, rg = threadIdx.x / D;
  const float* P = ctx + ((long)src * heads + head) * D * D;
  const float* dP = dctx + ((long)dst * heads + head) * D * D;
  float p[RPT], dp[RPT];
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int i = rg * RPT + r;
    p[r] = P[i * D + j];
    dp[r] = dP[i * D + j];
    s += p[r] * dp[r];
  }
  part[rg][j] = s;
  __syncthreads();
  s = 0.f;
#pragma unroll
  for (int q = 0; q < RG; ++q) s += part[q][j];
  T* o = da + ((long)src * heads + head) * D * D;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int i = rg * RPT + r;
    o[i * D + j] = from_f32<T>(scale * p[r] * (dp[r] - s));
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

int cmx_ffm_ctx_fwd(const float* kv, float* ctx, void* ctxT, int G, int B, int heads, int D, float scale, int dtype,
                    hipStream_t s) {
  CMX_REQUIRE(G == 2 && B > 0 && heads > 0, CMX_ERR_SHAPE, "ffm_ctx_fwd: G=%d B=%d heads=%d", G, B, heads);
  CMX_DISPATCH(dtype, T, {
    FFM_D_DISPATCH(D, hipLaunchKernelGGL((ffm_ctx_fwd_kernel<T, DD>), dim3(G * B * heads), dim3(256), 0, s, kv, ctx,
                                         (T*)ctxT, B, heads, scale));
  });
  return cmx_check_launch("ffm_ctx_fwd");
}

int cmx_ffm_ctx_bwd(const float* ctx, const float* dctx, void* da, int G, int B, int heads, int D, float scale,
                    int dtype, hipStream_t s) {
  CMX_REQUIRE(G == 2 && B > 0 && heads > 0, CMX_ERR_SHAPE, "ffm_ctx_bwd: G=%d B=%d heads=%d", G, B, heads);
  CMX_DISPATCH(dtype, T, {
    FFM_D_DISPATCH(D, hipLaunchKernelGGL((ffm_ctx_bwd_kernel<T, DD>), dim3(G * B * heads), dim3(256), 0, s, ctx, dctx,
                                         (T*)da, B, heads, scale));
  });
  return cmx_check_launch("ffm_ctx_bwd");
}

}  // extern "C"
