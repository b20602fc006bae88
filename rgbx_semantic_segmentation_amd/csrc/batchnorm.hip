// BatchNorm over token-major (M rows x C channels) activations, train and eval.
//
// Replaces nn.BatchNorm2d in ChannelEmbed (channel_embed.4 and norm, eps 1e-5, local
// statistics, net_utils.py:319-329) and the decoder's linear_fuse BN (SyncBatchNorm under
// DDP, eps 1e-3 / momentum 0.1 from init_weight, MLPDecoder.py:51-55, builder.py:204-206).
//
// Statistics are accumulated in fp64 per channel (sum, sum of squares), so the split
// stats -> (optional all-reduce over ranks = SyncBN) -> finalize needs no Welford merge.
// apply: y = act(xhat*gamma + beta + res) * dscale[b, c]   (res: ChannelEmbed's residual
//        branch added after the affine; dscale: Dropout2d keep/(1-p) mask of the decoder)
// backward: g = dy * dscale * act'(pre);  local sums (sum g, sum g*xhat) give dgamma/dbeta
//        (per-rank, averaged by the gradient all-reduce like PyTorch SyncBN); the sums
//        (all-reduced for SyncBN) give dx = gamma*invstd*(g - sum_g/n - xhat*sum_gx/n).
#include "cmx_common.h"

namespace {
// lanes across a row's 16-B channel chunks: TPR = min(32, chunks) rounded up to a power of two,
// so narrow layers (C = 64 bf16: 8 chunks) do not leave 3 of 4 lanes idle; RS = 256 / TPR rows
// in flight per block
int bn_tpr(int chunks) {
  int t = 4;
  while (t < chunks && t < 32) t <<= 1;
  return t;
}

int bn_nblk(long M) {
  long nb = (M + 8 * 16 - 1) / (8 * 16);
  return (int)(nb < 256 ? (nb > 0 ? nb : 1) : 256);
}

template <typename T, int TPR>
__global__ __launch_bounds__(256) void bn_stats_kernel(const T* __restrict__ x, double* __restrict__ ws, long M, int C) {
  constexpr int RS = 256 / TPR;
  constexpr int V = VecT<T>::N;
  __shared__ double red[RS][TPR * V * 2];
  const int lane = threadIdx.x % TPR, slot = threadIdx.x / TPR;
  const int ch = blockIdx.y * TPR + lane;
  const bool live = ch * V < C;
  double s[V], q[V];
#pragma unroll
  for (int j = 0; j < V; ++j) s[j] = q[j] = 0.0;
  if (live) {
    for (long m = (long)blockIdx.x * RS + slot; m < M; m += (long)gridDim.x * RS) {
      float v[V];
      load_vec<T>(x + m * C + ch * V, v);
#pragma unroll
      for (int j = 0; j < V; ++j) { s[j] += v[j]; q[j] += (double)v[j] * v[j]; }
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) { red[slot][lane * V + j] = s[j]; red[slot][TPR * V + lane * V + j] = q[j]; }
  __syncthreads();
  for (int e = threadIdx.x; e < TPR * V * 2; e += 256) {
    double a = 0.0;
    for (int r = 0; r < RS; ++r) a += red[r][e];
    const int half = e / (TPR * V), cc = blockIdx.y * TPR * V + e % (TPR * V);
    if (cc < C) ws[((long)blockIdx.x * 2 + half) * C + cc] = a;
  }
}

// sums (2, C) = sum over blocks of ws (nblk, 2, C); 64 columns x 4 row slices per block
__global__ __launch_bounds__(256) void bn_sum_blocks_kernel(const double* __restrict__ ws, double* __restrict__ sums,
                                                            int nblk, int C) {
  __shared__ double red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + tx;
  double a0 = 0.0, a1 = 0.0;
  if (e < 2 * C) {
    int b = ty;
    for (; b + 4 < nblk; b += 8) { a0 += ws[(long)b * 2 * C + e]; a1 += ws[(long)(b + 4) * 2 * C + e]; }
    for (; b < nblk; b += 4) a0 += ws[(long)b * 2 * C + e];
  }
  red[ty][tx] = a0 + a1;
  __syncthreads();
  if (ty == 0 && e < 2 * C) sums[e] = ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx];
}

__global__ void bn_finalize_kernel(const double* __restrict__ sums, double count, float eps, float momentum,
                                   float* __restrict__ running_mean, float* __restrict__ running_var,
                                   float* __restrict__ mean, float* __restrict__ invstd, int C, int update) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double mu = sums[c] / count;
  double var = sums[C + c] / count - mu * mu;
  if (var < 0) var = 0;
  mean[c] = (float)mu;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (update) {
    const double unb = count > 1 ? var * count / (count - 1) : var;
    running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mu);
    running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
  }
}

__global__ void bn_eval_stats_kernel(const float* __restrict__ rm, const float* __restrict__ rv, float eps,
                                     float* __restrict__ mean, float* __restrict__ invstd, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = rm[c];
  invstd[c] = 1.f / sqrtf(rv[c] + eps);
}

template <typename T>
__device__ __forceinline__ void bn_pre(const T* x, const T* res, const float* mean, const float* invstd,
                                       const float* gamma, const float* beta, long e, int c0, float* xh, float* pre) {
  constexpr int V = VecT<T>::N;
  float v[V], r[V];
  load_vec<T>(x + e, v);
  if (res) load_vec<T>(res + e, r);
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int c = c0 + j;
    xh[j] = (v[j] - mean[c]) * invstd[c];
    pre[j] = xh[j] * gamma[c] + beta[c] + (res ? r[j] : 0.f);
  }
}

template <typename T>
__global__ void bn_apply_kernel(const T* __restrict__ x, const float* __restrict__ mean, const float* __restrict__ invstd,
                                const float* __restrict__ gamma, const float* __restrict__ beta, const T* __restrict__ res,
                                const float* __restrict__ dscale, T* __restrict__ y, long M, int C, long rps, int act) {
  constexpr int V = VecT<T>::N;
  const long nvec = M * C / V;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)nvec; i += gridDim.x * blockDim.x) {
    const int e = i * V;
    const int c0 = e % C;
    float xh[V], pre[V];
    bn_pre<T>(x, res, mean, invstd, gamma, beta, e, c0, xh, pre);
    float o[V];
    const int b = (e / C) / (int)rps;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      o[j] = act_fwd(pre[j], act);
      if (dscale) o[j] *= dscale[b * C + c0 + j];
    }
    store_vec<T>(y + e, o);
  }
}

// partials (nblk, 2, C) doubles of sum g and sum g*xhat
template <typename T, int TPR>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                            const float* __restrict__ mean, const float* __restrict__ invstd,
                                                            const float* __restrict__ gamma, const float* __restrict__ beta,
                                                            const T* __restrict__ res, const float* __restrict__ dscale,
                                                            double* __restrict__ ws, long M, int C, long rps, int act) {
  constexpr int RS = 256 / TPR;
  constexpr int V = VecT<T>::N;
  __shared__ double red[RS][TPR * V * 2];
  const int lane = threadIdx.x % TPR, slot = threadIdx.x / TPR;
  const int ch = blockIdx.y * TPR + lane;
  const bool live = ch * V < C;
  double s[V], q[V];
#pragma unroll
  for (int j = 0; j < V; ++j) s[j] = q[j] = 0.0;
  if (live) {
    const int c0 = ch * V;
    for (long m = (long)blockIdx.x * RS + slot; m < M; m += (long)gridDim.x * RS) {
      const long e = m * C + c0;
      float xh[V], pre[V], d[V];
      bn_pre<T>(x, res, mean, invstd, gamma, beta, e, c0, xh, pre);
      load_vec<T>(dy + e, d);
      const long b = m / rps;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float g = d[j] * act_grad(pre[j], act);
        if (dscale) g *= dscale[b * C + c0 + j];
        s[j] += g;
        q[j] += (double)g * xh[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) { red[slot][lane * V + j] = s[j]; red[slot][TPR * V + lane * V + j] = q[j]; }
  __syncthreads();
  for (int e = threadIdx.x; e < TPR * V * 2; e += 256) {
    double a = 0.0;
    for (int r = 0; r < RS; ++r) a += red[r][e];
    const int half = e / (TPR * V), cc = blockIdx.y * TPR * V + e % (TPR * V);
    if (cc < C) ws[((long)blockIdx.x * 2 + half) * C + cc] = a;
  }
}

__global__ void bn_param_grad_kernel(const double* __restrict__ sums, float* __restrict__ dgamma,
                                     float* __restrict__ dbeta, int C, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float gb = (float)sums[c], gg = (float)sums[C + c];
  if (dbeta) dbeta[c] = accumulate ? dbeta[c] + gb : gb;
  if (dgamma) dgamma[c] = accumulate ? dgamma[c] + gg : gg;
}

template <typename T>
__global__ void bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ x, const float* __restrict__ mean,
                                    const float* __restrict__ invstd, const float* __restrict__ gamma,
                                    const float* __restrict__ beta, const T* __restrict__ res,
                                    const float* __restrict__ dscale, const double* __restrict__ sums, double count,
                                    T* __restrict__ dx, T* __restrict__ dres, long M, int C, long rps, int act,
                                    int training) {
  constexpr int V = VecT<T>::N;
  const long nvec = M * C / V;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)nvec; i += gridDim.x * blockDim.x) {
    const int e = i * V;
    const int c0 = e % C;
    float xh[V], pre[V], d[V], o[V], gr[V];
    bn_pre<T>(x, res, mean, invstd, gamma, beta, e, c0, xh, pre);
    load_vec<T>(dy + e, d);
    const int b = (e / C) / (int)rps;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = c0 + j;
      float g = d[j] * act_grad(pre[j], act);
      if (dscale) g *= dscale[b * C + c];
      gr[j] = g;
      if (training) {
        const float mg = (float)(sums[c] / count), mgx = (float)(sums[C + c] / count);
        o[j] = gamma[c] * invstd[c] * (g - mg - xh[j] * mgx);
      } else {
        o[j] = gamma[c] * invstd[c] * g;
      }
    }
    store_vec<T>(dx + e, o);
    if (dres) store_vec<T>(dres + e, gr);
  }
}

unsigned ew_grid(long nvec) {
  const unsigned g = cdiv(nvec, 256);
  return g < 8192 ? (g ? g : 1) : 8192;
}
}  // namespace

extern "C" {

size_t cmx_bn_workspace(int64_t M, int C) { return (size_t)bn_nblk(M) * 2 * C * sizeof(double); }

// sums (2, C) fp64 = [sum x | sum x^2] over the M local rows
int cmx_bn_stats(const void* x, double* sums, double* workspace, int64_t M, int C, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0 && M > 0, CMX_ERR_SHAPE, "bn_stats: C=%d", C);
  const int nb = bn_nblk(M);
  const int tpr = bn_tpr(C / V);
#define BNS(TP) hipLaunchKernelGGL((bn_stats_kernel<T, TP>), dim3(nb, cdiv(C / V, TP)), dim3(256), 0, s, \
                                   (const T*)x, workspace, (long)M, C)
  CMX_DISPATCH(dtype, T, {
    if (tpr == 4) BNS(4);
    else if (tpr == 8) BNS(8);
    else if (tpr == 16) BNS(16);
    else BNS(32);
  });
#undef BNS
  hipLaunchKernelGGL(bn_sum_blocks_kernel, dim3(cdiv(2 * C, 64)), dim3(256), 0, s, workspace, sums, nb, C);
  return cmx_check_launch("bn_stats");
}

// training: mean/invstd from (possibly all-reduced) sums over `count` rows, running stats
// updated with momentum (unbiased var).  eval (training=0): from running stats.
int cmx_bn_finalize(const double* sums, double count, float eps, float momentum, float* running_mean,
                    float* running_var, float* mean, float* invstd, int C, int training, hipStream_t s) {
  if (training) {
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(cdiv(C, 256)), dim3(256), 0, s, sums, count, eps, momentum,
                       running_mean, running_var, mean, invstd, C, running_mean != nullptr ? 1 : 0);
  } else {
    hipLaunchKernelGGL(bn_eval_stats_kernel, dim3(cdiv(C, 256)), dim3(256), 0, s, running_mean, running_var, eps, mean,
                       invstd, C);
  }
  return cmx_check_launch("bn_finalize");
}

int cmx_bn_apply(const void* x, const float* mean, const float* invstd, const float* gamma, const float* beta,
                 const void* res, const float* dscale, void* y, int64_t M, int C, int64_t rows_per_sample, int act,
                 int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0, CMX_ERR_SHAPE, "bn_apply: C=%d", C);
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(ew_grid(M * C / V)), dim3(256), 0, s, (const T*)x, mean, invstd,
                       gamma, beta, (const T*)res, dscale, (T*)y, (long)M, C, (long)rows_per_sample, act);
  });
  return cmx_check_launch("bn_apply");
}

// sums (2, C) fp64 = [sum g | sum g*xhat] (local); dgamma/dbeta from these local sums
int cmx_bn_bwd_reduce(const void* dy, const void* x, const float* mean, const float* invstd, const float* gamma,
                      const float* beta, const void* res, const float* dscale, double* sums, float* dgamma,
                      float* dbeta, double* workspace, int64_t M, int C, int64_t rows_per_sample, int act,
                      int accumulate, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0 && M > 0, CMX_ERR_SHAPE, "bn_bwd_reduce: C=%d", C);
  const int nb = bn_nblk(M);
  const int tpr = bn_tpr(C / V);
#define BNR(TP) hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, TP>), dim3(nb, cdiv(C / V, TP)), dim3(256), 0, s, \
                                   (const T*)dy, (const T*)x, mean, invstd, gamma, beta, (const T*)res, dscale, \
                                   workspace, (long)M, C, (long)rows_per_sample, act)
  CMX_DISPATCH(dtype, T, {
    if (tpr == 4) BNR(4);
    else if (tpr == 8) BNR(8);
    else if (tpr == 16) BNR(16);
    else BNR(32);
  });
#undef BNR
  hipLaunchKernelGGL(bn_sum_blocks_kernel, dim3(cdiv(2 * C, 64)), dim3(256), 0, s, workspace, sums, nb, C);
  hipLaunchKernelGGL(bn_param_grad_kernel, dim3(cdiv(C, 256)), dim3(256), 0, s, sums, dgamma, dbeta, C, accumulate);
  return cmx_check_launch("bn_bwd_reduce");
}

// dx from (global) sums over `count` rows; dres (optional) = grad of the pre-activation
int cmx_bn_bwd_apply(const void* dy, const void* x, const float* mean, const float* invstd, const float* gamma,
                     const float* beta, const void* res, const float* dscale, const double* sums, double count,
                     void* dx, void* dres, int64_t M, int C, int64_t rows_per_sample, int act, int training, int dtype,
                     hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0, CMX_ERR_SHAPE, "bn_bwd_apply: C=%d", C);
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(ew_grid(M * C / V)), dim3(256), 0, s, (const T*)dy, (const T*)x,
                       mean, invstd, gamma, beta, (const T*)res, dscale, sums, count, (T*)dx, (T*)dres, (long)M, C,
                       (long)rows_per_sample, act, training);
  });
  return cmx_check_launch("bn_bwd_apply");
}

}  // extern "C"
