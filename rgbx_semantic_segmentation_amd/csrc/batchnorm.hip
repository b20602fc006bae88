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
//
// Launch shape: the row reductions keep 4 rows' loads in flight per lane (a 2-4 us HBM latency
// per dependent load otherwise bounds them); the per-block partials are folded by one
// 1024-lane kernel that also finalizes (mean / invstd / running stats) or writes the
// parameter gradients; the elementwise passes stage per-channel coefficients in LDS once
// per block (no per-element fp64 divide or scalar parameter loads).
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

// row blocks of the reduce passes: ~16 rows each, at most 256 (the grid is this x the channel
// blocks; more blocks only lengthen the fp64 fold).  The small maps (stage-3/4 FFM BNs:
// M = 600 .. 2400 rows) then spread over 38 .. 150 row blocks instead of 5 .. 19 whose few
// lanes walked all rows serially (bn_bwd_reduce 600 x 512: 21 -> 12 us, 2400 x 320: 22 -> 13).
int bn_nblk(long M) {
  static int& cap = cmx_knob("BN_NBLK", 256);      // row blocks at most (A/B knob)
  long nb = (M + 15) / 16;
  return (int)(nb < cap ? (nb > 0 ? nb : 1) : cap);
}

constexpr int UNR = 4;            // rows per lane with loads in flight together
constexpr int UNRB = 2;           // ... in bn_bwd_reduce_kernel (four operands per row)
constexpr int BN_MAXC = 2048;     // LDS coefficient staging limit of the elementwise passes

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
    const long stride = (long)gridDim.x * RS;
    for (long m = (long)blockIdx.x * RS + slot; m < M; m += UNR * stride) {
      // the UNR rows as raw vectors first, unpacked after (all UNR loads in flight: a load_vec per
      // row, and before that a load inside `if (mu < M)`, was one round trip per row)
      typename VecT<T>::raw raw[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const long mu = m + u * stride;
        raw[u] = load_raw<T>(x + (mu < M ? mu * C : 0) + ch * V);
      }
      float v[UNR][V];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        unpack_raw<T>(raw[u], v[u]);
#pragma unroll
        for (int j = 0; j < V; ++j) v[u][j] = m + u * stride < M ? v[u][j] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u)
#pragma unroll
        for (int j = 0; j < V; ++j) { s[j] += v[u][j]; q[j] += (double)v[u][j] * v[u][j]; }
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

// what the block-partials fold does with the (2, C) sums besides storing them
struct BnFold {
  int mode;                        // 0: sums only; 1: + finalize (forward); 2: + dgamma / dbeta (backward)
  double count;
  float eps, momentum;
  float *running_mean, *running_var, *mean, *invstd;
  float *dgamma, *dbeta;
  int accumulate;
};

// sums (2, C) = sum over blocks of ws (nblk, 2, C).  A block owns 32 channels (both halves:
// lanes tx < 32 sum column c, lanes tx >= 32 column C + c) and 16 row slices of the partials,
// 4 independent loads in flight per lane; then the channel's epilogue per BnFold.
__global__ __launch_bounds__(1024) void bn_fold_kernel(const double* __restrict__ ws, double* __restrict__ sums,
                                                      int nblk, int C, BnFold f) {
  __shared__ double red[16][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 32 + (tx & 31);
  const int e = (tx < 32 ? 0 : C) + c;
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  if (c < C) {
    int b = ty;
    // 16 independent loads in flight per lane: a 256-block fold is one round trip, not four
    // (18 folds per B2 step: 111 -> 96-100 us)
    for (; b + 240 < nblk; b += 256) {
      double t[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) t[u] = ws[(long)(b + 16 * u) * 2 * C + e];
#pragma unroll
      for (int u = 0; u < 16; ++u) a[u & 3] += t[u];
    }
    for (; b + 48 < nblk; b += 64) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += ws[(long)(b + 16 * u) * 2 * C + e];
    }
    for (; b < nblk; b += 16) a[0] += ws[(long)b * 2 * C + e];
  }
  red[ty][tx] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (ty != 0) return;
  double t = 0.0;
#pragma unroll
  for (int r = 0; r < 16; ++r) t += red[r][tx];
  const double t2 = __shfl(t, (tx + 32) & 63);      // lane tx < 32: the sum of column C + c
  if (c >= C) return;
  sums[e] = t;
  if (tx >= 32) return;
  const double s1 = t, s2 = t2;
  if (f.mode == 1) {
    const double mu = s1 / f.count;
    double var = s2 / f.count - mu * mu;
    if (var < 0) var = 0;
    f.mean[c] = (float)mu;
    f.invstd[c] = (float)(1.0 / sqrt(var + (double)f.eps));
    if (f.running_mean) {
      const double unb = f.count > 1 ? var * f.count / (f.count - 1) : var;
      f.running_mean[c] = (float)((1.0 - f.momentum) * f.running_mean[c] + f.momentum * mu);
      f.running_var[c] = (float)((1.0 - f.momentum) * f.running_var[c] + f.momentum * unb);
    }
  } else if (f.mode == 2) {
    const float gb = (float)s1, gg = (float)s2;
    if (f.dbeta) f.dbeta[c] = f.accumulate ? f.dbeta[c] + gb : gb;
    if (f.dgamma) f.dgamma[c] = f.accumulate ? f.dgamma[c] + gg : gg;
  }
}

int launch_fold(const double* ws, double* sums, int nblk, int C, const BnFold& f, hipStream_t s) {
  hipLaunchKernelGGL(bn_fold_kernel, dim3(cdiv(C, 32)), dim3(1024), 0, s, ws, sums, nblk, C, f);
  return 0;
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

// 8 (bf16) / 4 (fp32) consecutive floats of an LDS or global array
template <int V>
__device__ __forceinline__ void ld_coef(const float* p, float* o) {
#pragma unroll
  for (int j = 0; j < V; j += 4) {
    const float4 t = *reinterpret_cast<const float4*>(p + j);
    o[j] = t.x; o[j + 1] = t.y; o[j + 2] = t.z; o[j + 3] = t.w;
  }
}

// y = act(x*sc + sh + res) * dscale, sc = gamma*invstd, sh = beta - mean*sc (LDS per block)
template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(const T* __restrict__ x, const float* __restrict__ mean,
                                                       const float* __restrict__ invstd, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, const T* __restrict__ res,
                                                       const float* __restrict__ dscale, T* __restrict__ y, long M,
                                                       int C, long rps, int act) {
  constexpr int V = VecT<T>::N;
  extern __shared__ float sp[];
  float* ssc = sp;
  float* ssh = sp + C;
  const int nvec = (int)(M * C / V), stride = gridDim.x * blockDim.x;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  // the first vector's loads go out before the coefficient prologue and its barrier (they
  // were a second memory round trip after it), each later one before the previous store
  using Raw = typename VecT<T>::raw;
  const T* rp = res ? res : x;                                   // (an absent residual: unused)
  Raw xr = load_raw<T>(x + (i < nvec ? (long)i * V : 0)), rr = load_raw<T>(rp + (i < nvec ? (long)i * V : 0));
  for (int c = threadIdx.x; c < C; c += 256) {
    const float sc = gamma[c] * invstd[c];
    ssc[c] = sc;
    ssh[c] = beta[c] - mean[c] * sc;
  }
  __syncthreads();
  for (; i < nvec; i += stride) {
    const int e = i * V;
    const int c0 = e % C;
    float v[V], r[V], sc[V], sh[V], ds[V];
    unpack_raw<T>(xr, v);
    unpack_raw<T>(rr, r);
    ld_coef<V>(ssc + c0, sc);
    ld_coef<V>(ssh + c0, sh);
    if (dscale) ld_coef<V>(dscale + (long)((e / C) / (int)rps) * C + c0, ds);
    float o[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      o[j] = act_fwd(v[j] * sc[j] + sh[j] + (res ? r[j] : 0.f), act);
      if (dscale) o[j] *= ds[j];
    }
    const long nx = i + stride < nvec ? (long)(i + stride) * V : 0;
    xr = load_raw<T>(x + nx);
    rr = load_raw<T>(rp + nx);
    store_vec<T>(y + e, o);
  }
}

// partials (nblk, 2, C) doubles of sum g and sum g*xhat
// (two rows per lane in flight, not UNR = 4: with the residual and Dropout2d operands the
// four-row form held 256 VGPRs -- one wave per SIMD)
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
  // a lane sums its ~M / (nblk * RS) <= ~10 rows in fp32 (centred terms: no cancellation);
  // the block and grid partials are fp64
  float s[V], q[V];
#pragma unroll
  for (int j = 0; j < V; ++j) s[j] = q[j] = 0.f;
  if (live) {
    const int c0 = ch * V;
    float mu[V], is[V], sc[V], sh[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      mu[j] = mean[c0 + j];
      is[j] = invstd[c0 + j];
      sc[j] = gamma[c0 + j] * is[j];
      sh[j] = beta[c0 + j] - mu[j] * sc[j];
    }
    const long stride = (long)gridDim.x * RS;
    for (long m = (long)blockIdx.x * RS + slot; m < M; m += UNRB * stride) {
      float xv[UNRB][V], d[UNRB][V], r[UNRB][V], ds[UNRB][V];
#pragma unroll
      for (int u = 0; u < UNRB; ++u) {
        const long mu_ = m + u * stride;
        const bool ok = mu_ < M;
        const long e = mu_ * C + c0;
        // unconditional loads of clamped rows (all UNRB rows' operands in flight together); an
        // absent residual re-reads dy (from cache) and is not used
        load_vec_if<T>(x, e, c0, ok, xv[u]);
        load_vec_if<T>(dy, e, c0, ok, d[u]);
        load_vec_if<T>(res ? res : dy, e, c0, ok, r[u]);
        if (dscale) ld_coef<V>(dscale + ((ok ? mu_ : 0) / rps) * C + c0, ds[u]);
        else {
#pragma unroll
          for (int j = 0; j < V; ++j) ds[u][j] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < UNRB; ++u)
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float pre = xv[u][j] * sc[j] + sh[j] + (res ? r[u][j] : 0.f);
          float g = d[u][j] * act_grad(pre, act);
          if (dscale) g *= ds[u][j];
          s[j] += g;
          q[j] += g * ((xv[u][j] - mu[j]) * is[j]);
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

// dx = sc*(g - mg - xhat*mgx) (training) or sc*g (eval); per-channel mean, invstd, sc, sh,
// mg = sum_g/n and mgx = sum_gx/n staged in LDS once per block
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                           const float* __restrict__ mean, const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma, const float* __restrict__ beta,
                                                           const T* __restrict__ res, const float* __restrict__ dscale,
                                                           const double* __restrict__ sums, double rcount,
                                                           T* __restrict__ dx, T* __restrict__ dres, long M, int C,
                                                           long rps, int act, int training) {
  constexpr int V = VecT<T>::N;
  extern __shared__ float sp[];
  float *smu = sp, *sis = sp + C, *ssc = sp + 2 * C, *ssh = sp + 3 * C, *smg = sp + 4 * C, *smx = sp + 5 * C;
  const int nvec = (int)(M * C / V), stride = gridDim.x * blockDim.x;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  // the first vector's loads before the coefficient prologue (as bn_apply_kernel)
  using Raw = typename VecT<T>::raw;
  const T* rp = res ? res : dy;                                  // (an absent residual: unused)
  const long f0 = i < nvec ? (long)i * V : 0;
  Raw xr = load_raw<T>(x + f0), dr = load_raw<T>(dy + f0), rr = load_raw<T>(rp + f0);
  for (int c = threadIdx.x; c < C; c += 256) {
    const float is = invstd[c], sc = gamma[c] * is;
    smu[c] = mean[c];
    sis[c] = is;
    ssc[c] = sc;
    ssh[c] = beta[c] - mean[c] * sc;
    smg[c] = training ? (float)(sums[c] * rcount) : 0.f;
    smx[c] = training ? (float)(sums[C + c] * rcount) : 0.f;
  }
  __syncthreads();
  for (; i < nvec; i += stride) {
    const int e = i * V;
    const int c0 = e % C;
    float xv[V], d[V], r[V], ds[V], mu[V], is[V], sc[V], sh[V], mg[V], mx[V];
    unpack_raw<T>(xr, xv);
    unpack_raw<T>(dr, d);
    unpack_raw<T>(rr, r);
    if (dscale) ld_coef<V>(dscale + (long)((e / C) / (int)rps) * C + c0, ds);
    ld_coef<V>(smu + c0, mu);
    ld_coef<V>(sis + c0, is);
    ld_coef<V>(ssc + c0, sc);
    ld_coef<V>(ssh + c0, sh);
    ld_coef<V>(smg + c0, mg);
    ld_coef<V>(smx + c0, mx);
    float o[V], gr[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float pre = xv[j] * sc[j] + sh[j] + (res ? r[j] : 0.f);
      float g = d[j] * act_grad(pre, act);
      if (dscale) g *= ds[j];
      gr[j] = g;
      o[j] = sc[j] * (g - mg[j] - (xv[j] - mu[j]) * is[j] * mx[j]);
    }
    const long nx = i + stride < nvec ? (long)(i + stride) * V : 0;
    xr = load_raw<T>(x + nx);
    dr = load_raw<T>(dy + nx);
    rr = load_raw<T>(rp + nx);
    store_vec<T>(dx + e, o);
    if (dres) store_vec<T>(dres + e, gr);
  }
}

// ---------------------------------------------------------------- small maps, one launch
// Small local-statistics BatchNorms (the stage-4 ChannelEmbed BNs, 600 rows): a workgroup of 1024
// lanes owns BS_SC = 16 channels over ALL rows, so the statistics, the finalize and the apply
// (forward), or both backward sums, dgamma / dbeta and dx (backward), are one launch instead of
// three (each of which costs ~5 us of latency at these sizes).  Lanes: TPR = 16 / V per row, two
// rows' loads in flight per lane; a wave folds its rows by xor-shuffles, the block folds its 16
// waves in LDS.  fp64 sums as the multi-launch path (different order: the fp64 sums agree to
// rounding).  Measured (bench_ops.py bnsmall): 600 x 512 forward 11.9 vs 20.2 us, backward 12.9
// vs 21.2; at 2400 x 320 the 20 workgroups' row chains lose (15.3 / 19.1 vs 18.2 / 20.4, and one
// 8-channel chunk per workgroup was slower still: 15.9 / 22.7), hence CMX_BN_SMALL_M = 600.
constexpr int BS_NT = 1024, BS_SC = 16;

template <int TPR>
__device__ __forceinline__ double wave_fold_rows(double v) {
#pragma unroll
  for (int o = TPR; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__global__ __launch_bounds__(BS_NT) void bn_small_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta,
                                                             const float* __restrict__ dscale, T* __restrict__ y,
                                                             double* __restrict__ sums, float* __restrict__ mean,
                                                             float* __restrict__ invstd, float* __restrict__ rmean,
                                                             float* __restrict__ rvar, long M, int C, long rps,
                                                             int act, float eps, float momentum) {
  constexpr int V = VecT<T>::N, TPR = BS_SC / V, RS = BS_NT / TPR, NW = BS_NT / 64;
  __shared__ double part[NW][2 * BS_SC];
  __shared__ float coef[2][BS_SC];
  const int lane = threadIdx.x % TPR, row = threadIdx.x / TPR, w = threadIdx.x >> 6;
  const int c0 = blockIdx.x * BS_SC + lane * V;
  double s[V], q[V];
#pragma unroll
  for (int j = 0; j < V; ++j) s[j] = q[j] = 0.0;
  for (long m = row; m < M; m += 2 * RS) {
    float v[2][V];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (m + u * RS < M) load_vec<T>(x + (m + u * RS) * C + c0, v[u]);
      else
#pragma unroll
        for (int j = 0; j < V; ++j) v[u][j] = 0.f;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < V; ++j) { s[j] += v[u][j]; q[j] += (double)v[u][j] * v[u][j]; }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) {
    s[j] = wave_fold_rows<TPR>(s[j]);
    q[j] = wave_fold_rows<TPR>(q[j]);
  }
  if ((threadIdx.x & 63) < TPR)
#pragma unroll
    for (int j = 0; j < V; ++j) { part[w][lane * V + j] = s[j]; part[w][BS_SC + lane * V + j] = q[j]; }
  __syncthreads();
  if (threadIdx.x < BS_SC) {
    const int c = blockIdx.x * BS_SC + threadIdx.x;
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int i = 0; i < NW; ++i) { s1 += part[i][threadIdx.x]; s2 += part[i][BS_SC + threadIdx.x]; }
    sums[c] = s1;
    sums[C + c] = s2;
    const double cnt = (double)M, mu = s1 / cnt;
    double var = s2 / cnt - mu * mu;
    if (var < 0) var = 0;
    const float is = (float)(1.0 / sqrt(var + (double)eps));
    mean[c] = (float)mu;
    invstd[c] = is;
    if (rmean) {
      const double unb = cnt > 1 ? var * cnt / (cnt - 1) : var;
      rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mu);
      rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unb);
    }
    const float sc = gamma[c] * is;
    coef[0][threadIdx.x] = sc;
    coef[1][threadIdx.x] = beta[c] - (float)mu * sc;
  }
  __syncthreads();
  float sc[V], sh[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { sc[j] = coef[0][lane * V + j]; sh[j] = coef[1][lane * V + j]; }
  for (long m0 = row; m0 < M; m0 += 2 * RS) {
    float v[2][V], r[2][V], ds[2][V];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long m = m0 + u * RS;
      if (m < M) {
        load_vec<T>(x + m * C + c0, v[u]);
        if (res) load_vec<T>(res + m * C + c0, r[u]);
        if (dscale) ld_coef<V>(dscale + (m / rps) * C + c0, ds[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long m = m0 + u * RS;
      if (m >= M) continue;
      float o[V];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        o[j] = act_fwd(v[u][j] * sc[j] + sh[j] + (res ? r[u][j] : 0.f), act);
        if (dscale) o[j] *= ds[u][j];
      }
      store_vec<T>(y + m * C + c0, o);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(BS_NT) void bn_small_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, const T* __restrict__ res,
                                                             const float* __restrict__ dscale,
                                                             float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                             T* __restrict__ dx, T* __restrict__ dres, long M, int C,
                                                             long rps, int act, int accumulate) {
  constexpr int V = VecT<T>::N, TPR = BS_SC / V, RS = BS_NT / TPR, NW = BS_NT / 64;
  __shared__ double part[NW][2 * BS_SC];
  __shared__ float coef[2][BS_SC];
  const int lane = threadIdx.x % TPR, row = threadIdx.x / TPR, w = threadIdx.x >> 6;
  const int c0 = blockIdx.x * BS_SC + lane * V;
  float mu[V], is[V], sc[V], sh[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    mu[j] = mean[c0 + j];
    is[j] = invstd[c0 + j];
    sc[j] = gamma[c0 + j] * is[j];
    sh[j] = beta[c0 + j] - mu[j] * sc[j];
  }
  double s[V], q[V];
#pragma unroll
  for (int j = 0; j < V; ++j) s[j] = q[j] = 0.0;
  for (long m = row; m < M; m += RS) {
    const long e = m * C + c0;
    float xv[V], d[V], r[V], ds[V];
    load_vec<T>(x + e, xv);
    load_vec<T>(dy + e, d);
    if (res) load_vec<T>(res + e, r);
    if (dscale) ld_coef<V>(dscale + (m / rps) * C + c0, ds);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float g = d[j] * act_grad(xv[j] * sc[j] + sh[j] + (res ? r[j] : 0.f), act);
      if (dscale) g *= ds[j];
      s[j] += g;
      q[j] += (double)g * ((xv[j] - mu[j]) * is[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) {
    s[j] = wave_fold_rows<TPR>(s[j]);
    q[j] = wave_fold_rows<TPR>(q[j]);
  }
  if ((threadIdx.x & 63) < TPR)
#pragma unroll
    for (int j = 0; j < V; ++j) { part[w][lane * V + j] = s[j]; part[w][BS_SC + lane * V + j] = q[j]; }
  __syncthreads();
  if (threadIdx.x < BS_SC) {
    const int c = blockIdx.x * BS_SC + threadIdx.x;
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int i = 0; i < NW; ++i) { s1 += part[i][threadIdx.x]; s2 += part[i][BS_SC + threadIdx.x]; }
    const float gb = (float)s1, gg = (float)s2;
    if (dbeta) dbeta[c] = accumulate ? dbeta[c] + gb : gb;
    if (dgamma) dgamma[c] = accumulate ? dgamma[c] + gg : gg;
    coef[0][threadIdx.x] = (float)(s1 / (double)M);
    coef[1][threadIdx.x] = (float)(s2 / (double)M);
  }
  __syncthreads();
  float mg[V], mx[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { mg[j] = coef[0][lane * V + j]; mx[j] = coef[1][lane * V + j]; }
  for (long m = row; m < M; m += RS) {
    const long e = m * C + c0;
    float xv[V], d[V], r[V], ds[V], o[V], gr[V];
    load_vec<T>(x + e, xv);
    load_vec<T>(dy + e, d);
    if (res) load_vec<T>(res + e, r);
    if (dscale) ld_coef<V>(dscale + (m / rps) * C + c0, ds);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float g = d[j] * act_grad(xv[j] * sc[j] + sh[j] + (res ? r[j] : 0.f), act);
      if (dscale) g *= ds[j];
      gr[j] = g;
      o[j] = sc[j] * (g - mg[j] - (xv[j] - mu[j]) * is[j] * mx[j]);
    }
    store_vec<T>(dx + e, o);
    if (dres) store_vec<T>(dres + e, gr);
  }
}

unsigned ew_grid(long nvec) {
  const unsigned g = cdiv(nvec, 256);
  return g < 2048 ? (g ? g : 1) : 2048;
}

template <typename T>
int launch_stats(const void* x, double* workspace, long M, int C, int nb, hipStream_t s) {
  constexpr int V = VecT<T>::N;
  const int tpr = bn_tpr(C / V);
#define BNS(TP) hipLaunchKernelGGL((bn_stats_kernel<T, TP>), dim3(nb, cdiv(C / V, TP)), dim3(256), 0, s, \
                                   (const T*)x, workspace, M, C)
  if (tpr == 4) BNS(4);
  else if (tpr == 8) BNS(8);
  else if (tpr == 16) BNS(16);
  else BNS(32);
#undef BNS
  return 0;
}
}  // namespace

extern "C" {

size_t cmx_bn_workspace(int64_t M, int C) { return (size_t)bn_nblk(M) * 2 * C * sizeof(double); }

// sums (2, C) fp64 = [sum x | sum x^2] over the M local rows
int cmx_bn_stats(const void* x, double* sums, double* workspace, int64_t M, int C, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0 && M > 0, CMX_ERR_SHAPE, "bn_stats: C=%d", C);
  const int nb = bn_nblk(M);
  CMX_DISPATCH(dtype, T, { launch_stats<T>(x, workspace, (long)M, C, nb, s); });
  BnFold f{};
  launch_fold(workspace, sums, nb, C, f, s);
  return cmx_check_launch("bn_stats");
}

// local statistics in two launches: the row reduction, then the fold that also finalizes
// (mean / invstd, running stats with momentum and the unbiased variance) -- BatchNorm2d
// training forward without a SyncBN exchange between the sums and the finalize
int cmx_bn_stats_finalize(const void* x, double* sums, double* workspace, int64_t M, int C, float eps, float momentum,
                          float* running_mean, float* running_var, float* mean, float* invstd, int dtype,
                          hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0 && M > 0, CMX_ERR_SHAPE, "bn_stats_finalize: C=%d", C);
  const int nb = bn_nblk(M);
  CMX_DISPATCH(dtype, T, { launch_stats<T>(x, workspace, (long)M, C, nb, s); });
  BnFold f{};
  f.mode = 1; f.count = (double)M; f.eps = eps; f.momentum = momentum;
  f.running_mean = running_mean; f.running_var = running_var; f.mean = mean; f.invstd = invstd;
  launch_fold(workspace, sums, nb, C, f, s);
  return cmx_check_launch("bn_stats_finalize");
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
  CMX_REQUIRE(C % V == 0 && C <= BN_MAXC, CMX_ERR_SHAPE, "bn_apply: C=%d", C);
  CMX_REQUIRE(!dscale || ((uintptr_t)dscale & 15) == 0, CMX_ERR_ARG, "bn_apply: dscale alignment");
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(ew_grid(M * C / V)), dim3(256), 2 * C * sizeof(float), s,
                       (const T*)x, mean, invstd, gamma, beta, (const T*)res, dscale, (T*)y, (long)M, C,
                       (long)rows_per_sample, act);
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
  CMX_REQUIRE(!dscale || ((uintptr_t)dscale & 15) == 0, CMX_ERR_ARG, "bn_bwd_reduce: dscale alignment");
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
  BnFold f{};
  f.mode = 2; f.dgamma = dgamma; f.dbeta = dbeta; f.accumulate = accumulate;
  launch_fold(workspace, sums, nb, C, f, s);
  return cmx_check_launch("bn_bwd_reduce");
}

// dx from (global) sums over `count` rows; dres (optional) = grad of the pre-activation
int cmx_bn_bwd_apply(const void* dy, const void* x, const float* mean, const float* invstd, const float* gamma,
                     const float* beta, const void* res, const float* dscale, const double* sums, double count,
                     void* dx, void* dres, int64_t M, int C, int64_t rows_per_sample, int act, int training, int dtype,
                     hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0 && C <= BN_MAXC, CMX_ERR_SHAPE, "bn_bwd_apply: C=%d", C);
  CMX_REQUIRE(!dscale || ((uintptr_t)dscale & 15) == 0, CMX_ERR_ARG, "bn_bwd_apply: dscale alignment");
  CMX_REQUIRE(!training || count > 0, CMX_ERR_ARG, "bn_bwd_apply: count");
  const double rcount = training ? 1.0 / count : 0.0;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(ew_grid(M * C / V)), dim3(256), 6 * C * sizeof(float), s,
                       (const T*)dy, (const T*)x, mean, invstd, gamma, beta, (const T*)res, dscale, sums, rcount,
                       (T*)dx, (T*)dres, (long)M, C, (long)rows_per_sample, act, training);
  });
  return cmx_check_launch("bn_bwd_apply");
}

// the small-map forms (local statistics, training): C % 16 == 0, one launch each
int cmx_bn_small_fwd(const void* x, const void* res, const float* gamma, const float* beta, const float* dscale,
                     void* y, double* sums, float* mean, float* invstd, float* running_mean, float* running_var,
                     int64_t M, int C, int64_t rows_per_sample, int act, float eps, float momentum, int dtype,
                     hipStream_t s) {
  CMX_REQUIRE(M > 0 && C % BS_SC == 0 && (!dscale || ((uintptr_t)dscale & 15) == 0), CMX_ERR_SHAPE,
              "bn_small_fwd: C=%d (a multiple of %d)", C, BS_SC);
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(bn_small_fwd_kernel<T>, dim3(C / BS_SC), dim3(BS_NT), 0, s, (const T*)x, (const T*)res, gamma,
                       beta, dscale, (T*)y, sums, mean, invstd, running_mean, running_var, (long)M, C,
                       (long)rows_per_sample, act, eps, momentum);
  });
  return cmx_check_launch("bn_small_fwd");
}

int cmx_bn_small_bwd(const void* dy, const void* x, const float* mean, const float* invstd, const float* gamma,
                     const float* beta, const void* res, const float* dscale, float* dgamma, float* dbeta, void* dx,
                     void* dres, int64_t M, int C, int64_t rows_per_sample, int act, int accumulate, int dtype,
                     hipStream_t s) {
  CMX_REQUIRE(M > 0 && C % BS_SC == 0 && (!dscale || ((uintptr_t)dscale & 15) == 0), CMX_ERR_SHAPE,
              "bn_small_bwd: C=%d (a multiple of %d)", C, BS_SC);
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(bn_small_bwd_kernel<T>, dim3(C / BS_SC), dim3(BS_NT), 0, s, (const T*)dy, (const T*)x, mean,
                       invstd, gamma, beta, (const T*)res, dscale, dgamma, dbeta, (T*)dx, (T*)dres, (long)M, C,
                       (long)rows_per_sample, act, accumulate);
  });
  return cmx_check_launch("bn_small_bwd");
}

}  // extern "C"
