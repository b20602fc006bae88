// Improved Feature Rectify Module (config.feature_rectify_module = 'IFRM', net_utils.py:155-180):
// the kernels the existing families do not cover.
//
//   cmx_mul2 / cmx_mul2_bwd     cw = y * sigmoid-gate(y) of ImprovedChannelWeights (:61-63), fp32
//                               (B, 2C) vectors; backward dy = d * g, dg = d * y
//   cmx_rowln_fwd / _bwd        LayerNorm of a few fp32 rows of any width (the channel MLP's
//                               LN(4C) / LN(2C), :42,45: up to 2048 wide, beyond the token LN)
//   cmx_ifrm_combine_fwd/_bwd   the rectification with learnable lambdas and the UN-squashed
//                               spatial logits (:174-175):
//       o1 = x1 + (lc * cw[1] + ls * sw[1]) * x2 ,  o2 = x2 + (lc * cw[0] + ls * sw[0]) * x1
//     x (2, B, N, C) token-major in the compute dtype, cw (B, 2C) fp32 (cw[g] = cw[:, gC:(g+1)C]),
//     sw (B*N, 2) in the compute dtype (conv3 output, channel g = modality g), lc / ls fp32
//     scalars on the device.  Backward: dx directly; dsw per pixel (a wave-reduction over C);
//     dcw and the two lambda gradients as per-block partials (summed by cmx_partials_sum).
//
// Memory-bound (x read, out written; dout + x read, dx written in the backward): one wave per
// pixel at a time, lanes across channels, 16-B vector accesses.
#include "cmx_common.h"

namespace {

__global__ void mul2_kernel(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ o, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) o[i] = a[i] * b[i];
}

__global__ void mul2_bwd_kernel(const float* __restrict__ d, const float* __restrict__ a, const float* __restrict__ b,
                                float* __restrict__ da, float* __restrict__ db, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    da[i] = d[i] * b[i];
    db[i] = d[i] * a[i];
  }
}

// one block per row; two passes over the row (mean, then centred variance), fp32
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void rowln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                        const float* __restrict__ b, float* __restrict__ y,
                                                        float* __restrict__ mean, float* __restrict__ rstd, int C,
                                                        float eps) {
  __shared__ float red[4];
  const float* xr = x + (long)blockIdx.x * C;
  float s = 0.f;
  for (int c = threadIdx.x; c < C; c += 256) s += xr[c];
  const float mu = block_sum(s, red) / C;
  float q = 0.f;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float d = xr[c] - mu;
    q += d * d;
  }
  const float rs = rsqrtf(block_sum(q, red) / C + eps);
  for (int c = threadIdx.x; c < C; c += 256) y[(long)blockIdx.x * C + c] = (xr[c] - mu) * rs * g[c] + b[c];
  if (threadIdx.x == 0) {
    mean[blockIdx.x] = mu;
    rstd[blockIdx.x] = rs;
  }
}

// dx = rstd * (dy*g - mean_c(dy*g) - xhat * mean_c(dy*g*xhat)), one block per row
__global__ __launch_bounds__(256) void rowln_bwd_dx_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                           const float* __restrict__ g, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, float* __restrict__ dx,
                                                           int C) {
  __shared__ float red[4];
  const long o = (long)blockIdx.x * C;
  const float mu = mean[blockIdx.x], rs = rstd[blockIdx.x];
  float s1 = 0.f, s2 = 0.f;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float t = dy[o + c] * g[c];
    s1 += t;
    s2 += t * (x[o + c] - mu) * rs;
  }
  const float m1 = block_sum(s1, red) / C;
  const float m2 = block_sum(s2, red) / C;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float xh = (x[o + c] - mu) * rs;
    dx[o + c] = rs * (dy[o + c] * g[c] - m1 - xh * m2);
  }
}

// dgamma / dbeta: one thread per column, summed over the (few) rows
__global__ void rowln_bwd_dgb_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                     float* __restrict__ dg, float* __restrict__ db, int R, int C) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float a = 0.f, bsum = 0.f;
  for (int r = 0; r < R; ++r) {
    const float d = dy[(long)r * C + c];
    a += d * (x[(long)r * C + c] - mean[r]) * rstd[r];
    bsum += d;
  }
  dg[c] = a;
  db[c] = bsum;
}

constexpr int PPB = 16;                         // pixels per block
constexpr int CMAX = 512;                       // channels (every CMX stage)

template <typename T>
__global__ __launch_bounds__(256) void combine_fwd_kernel(const T* __restrict__ x, const float* __restrict__ cw,
                                                          const T* __restrict__ sw, const float* __restrict__ lc,
                                                          const float* __restrict__ ls, T* __restrict__ out, int B,
                                                          int N, int C) {
  constexpr int V = VecT<T>::N;
  const int nblk = (N + PPB - 1) / PPB;
  const int b = blockIdx.x / nblk, p0 = (blockIdx.x % nblk) * PPB;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float Lc = *lc, Ls = *ls;
  const long plane = (long)B * N * C;
  for (int pp = w; pp < PPB; pp += 4) {
    const int n = p0 + pp;
    if (n >= N) break;
    const long row = (long)b * N + n;
    const float s0 = to_f32(sw[row * 2]), s1 = to_f32(sw[row * 2 + 1]);
    for (int c = lane * V; c < C; c += 64 * V) {
      float a[V], bb[V];
      load_vec<T>(x + row * C + c, a);
      load_vec<T>(x + plane + row * C + c, bb);
      float o1[V], o2[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float k1 = Lc * cw[(long)b * 2 * C + C + c + e] + Ls * s1;     // o1 = x1 + k1 * x2
        const float k0 = Lc * cw[(long)b * 2 * C + c + e] + Ls * s0;         // o2 = x2 + k0 * x1
        o1[e] = a[e] + k1 * bb[e];
        o2[e] = bb[e] + k0 * a[e];
      }
      store_vec<T>(out + row * C + c, o1);
      store_vec<T>(out + plane + row * C + c, o2);
    }
  }
}

// part: per block dcw (2C floats), blocks image-major (B, N / PPB); lpart (2, nblk): dlc, dls
template <typename T>
__global__ __launch_bounds__(256) void combine_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ x,
                                                          const float* __restrict__ cw, const T* __restrict__ sw,
                                                          const float* __restrict__ lc, const float* __restrict__ ls,
                                                          T* __restrict__ dx, T* __restrict__ dsw,
                                                          float* __restrict__ part, float* __restrict__ lpart, int B,
                                                          int N, int C) {
  constexpr int V = VecT<T>::N;
  constexpr int NC = CMAX / (64 * V) > 0 ? CMAX / (64 * V) : 1;   // channel vectors per lane
  __shared__ float red[4][2 * CMAX + 2];
  const int nblk = (N + PPB - 1) / PPB;
  const int b = blockIdx.x / nblk, p0 = (blockIdx.x % nblk) * PPB;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float Lc = *lc, Ls = *ls;
  const long plane = (long)B * N * C;
  // per-lane channel partials: t1[c] = sum_n do1 * x2 (-> dcw[1]), t0[c] = sum_n do2 * x1 (-> dcw[0])
  float t0[NC][V], t1[NC][V];
#pragma unroll
  for (int q = 0; q < NC; ++q)
#pragma unroll
    for (int e = 0; e < V; ++e) t0[q][e] = t1[q][e] = 0.f;
  float gls = 0.f;                               // lambda_spatial partial (lambda_channel from t0 / t1 later)
  for (int pp = w; pp < PPB; pp += 4) {
    const int n = p0 + pp;
    if (n >= N) break;
    const long row = (long)b * N + n;
    const float s0 = to_f32(sw[row * 2]), s1 = to_f32(sw[row * 2 + 1]);
    float r0 = 0.f, r1 = 0.f;                    // sum_c do2 * x1, sum_c do1 * x2
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int c = (q * 64 + lane) * V;
      if (c >= C) break;
      float a[V], bb[V], d1[V], d2[V];
      load_vec<T>(x + row * C + c, a);
      load_vec<T>(x + plane + row * C + c, bb);
      load_vec<T>(dout + row * C + c, d1);
      load_vec<T>(dout + plane + row * C + c, d2);
      float g1[V], g2[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float k1 = Lc * cw[(long)b * 2 * C + C + c + e] + Ls * s1;
        const float k0 = Lc * cw[(long)b * 2 * C + c + e] + Ls * s0;
        g1[e] = d1[e] + k0 * d2[e];              // dx1 = do1 + k0 * do2
        g2[e] = d2[e] + k1 * d1[e];              // dx2 = do2 + k1 * do1
        const float u1 = d1[e] * bb[e], u0 = d2[e] * a[e];
        t1[q][e] += u1;
        t0[q][e] += u0;
        r1 += u1;
        r0 += u0;
      }
      store_vec<T>(dx + row * C + c, g1);
      store_vec<T>(dx + plane + row * C + c, g2);
    }
    r0 = wave_sum(r0);
    r1 = wave_sum(r1);
    if (lane == 0) {
      dsw[row * 2] = from_f32<T>(Ls * r0);
      dsw[row * 2 + 1] = from_f32<T>(Ls * r1);
    }
    gls += s0 * r0 + s1 * r1;                    // wave-uniform after the reductions
  }
  // block partials: dcw[g][c] = lc * sum, dlc = sum_c cw * t, dls = gls
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int c = (q * 64 + lane) * V;
    if (c < C) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        red[w][c + e] = t0[q][e];
        red[w][C + c + e] = t1[q][e];
      }
    }
  }
  if (lane == 0) red[w][2 * C] = gls;
  __syncthreads();
  float* dst = part + (long)blockIdx.x * 2 * C;
  float lcp = 0.f;
  for (int c = threadIdx.x; c < 2 * C; c += 256) {
    const float t = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    dst[c] = Lc * t;
    lcp += cw[(long)b * 2 * C + c] * t;
  }
  lcp = wave_sum(lcp);
  __syncthreads();
  if (lane == 0) red[w][2 * C + 1] = lcp;
  __syncthreads();
  if (threadIdx.x == 0) {
    lpart[blockIdx.x] = red[0][2 * C + 1] + red[1][2 * C + 1] + red[2][2 * C + 1] + red[3][2 * C + 1];
    lpart[gridDim.x + blockIdx.x] = red[0][2 * C] + red[1][2 * C] + red[2][2 * C] + red[3][2 * C];
  }
}

}  // namespace

extern "C" {

int cmx_mul2(const float* a, const float* b, float* out, int64_t n, hipStream_t s) {
  CMX_REQUIRE(n > 0, CMX_ERR_SHAPE, "mul2: n=%ld", (long)n);
  hipLaunchKernelGGL(mul2_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, b, out, (long)n);
  return cmx_check_launch("mul2");
}

int cmx_mul2_bwd(const float* d, const float* a, const float* b, float* da, float* db, int64_t n, hipStream_t s) {
  CMX_REQUIRE(n > 0, CMX_ERR_SHAPE, "mul2_bwd: n=%ld", (long)n);
  hipLaunchKernelGGL(mul2_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d, a, b, da, db, (long)n);
  return cmx_check_launch("mul2_bwd");
}

int cmx_rowln_fwd(const float* x, const float* gamma, const float* beta, float* y, float* mean, float* rstd, int R,
                  int C, float eps, hipStream_t s) {
  CMX_REQUIRE(R > 0 && C > 0, CMX_ERR_SHAPE, "rowln_fwd: R=%d C=%d", R, C);
  hipLaunchKernelGGL(rowln_fwd_kernel, dim3(R), dim3(256), 0, s, x, gamma, beta, y, mean, rstd, C, eps);
  return cmx_check_launch("rowln_fwd");
}

int cmx_rowln_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd, float* dx,
                  float* dgamma, float* dbeta, int R, int C, hipStream_t s) {
  CMX_REQUIRE(R > 0 && C > 0, CMX_ERR_SHAPE, "rowln_bwd: R=%d C=%d", R, C);
  hipLaunchKernelGGL(rowln_bwd_dx_kernel, dim3(R), dim3(256), 0, s, dy, x, gamma, mean, rstd, dx, C);
  hipLaunchKernelGGL(rowln_bwd_dgb_kernel, dim3((C + 255) / 256), dim3(256), 0, s, dy, x, mean, rstd, dgamma, dbeta,
                     R, C);
  return cmx_check_launch("rowln_bwd");
}

int cmx_ifrm_combine_nblk(int B, int N) { return B * ((N + PPB - 1) / PPB); }

int cmx_ifrm_combine_fwd(const void* x, const float* cw, const void* sw, const float* lc, const float* ls, void* out,
                         int B, int N, int C, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(B > 0 && N > 0 && C > 0 && C % V == 0 && C <= CMAX, CMX_ERR_SHAPE, "ifrm_combine: B=%d N=%d C=%d", B,
              N, C);
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(combine_fwd_kernel<T>, dim3(cmx_ifrm_combine_nblk(B, N)), dim3(256), 0, s, (const T*)x, cw,
                       (const T*)sw, lc, ls, (T*)out, B, N, C);
  });
  return cmx_check_launch("ifrm_combine_fwd");
}

int cmx_ifrm_combine_bwd(const void* dout, const void* x, const float* cw, const void* sw, const float* lc,
                         const float* ls, void* dx, void* dsw, float* part, float* lpart, int B, int N, int C,
                         int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(B > 0 && N > 0 && C > 0 && C % V == 0 && C <= CMAX, CMX_ERR_SHAPE, "ifrm_combine: B=%d N=%d C=%d", B,
              N, C);
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(combine_bwd_kernel<T>, dim3(cmx_ifrm_combine_nblk(B, N)), dim3(256), 0, s, (const T*)dout,
                       (const T*)x, cw, (const T*)sw, lc, ls, (T*)dx, (T*)dsw, part, lpart, B, N, C);
  });
  return cmx_check_launch("ifrm_combine_bwd");
}

}  // extern "C"
