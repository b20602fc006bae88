// LayerNorm over the channel dim of token-major activations (G groups of R rows x C).
//
// Replaces nn.LayerNorm at: Block.norm1/norm2 + stage norms (eps 1e-6,
// dual_segformer.py:148,155,257...), OverlapPatchEmbed.norm / Attention.norm (eps 1e-5,
// :198,:97), CrossPath.norm1/2 (eps 1e-5, net_utils.py:270-271).  Group g has its own
// gamma/beta (the RGB and X streams are processed in one launch).
//
// Layout: a row is C contiguous elements; TPR lanes own one row, each lane NCH chunks
// of one 16-byte vector.  HBM-bound: fwd reads x once and writes y once (+8 B/row stats).
#include "cmx_common.h"

// RPT rows per thread, spaced RPB apart: every row's loads are issued before any reduction, so
// a narrow-row launch (C = 64 / 128: one 16-B chunk per lane) keeps RPT loads in flight per lane
template <typename T, int TPR, int NCH, int RPT>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta,
                                                     T* __restrict__ y, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, long R, int C,
                                                     float eps) {
  constexpr int V = VecT<T>::N;
  constexpr int RPB = 256 / TPR;
  const int g = blockIdx.y;
  const int lane = threadIdx.x % TPR;
  const long row0 = (long)blockIdx.x * RPB * RPT + threadIdx.x / TPR;
  const int nchunk = C / V;
  float v[RPT][NCH][V];
#pragma unroll
  for (int u = 0; u < RPT; ++u) {
    const long row = row0 + (long)u * RPB;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int ch = lane + k * TPR;
      if (row < R && ch < nchunk) {
        load_vec<T>(x + ((long)g * R + row) * C + ch * V, v[u][k]);
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) v[u][k][j] = 0.f;
      }
    }
  }
  const float* gg = gamma + (long)g * C;
  const float* bb = beta + (long)g * C;
#pragma unroll
  for (int u = 0; u < RPT; ++u) {
    const long row = row0 + (long)u * RPB;
    const long grow = (long)g * R + row;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
      for (int j = 0; j < V; ++j) s += v[u][k][j];
    s = group_sum(s, TPR);
    const float mu = s / C;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int ch = lane + k * TPR;
      if (ch < nchunk) {
#pragma unroll
        for (int j = 0; j < V; ++j) { float d = v[u][k][j] - mu; q += d * d; }
      }
    }
    q = group_sum(q, TPR);
    const float rstd = rsqrtf(q / C + eps);
    if (row >= R) continue;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int ch = lane + k * TPR;
      if (ch < nchunk) {
        float o[V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const int c = ch * V + j;
          o[j] = (v[u][k][j] - mu) * rstd * gg[c] + bb[c];
        }
        store_vec<T>(y + grow * C + ch * V, o);
      }
    }
    if (lane == 0) {
      if (mean_out) mean_out[grow] = mu;
      if (rstd_out) rstd_out[grow] = rstd;
    }
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma  (+ dres: the gradient
// of a residual branch that bypasses the norm, Block.forward's x + drop_path(...),
// dual_segformer.py:168-169, summed here instead of by a separate add).  dxs (optional) =
// sscale[row / rps] * dx: the DropPath-scaled copy the residual branch's own backward needs.
// Per-block partial column sums of dy*xhat (dgamma) and dy (dbeta) go to ws.
template <typename T, int TPR, int NCH, int RPT>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ rstd,
                                                     T* __restrict__ dx, float* __restrict__ ws,
                                                     long R, int C, const T* __restrict__ dres,
                                                     const float* __restrict__ sscale, T* __restrict__ dxs,
                                                     long rps, const T* __restrict__ dy2) {
  constexpr int V = VecT<T>::N;
  constexpr int RPB = 256 / TPR;
  __shared__ float red[256 / TPR][2][NCH * TPR * V > 512 ? 512 : NCH * TPR * V];
  const int g = blockIdx.y;
  const int lane = threadIdx.x % TPR;
  const int rslot = threadIdx.x / TPR;
  const int nchunk = C / V;
  const float* gg = gamma + (long)g * C;
  float dg[NCH][V], db[NCH][V];
#pragma unroll
  for (int k = 0; k < NCH; ++k)
#pragma unroll
    for (int j = 0; j < V; ++j) dg[k][j] = db[k][j] = 0.f;

  // RPT rows per iteration, all their loads issued before the row reductions
  const long stride = (long)gridDim.x * RPB;
  for (long row0 = (long)blockIdx.x * RPB + rslot; row0 < R; row0 += stride * RPT) {
    float xv[RPT][NCH][V], gv[RPT][NCH][V], dv[RPT][NCH][V];
    float mu[RPT], rs[RPT];
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const long row = row0 + u * stride;
      const bool live = row < R;
      const long grow = (long)g * R + (live ? row : 0);
      mu[u] = live ? mean[grow] : 0.f;
      rs[u] = live ? rstd[grow] : 0.f;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int ch = lane + k * TPR;
        if (live && ch < nchunk) {
          load_vec<T>(x + grow * C + ch * V, xv[u][k]);
          load_vec<T>(dy + grow * C + ch * V, dv[u][k]);
          if (dy2) {              // second consumer of y (q and the SR conv both read norm1's output)
            float d2[V];
            load_vec<T>(dy2 + grow * C + ch * V, d2);
#pragma unroll
            for (int j = 0; j < V; ++j) dv[u][k][j] += d2[j];
          }
        } else {
#pragma unroll
          for (int j = 0; j < V; ++j) xv[u][k][j] = dv[u][k][j] = 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const long row = row0 + u * stride;
      const long grow = (long)g * R + row;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int ch = lane + k * TPR;
        if (ch < nchunk) {
#pragma unroll
          for (int j = 0; j < V; ++j) {
            const float xh = (xv[u][k][j] - mu[u]) * rs[u];
            xv[u][k][j] = xh;
            gv[u][k][j] = dv[u][k][j] * gg[ch * V + j];
            s1 += gv[u][k][j];
            s2 += gv[u][k][j] * xh;
            dg[k][j] += dv[u][k][j] * xh;
            db[k][j] += dv[u][k][j];
          }
        }
      }
      s1 = group_sum(s1, TPR) / C;
      s2 = group_sum(s2, TPR) / C;
      if (row >= R) continue;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int ch = lane + k * TPR;
        if (ch < nchunk) {
          float o[V];
#pragma unroll
          for (int j = 0; j < V; ++j) o[j] = rs[u] * (gv[u][k][j] - s1 - xv[u][k][j] * s2);
          if (dres) {
            float rv[V];
            load_vec<T>(dres + grow * C + ch * V, rv);
#pragma unroll
            for (int j = 0; j < V; ++j) o[j] += rv[j];
          }
          store_vec<T>(dx + grow * C + ch * V, o);
          if (dxs) {
            const float sc = sscale[grow / rps];
#pragma unroll
            for (int j = 0; j < V; ++j) o[j] *= sc;
            store_vec<T>(dxs + grow * C + ch * V, o);
          }
        }
      }
    }
  }
  // block reduction of the column partials over the RPB row slots
  float* out = ws + ((long)g * gridDim.x + blockIdx.x) * 2 * C;
  for (int base = 0; base < C; base += 512) {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int ch = lane + k * TPR;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int c = ch * V + j - base;
        if (ch < nchunk && c >= 0 && c < 512) {
          red[rslot][0][c] = dg[k][j];
          red[rslot][1][c] = db[k][j];
        }
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 512 && base + c < C; c += 256) {
      float a = 0.f, b = 0.f;
      for (int r = 0; r < RPB; ++r) { a += red[r][0][c]; b += red[r][1][c]; }
      out[base + c] = a;
      out[C + base + c] = b;
    }
    __syncthreads();
  }
}

// out[g, w] (+)= alpha * sum_b ws[g, b, w]; used by every two-stage column reduction.
// ws is (G, nblk, stride); columns [0, W) are reduced into out (G, W).  Block = 64 columns
// x 4 row slices; each slice keeps 4 independent loads in flight, the slices meet in LDS
// (one thread per column walking nblk rows serially was latency-bound: 25 us per call).
__global__ __launch_bounds__(256) void reduce_partials_kernel(const float* __restrict__ ws, float* __restrict__ out,
                                                              int nblk, int W, int stride, int accumulate, float alpha) {
  __shared__ float red[4][64];
  const int g = blockIdx.y;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int w = blockIdx.x * 64 + tx;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (w < W) {
    const float* p = ws + (long)g * nblk * stride + w;
    int b = ty;
    for (; b + 12 < nblk; b += 16) {
      s0 += p[(long)b * stride];
      s1 += p[(long)(b + 4) * stride];
      s2 += p[(long)(b + 8) * stride];
      s3 += p[(long)(b + 12) * stride];
    }
    for (; b < nblk; b += 4) s0 += p[(long)b * stride];
  }
  red[ty][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ty == 0 && w < W) {
    const float s = alpha * (((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx]);
    float* o = out + (long)g * W + w;
    *o = accumulate ? *o + s : s;
  }
}

int cmx_reduce_partials(const float* ws, float* out, int G, int nblk, int W, int accumulate,
                        float alpha, hipStream_t s) {
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(cdiv(W, 64), G), dim3(256), 0, s, ws, out, nblk,
                     W, W, accumulate, alpha);
  return cmx_check_launch("reduce_partials");
}

int cmx_reduce_partials_strided(const float* ws, float* out, int nblk, int W, int stride, int accumulate,
                                hipStream_t s) {
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(cdiv(W, 64), 1), dim3(256), 0, s, ws, out, nblk, W, stride,
                     accumulate, 1.0f);
  return cmx_check_launch("reduce_partials_strided");
}

static int ln_tpr(int chunks) {
  int t = 1;
  while (t < chunks && t < 64) t <<= 1;
  return t < 4 ? 4 : t;
}

template <typename T>
static int ln_fwd_launch(const void* x, const float* g, const float* b, void* y, float* mu, float* rs,
                         long R, int G, int C, float eps, hipStream_t s) {
  constexpr int V = VecT<T>::N;
  const int chunks = C / V;
  const int tpr = ln_tpr(chunks);
  const int nch = (chunks + tpr - 1) / tpr;
  // 4 rows per thread for narrow rows when that still leaves >= 256 blocks (one per CU)
  const int rpt = (nch == 1 && tpr <= 16 && R * G / ((256 / tpr) * 4) >= 256) ? 4 : 1;
  const dim3 grid(cdiv(R, (256 / tpr) * rpt), G);
#define LNF(TPR, NCH, RPT)                                                                  \
  if (tpr == TPR && nch == NCH && rpt == RPT) {                                             \
    hipLaunchKernelGGL((ln_fwd_kernel<T, TPR, NCH, RPT>), grid, dim3(256), 0, s, (const T*)x, g, b, \
                       (T*)y, mu, rs, R, C, eps);                                           \
    return cmx_check_launch("layernorm_fwd");                                               \
  }
  LNF(4, 1, 4) LNF(8, 1, 4) LNF(16, 1, 4)
  LNF(4, 1, 1) LNF(8, 1, 1) LNF(16, 1, 1) LNF(32, 1, 1) LNF(64, 1, 1) LNF(64, 2, 1) LNF(64, 4, 1)
#undef LNF
  cmx_set_error("layernorm_fwd: unsupported C=%d", C);
  return CMX_ERR_SHAPE;
}

static int ln_bwd_blocks(long R, int rpb) {     // <= 512 blocks per group: ~2 rows per thread at stage 1
  long nb = (R + rpb - 1) / rpb;
  return (int)(nb < 512 ? nb : 512);
}

template <typename T>
static int ln_bwd_launch(const void* dy, const void* x, const float* g, const float* mu,
                         const float* rs, void* dx, float* dgamma, float* dbeta, float* ws, long R,
                         int G, int C, int accumulate, const void* dres, const float* sscale, void* dxs,
                         long rps, const void* dy2, hipStream_t s) {
  constexpr int V = VecT<T>::N;
  const int chunks = C / V;
  const int tpr = ln_tpr(chunks);
  const int nch = (chunks + tpr - 1) / tpr;
  const int nb = ln_bwd_blocks(R, 256 / tpr);
  const dim3 grid(nb, G);
  // two rows per iteration where a thread walks more than one (narrow rows, stage 1 / 2)
  const int rpt = (nch == 1 && tpr <= 16 && R > (long)nb * (256 / tpr)) ? 2 : 1;
#define LNB(TPR, NCH, RPT)                                                                  \
  if (tpr == TPR && nch == NCH && rpt == RPT) {                                             \
    hipLaunchKernelGGL((ln_bwd_kernel<T, TPR, NCH, RPT>), grid, dim3(256), 0, s, (const T*)dy, \
                       (const T*)x, g, mu, rs, (T*)dx, ws, R, C, (const T*)dres, sscale,     \
                       (T*)dxs, rps, (const T*)dy2);                                         \
    goto reduce;                                                                            \
  }
  LNB(4, 1, 2) LNB(8, 1, 2) LNB(16, 1, 2)
  LNB(4, 1, 1) LNB(8, 1, 1) LNB(16, 1, 1) LNB(32, 1, 1) LNB(64, 1, 1) LNB(64, 2, 1) LNB(64, 4, 1)
#undef LNB
  cmx_set_error("layernorm_bwd: unsupported C=%d", C);
  return CMX_ERR_SHAPE;
reduce : {
  int st = cmx_check_launch("layernorm_bwd");
  if (st) return st;
  // ws layout per (g, blk): [dgamma C | dbeta C]; reduce into interleaved temp then split.
  // dgamma and dbeta are separate (G, C) arrays: reduce each half.
  for (int half = 0; half < 2; ++half) {
    float* dst = half == 0 ? dgamma : dbeta;
    if (!dst) continue;
    // treat ws as (G, nb, 2C) and reduce columns [half*C, half*C + C)
    hipLaunchKernelGGL(reduce_partials_kernel, dim3(cdiv(C, 64), G), dim3(256), 0, s, ws + half * C,
                       dst, nb, C, 2 * C, accumulate, 1.0f);
  }
  return CMX_OK;
}
}

extern "C" {

// y = LN(x) over C; x, y: (G*R, C) of dtype; gamma/beta: (G, C) fp32; mean/rstd: (G*R) fp32
// (may be NULL).  Replaces nn.LayerNorm.forward (see header).
int cmx_layernorm_fwd(const void* x, const float* gamma, const float* beta, void* y, float* mean,
                      float* rstd, long R, int G, int C, float eps, int dtype, hipStream_t s) {
  CMX_REQUIRE(R >= 0 && G > 0 && C > 0, CMX_ERR_SHAPE, "layernorm_fwd: bad shape");
  CMX_REQUIRE(C % (dtype == 0 ? 4 : 8) == 0 && C <= 1024, CMX_ERR_SHAPE,
              "layernorm_fwd: C=%d must be a multiple of the vector width and <= 1024", C);
  if (R == 0) return CMX_OK;
  CMX_DISPATCH(dtype, T, return ln_fwd_launch<T>(x, gamma, beta, y, mean, rstd, R, G, C, eps, s));
}

size_t cmx_layernorm_bwd_workspace(long R, int G, int C, int dtype) {
  const int V = dtype == 0 ? 4 : 8;
  const int tpr = ln_tpr(C / V);
  return (size_t)G * ln_bwd_blocks(R, 256 / tpr) * 2 * C * sizeof(float);
}

// dx (dtype), dgamma/dbeta (G, C) fp32 (overwritten, or accumulated if accumulate=1).
int cmx_layernorm_bwd(const void* dy, const void* x, const float* gamma, const float* mean,
                      const float* rstd, void* dx, float* dgamma, float* dbeta, float* workspace,
                      long R, int G, int C, int accumulate, int dtype, hipStream_t s) {
  CMX_REQUIRE(R > 0 && G > 0 && C > 0 && C <= 1024, CMX_ERR_SHAPE, "layernorm_bwd: bad shape");
  CMX_REQUIRE(C % (dtype == 0 ? 4 : 8) == 0, CMX_ERR_SHAPE, "layernorm_bwd: C=%d", C);
  CMX_DISPATCH(dtype, T,
               return ln_bwd_launch<T>(dy, x, gamma, mean, rstd, dx, dgamma, dbeta, workspace, R,
                                       G, C, accumulate, nullptr, nullptr, nullptr, 1, nullptr, s));
}

// cmx_layernorm_bwd with dy + dy2 as the upstream gradient (two consumers of y), a residual
// gradient dres added to dx and an optional DropPath-scaled copy
// dxs = sscale[(g*R + row) / rows_per_sample] * dx (dy2 / dres / sscale / dxs may be NULL).
int cmx_layernorm_bwd_res(const void* dy, const void* dy2, const void* x, const float* gamma, const float* mean,
                          const float* rstd, const void* dres, const float* sscale, void* dxs, void* dx, float* dgamma,
                          float* dbeta,
                          float* workspace, long R, int G, int C, long rows_per_sample, int accumulate, int dtype,
                          hipStream_t s) {
  CMX_REQUIRE(R > 0 && G > 0 && C > 0 && C <= 1024, CMX_ERR_SHAPE, "layernorm_bwd_res: bad shape");
  CMX_REQUIRE(C % (dtype == 0 ? 4 : 8) == 0, CMX_ERR_SHAPE, "layernorm_bwd_res: C=%d", C);
  CMX_REQUIRE(!dxs || (sscale && rows_per_sample > 0), CMX_ERR_ARG, "layernorm_bwd_res: dxs needs sscale");
  CMX_DISPATCH(dtype, T,
               return ln_bwd_launch<T>(dy, x, gamma, mean, rstd, dx, dgamma, dbeta, workspace, R,
                                       G, C, accumulate, dres, sscale, dxs, rows_per_sample > 0 ? rows_per_sample : 1,
                                       dy2, s));
}

}  // extern "C"

extern "C" {
// out (G, W) (+)= alpha * sum over nblk of ws (G, nblk, W): the split-K combine of the
// chunked weight-gradient GEMMs and every other two-stage column reduction.
int cmx_partials_sum(const float* ws, float* out, int G, int nblk, int W, int accumulate, float alpha,
                     hipStream_t s) {
  CMX_REQUIRE(G > 0 && nblk > 0 && W > 0, CMX_ERR_SHAPE, "partials_sum: shape");
  return cmx_reduce_partials(ws, out, G, nblk, W, accumulate, alpha, s);
}
}
