// CM-FRM feature rectification (FeatureRectifyModule, net_utils.py:124-152) on token-major
// activations x (2, B, N, C) = (x1 = RGB stream, x2 = X stream).
//
//  pool        ChannelWeights avg/max pooling of cat(x1, x2) over H*W (net_utils.py:22-27):
//              pooled (B, 4C) = [avg x1 | avg x2 | max x1 | max x2]; argmax (B, 2C) int32 keeps
//              the FIRST maximal token (the index PyTorch's CPU max pool routes gradient to).
//  small_linear  y = act(x W^T + b) for the tiny-M channel MLP (B rows, :16-20) - a GEMV
//              with one wave per output feature; backward writes dW/db straight into the
//              gradient buffers.
//  spatial     SpatialWeights second 1x1 conv (C -> 2) + sigmoid on relu(h) (:74-83).
//  combine     out1 = x1 + 0.5*cw1*x2 + 0.5*sw1*x2 ; out2 = x2 + 0.5*cw0*x1 + 0.5*sw0*x1
//              (:147-152) and its backward (direct path + dcw/dsw reductions).
#include "cmx_common.h"

namespace {

// partial pooling over a token chunk: blockIdx = (chunk, g*B + b); thread = channel
template <typename T>
__global__ void pool_partial_kernel(const T* __restrict__ x, float* __restrict__ psum, float* __restrict__ pmax,
                                    int* __restrict__ pidx, int B, int N, int C, int chunk) {
  const int gb = blockIdx.y, c_ = blockIdx.x;
  const int n0 = c_ * chunk, n1 = min(N, n0 + chunk);
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f, m = -INFINITY;
    int mi = n0;
    const T* p = x + (long)gb * N * C + c;
    for (int n = n0; n < n1; ++n) {
      const float v = to_f32(p[(long)n * C]);
      s += v;
      if (v > m) { m = v; mi = n; }
    }
    const long o = ((long)gb * gridDim.x + c_) * C + c;
    psum[o] = s; pmax[o] = m; pidx[o] = mi;
  }
}

// block = 64 channels x 4 chunk slices of one (group, image); the slices meet in LDS.  Max ties
// resolve to the lowest token index, as the sequential scan over chunks would.
__global__ __launch_bounds__(256) void pool_final_kernel(const float* __restrict__ psum, const float* __restrict__ pmax,
                                                         const int* __restrict__ pidx, float* __restrict__ pooled,
                                                         int* __restrict__ argmax, int B, int N, int C, int nchunk) {
  __shared__ float rs[3][64], rm[3][64];
  __shared__ int ri[3][64];
  const int gb = blockIdx.y, cl = threadIdx.x & 63, zl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float sm = 0.f, m = -INFINITY;
  int mi = 0x7fffffff;
  if (c < C) {
#pragma unroll 4
    for (int k = zl; k < nchunk; k += 4) {
      const long o = ((long)gb * nchunk + k) * C + c;
      sm += psum[o];
      const float v = pmax[o];
      const int ix = pidx[o];
      if (v > m || (v == m && ix < mi)) { m = v; mi = ix; }
    }
  }
  if (zl > 0) { rs[zl - 1][cl] = sm; rm[zl - 1][cl] = m; ri[zl - 1][cl] = mi; }
  __syncthreads();
  if (zl > 0 || c >= C) return;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    sm += rs[q][cl];
    const float v = rm[q][cl];
    const int ix = ri[q][cl];
    if (v > m || (v == m && ix < mi)) { m = v; mi = ix; }
  }
  const int g = gb / B, b = gb % B;
  pooled[(long)b * 4 * C + g * C + c] = sm / N;
  pooled[(long)b * 4 * C + 2 * C + g * C + c] = m;
  argmax[(long)b * 2 * C + g * C + c] = mi;
}

// one wave per output feature n; M rows
__global__ void small_linear_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                        const float* __restrict__ b, float* __restrict__ y, int M, int K, int Nout,
                                        int act) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= Nout) return;
  const float* wr = w + (long)wave * K;
  for (int m = 0; m < M; ++m) {
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s += wr[k] * x[(long)m * K + k];
    s = wave_sum(s);
    if (lane == 0) y[(long)m * Nout + wave] = act_fwd(s + (b ? b[wave] : 0.f), act);
  }
}

// dz = dy * act'(.) evaluated from the saved OUTPUT y (relu / sigmoid / none)
__device__ __forceinline__ float act_grad_from_out(float y, int act) {
  if (act == ACT_RELU) return y > 0.f ? 1.f : 0.f;
  if (act == ACT_SIGMOID) return y * (1.f - y);
  return 1.f;
}

__global__ void small_linear_dz_kernel(const float* __restrict__ dy, const float* __restrict__ y, float* __restrict__ dz,
                                       long n, int act) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)n; i += gridDim.x * blockDim.x)
    dz[i] = dy[i] * act_grad_from_out(y[i], act);
}

// partial dx over an n-slice: ws[slice][m][k] = sum_{n in slice} dz[m][n] w[n][k].
// Block = 64 k-columns x 4 n-subslices (coalesced W rows), grid = (K/64, NSLICE).
constexpr int DX_NSLICE = 16;
constexpr int DX_MMAX = 8;
__global__ __launch_bounds__(256) void small_linear_dx_kernel(const float* __restrict__ dz, const float* __restrict__ w,
                                                              float* __restrict__ ws, int M, int K, int Nout) {
  __shared__ float red[4][DX_MMAX][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + tx;
  const int per = (Nout + DX_NSLICE - 1) / DX_NSLICE;
  const int n0 = blockIdx.y * per, n1 = min(Nout, n0 + per);
  float acc[DX_MMAX];
#pragma unroll
  for (int m = 0; m < DX_MMAX; ++m) acc[m] = 0.f;
  if (k < K) {
    for (int n = n0 + ty; n < n1; n += 4) {
      const float wv = w[(long)n * K + k];
#pragma unroll
      for (int m = 0; m < DX_MMAX; ++m)
        if (m < M) acc[m] += dz[(long)m * Nout + n] * wv;
    }
  }
#pragma unroll
  for (int m = 0; m < DX_MMAX; ++m) red[ty][m][tx] = acc[m];
  __syncthreads();
  if (ty == 0 && k < K) {
    for (int m = 0; m < M; ++m)
      ws[((long)blockIdx.y * M + m) * K + k] = ((red[0][m][tx] + red[1][m][tx]) + red[2][m][tx]) + red[3][m][tx];
  }
}

// dw[n][k] = sum_m dz[m][n] x[m][k]; db[n] = sum_m dz[m][n]
__global__ void small_linear_dw_kernel(const float* __restrict__ dz, const float* __restrict__ x, float* __restrict__ dw,
                                       float* __restrict__ db, int M, int K, int Nout, int accumulate) {
  const long total = (long)Nout * K;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)total; i += gridDim.x * blockDim.x) {
    const int k = i % K, n = i / K;
    float s = 0.f;
    for (int m = 0; m < M; ++m) s += dz[(long)m * Nout + n] * x[(long)m * K + k];
    dw[i] = accumulate ? dw[i] + s : s;
    if (k == 0 && db) {
      float sb = 0.f;
      for (int m = 0; m < M; ++m) sb += dz[(long)m * Nout + n];
      db[n] = accumulate ? db[n] + sb : sb;
    }
  }
}

// sw[row][o] = sigmoid(sum_c relu(h[row][c]) w2[o][c] + b2[o]); 16 lanes per row
template <typename T>
__global__ void spatial_fwd_kernel(const T* __restrict__ h, const float* __restrict__ w2, const float* __restrict__ b2,
                                   float* __restrict__ sw, long rows, int C) {
  constexpr int V = VecT<T>::N;
  const int lane = threadIdx.x & 15;
  const long row = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  float s0 = 0.f, s1 = 0.f;
  if (row < rows) {
    for (int ch = lane; ch < C / V; ch += 16) {
      float v[V];
      load_vec<T>(h + row * C + ch * V, v);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float r = v[j] > 0.f ? v[j] : 0.f;
        s0 += r * w2[ch * V + j];
        s1 += r * w2[C + ch * V + j];
      }
    }
  }
  s0 = group_sum(s0, 16);
  s1 = group_sum(s1, 16);
  if (row < rows && lane == 0) {
    sw[row * 2] = 1.f / (1.f + __expf(-(s0 + b2[0])));
    sw[row * 2 + 1] = 1.f / (1.f + __expf(-(s1 + b2[1])));
  }
}

template <typename T>
__global__ void combine_fwd_kernel(const T* __restrict__ x, const float* __restrict__ cw, const float* __restrict__ sw,
                                   T* __restrict__ out, int B, int N, int C) {
  constexpr int V = VecT<T>::N;
  const long per = (long)B * N * C;
  const long nvec = per / V;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)nvec; i += gridDim.x * blockDim.x) {
    const int e = i * V;
    const int c0 = e % C;
    const int row = e / C;        // b*N + n
    const int b = row / N;
    float a[V], bb[V], o1[V], o2[V];
    load_vec<T>(x + e, a);
    load_vec<T>(x + per + e, bb);
    const float s0 = 0.5f * sw[row * 2], s1 = 0.5f * sw[row * 2 + 1];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float c0w = 0.5f * cw[(long)b * 2 * C + c0 + j];
      const float c1w = 0.5f * cw[(long)b * 2 * C + C + c0 + j];
      o1[j] = (a[j] + c1w * bb[j]) + s1 * bb[j];
      o2[j] = (bb[j] + c0w * a[j]) + s0 * a[j];
    }
    store_vec<T>(out + e, o1);
    store_vec<T>(out + per + e, o2);
  }
}

// direct-path dx, dsw (row sums) and per-block dcw partials.  blockIdx.y = b.
// TPR lanes per row; ws (B, nblk, 2C) = [dcw0 | dcw1] partials.
template <typename T, int TPR>
__global__ __launch_bounds__(256) void combine_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ x,
                                                          const float* __restrict__ cw, const float* __restrict__ sw,
                                                          T* __restrict__ dx, float* __restrict__ dsw,
                                                          float* __restrict__ ws, int B, int N, int C) {
  constexpr int V = VecT<T>::N;
  constexpr int RPB = 256 / TPR;
  constexpr int MAXCH = 4;  // chunks per lane (C <= 4 * TPR * V)
  __shared__ float red[2][512];
  const int b = blockIdx.y;
  const int lane = threadIdx.x % TPR, slot = threadIdx.x / TPR;
  const int nch = C / V;
  const long per = (long)B * N * C;
  float a0[MAXCH][V], a1[MAXCH][V];
#pragma unroll
  for (int k = 0; k < MAXCH; ++k)
#pragma unroll
    for (int j = 0; j < V; ++j) a0[k][j] = a1[k][j] = 0.f;
  for (int n = blockIdx.x * RPB + slot; n < N; n += gridDim.x * RPB) {
    const long row = (long)b * N + n;
    const float s0 = 0.5f * sw[row * 2], s1 = 0.5f * sw[row * 2 + 1];
    float r0 = 0.f, r1 = 0.f;
#pragma unroll
    for (int k = 0; k < MAXCH; ++k) {
      const int ch = lane + k * TPR;
      if (ch >= nch) continue;
      const long e = row * C + ch * V;
      float d1[V], d2[V], x1[V], x2[V], o1[V], o2[V];
      load_vec<T>(dout + e, d1);
      load_vec<T>(dout + per + e, d2);
      load_vec<T>(x + e, x1);
      load_vec<T>(x + per + e, x2);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int c = ch * V + j;
        const float c0w = 0.5f * cw[(long)b * 2 * C + c];
        const float c1w = 0.5f * cw[(long)b * 2 * C + C + c];
        o1[j] = d1[j] + (c0w + s0) * d2[j];
        o2[j] = d2[j] + (c1w + s1) * d1[j];
        const float p1 = d1[j] * x2[j];   // feeds dcw1, dsw1
        const float p0 = d2[j] * x1[j];   // feeds dcw0, dsw0
        r1 += p1; r0 += p0;
        a1[k][j] += p1; a0[k][j] += p0;
      }
      store_vec<T>(dx + e, o1);
      store_vec<T>(dx + per + e, o2);
    }
    r0 = group_sum(r0, TPR);
    r1 = group_sum(r1, TPR);
    if (lane == 0) { dsw[row * 2] = 0.5f * r0; dsw[row * 2 + 1] = 0.5f * r1; }
  }
  // reduce column partials over row slots, 512 columns at a time
  float* out = ws + ((long)b * gridDim.x + blockIdx.x) * 2 * C;
  for (int base = 0; base < C; base += 512) {
    for (int e = threadIdx.x; e < 2 * 512; e += 256) (&red[0][0])[e] = 0.f;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MAXCH; ++k) {
      const int ch = lane + k * TPR;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int c = ch * V + j - base;
        if (ch < nch && c >= 0 && c < 512) {
          atomicAdd(&red[0][c], a0[k][j]);
          atomicAdd(&red[1][c], a1[k][j]);
        }
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 512 && base + c < C; c += 256) {
      out[base + c] = 0.5f * red[0][c];
      out[C + base + c] = 0.5f * red[1][c];
    }
    __syncthreads();
  }
}

// spatial backward: dz2 = dsw * sw(1-sw); dh = [h>0] * (dz2 @ w2); partials of
// dw2 (2, C) = sum dz2^T relu(h) and db2 (2) into ws (nblk, 2C + 2).  16 lanes per row.
template <typename T>
__global__ __launch_bounds__(256) void spatial_bwd_kernel(const float* __restrict__ dsw, const float* __restrict__ sw,
                                                          const T* __restrict__ h, const float* __restrict__ w2,
                                                          T* __restrict__ dh, float* __restrict__ ws, long rows, int C) {
  constexpr int V = VecT<T>::N;
  __shared__ float red[2 * 512 + 2];
  for (int e = threadIdx.x; e < 2 * C + 2; e += 256) red[e] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 15;
  float db0 = 0.f, db1 = 0.f;
  for (long row = (long)blockIdx.x * 16 + (threadIdx.x >> 4); row < rows; row += (long)gridDim.x * 16) {
    const float g0 = dsw[row * 2] * sw[row * 2] * (1.f - sw[row * 2]);
    const float g1 = dsw[row * 2 + 1] * sw[row * 2 + 1] * (1.f - sw[row * 2 + 1]);
    if (lane == 0) { db0 += g0; db1 += g1; }
    for (int ch = lane; ch < C / V; ch += 16) {
      float v[V], o[V];
      load_vec<T>(h + row * C + ch * V, v);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int c = ch * V + j;
        const bool pos = v[j] > 0.f;
        o[j] = pos ? g0 * w2[c] + g1 * w2[C + c] : 0.f;
        const float r = pos ? v[j] : 0.f;
        atomicAdd(&red[c], g0 * r);
        atomicAdd(&red[C + c], g1 * r);
      }
      store_vec<T>(dh + row * C + ch * V, o);
    }
  }
  if (lane == 0) { atomicAdd(&red[2 * C], db0); atomicAdd(&red[2 * C + 1], db1); }
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * C + 2; e += 256) ws[(long)blockIdx.x * (2 * C + 2) + e] = red[e];
}

// dx[g][b][n][c] += dpooled_avg[b][gC+c] / N + (n == argmax[b][gC+c]) * dpooled_max[b][2C+gC+c]
template <typename T>
__global__ void pool_bwd_kernel(const float* __restrict__ dpooled, const int* __restrict__ argmax, T* __restrict__ dx,
                                int B, int N, int C) {
  const long total = 2L * B * N * C;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)total; i += gridDim.x * blockDim.x) {
    const int c = i % C;
    const int n = (i / C) % N;
    const int gb = i / (C * N);
    const int g = gb / B, b = gb % B;
    float v = dpooled[(long)b * 4 * C + g * C + c] / N;
    if (argmax[(long)b * 2 * C + g * C + c] == n) v += dpooled[(long)b * 4 * C + 2 * C + g * C + c];
    dx[i] = from_f32<T>(to_f32(dx[i]) + v);
  }
}

int pool_nchunk(int N, int GB) {
  long nc = (1024 + GB - 1) / GB;
  const long maxc = (N + 63) / 64;
  if (nc > maxc) nc = maxc;
  return nc < 1 ? 1 : (int)nc;
}
unsigned gridcap(long total) {
  const unsigned g = cdiv(total, 256);
  return g < 8192 ? (g ? g : 1) : 8192;
}
int combine_nblk(int N, int rpb) {              // <= 256 blocks per image (partials reduced after)
  int nb = (N + rpb - 1) / rpb;
  return nb < 256 ? nb : 256;
}
int spatial_nblk(long rows) {
  long nb = (rows + 15) / 16;
  return (int)(nb < 256 ? nb : 256);
}
}  // namespace

extern "C" {

// dz_ws of cmx_small_linear_bwd: M*Nout + 16*M*K floats
size_t cmx_small_linear_bwd_workspace(int M, int K, int Nout) {
  return ((size_t)M * Nout + (size_t)DX_NSLICE * M * K) * sizeof(float);
}

size_t cmx_frm_pool_workspace(int B, int N, int C) {
  const int nc = pool_nchunk(N, 2 * B);
  return (size_t)2 * B * nc * C * 3 * sizeof(float);
}

int cmx_frm_pool_fwd(const void* x, float* pooled, int* argmax, float* workspace, int B, int N, int C, int dtype,
                     hipStream_t s) {
  CMX_REQUIRE(B > 0 && N > 0 && C > 0, CMX_ERR_SHAPE, "frm_pool: shape");
  const int nc = pool_nchunk(N, 2 * B);
  const int chunk = (N + nc - 1) / nc;
  float* psum = workspace;
  float* pmax = psum + (size_t)2 * B * nc * C;
  int* pidx = (int*)(pmax + (size_t)2 * B * nc * C);
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(pool_partial_kernel<T>, dim3(nc, 2 * B), dim3(C < 256 ? 64 * ((C + 63) / 64) : 256), 0, s,
                       (const T*)x, psum, pmax, pidx, B, N, C, chunk);
  });
  hipLaunchKernelGGL(pool_final_kernel, dim3(cdiv(C, 64), 2 * B), dim3(256), 0, s, psum, pmax, pidx, pooled, argmax,
                     B, N, C, nc);
  return cmx_check_launch("frm_pool_fwd");
}

int cmx_frm_pool_bwd(const float* dpooled, const int* argmax, void* dx, int B, int N, int C, int dtype, hipStream_t s) {
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(pool_bwd_kernel<T>, dim3(gridcap(2L * B * N * C)), dim3(256), 0, s, dpooled, argmax, (T*)dx,
                       B, N, C);
  });
  return cmx_check_launch("frm_pool_bwd");
}

int cmx_small_linear_fwd(const float* x, const float* w, const float* b, float* y, int M, int K, int Nout, int act,
                         hipStream_t s) {
  hipLaunchKernelGGL(small_linear_fwd_kernel, dim3(cdiv((long)Nout * 64, 256)), dim3(256), 0, s, x, w, b, y, M, K,
                     Nout, act);
  return cmx_check_launch("small_linear_fwd");
}

// dz_ws: M*Nout floats; dx may be NULL
int cmx_small_linear_bwd(const float* dy, const float* y, const float* x, const float* w, float* dx, float* dw,
                         float* db, float* dz_ws, int M, int K, int Nout, int act, int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(small_linear_dz_kernel, dim3(gridcap((long)M * Nout)), dim3(256), 0, s, dy, y, dz_ws,
                     (long)M * Nout, act);
  CMX_REQUIRE(M <= DX_MMAX, CMX_ERR_SHAPE, "small_linear_bwd: M=%d > %d", M, DX_MMAX);
  if (dx) {
    float* part = dz_ws + (size_t)M * Nout;   // DX_NSLICE * M * K floats after dz
    hipLaunchKernelGGL(small_linear_dx_kernel, dim3(cdiv(K, 64), DX_NSLICE), dim3(256), 0, s, dz_ws, w, part, M, K,
                       Nout);
    const int st = cmx_reduce_partials(part, dx, 1, DX_NSLICE, M * K, 0, 1.f, s);
    if (st) return st;
  }
  hipLaunchKernelGGL(small_linear_dw_kernel, dim3(gridcap((long)Nout * K)), dim3(256), 0, s, dz_ws, x, dw, db, M, K,
                     Nout, accumulate);
  return cmx_check_launch("small_linear_bwd");
}

int cmx_frm_spatial_fwd(const void* h, const float* w2, const float* b2, float* sw, int64_t rows, int C, int dtype,
                        hipStream_t s) {
  CMX_REQUIRE(C % 8 == 0, CMX_ERR_SHAPE, "frm_spatial: C");
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(spatial_fwd_kernel<T>, dim3(cdiv(rows, 16)), dim3(256), 0, s, (const T*)h, w2, b2, sw,
                       (long)rows, C);
  });
  return cmx_check_launch("frm_spatial_fwd");
}

size_t cmx_frm_spatial_bwd_workspace(int64_t rows, int C) {
  return (size_t)spatial_nblk(rows) * (2 * C + 2) * sizeof(float);
}

// dw2 (2, C), db2 (2) fp32 written (or accumulated)
int cmx_frm_spatial_bwd(const float* dsw, const float* sw, const void* h, const float* w2, void* dh, float* dw2,
                        float* db2, float* workspace, int64_t rows, int C, int accumulate, int dtype, hipStream_t s) {
  CMX_REQUIRE(C % 8 == 0 && C <= 512, CMX_ERR_SHAPE, "frm_spatial_bwd: C");
  const int nb = spatial_nblk(rows);
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(spatial_bwd_kernel<T>, dim3(nb), dim3(256), 0, s, dsw, sw, (const T*)h, w2, (T*)dh, workspace,
                       (long)rows, C);
  });
  int st = cmx_check_launch("frm_spatial_bwd");
  if (st) return st;
  st = cmx_reduce_partials_strided(workspace, dw2, nb, 2 * C, 2 * C + 2, accumulate, s);
  if (st) return st;
  return cmx_reduce_partials_strided(workspace + 2 * C, db2, nb, 2, 2 * C + 2, accumulate, s);
}

int cmx_frm_combine_fwd(const void* x, const float* cw, const float* sw, void* out, int B, int N, int C, int dtype,
                        hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0, CMX_ERR_SHAPE, "frm_combine: C");
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(combine_fwd_kernel<T>, dim3(gridcap((long)B * N * C / V)), dim3(256), 0, s, (const T*)x, cw, sw,
                       (T*)out, B, N, C);
  });
  return cmx_check_launch("frm_combine_fwd");
}

size_t cmx_frm_combine_bwd_workspace(int B, int N, int C) {
  return (size_t)B * combine_nblk(N, 16) * 2 * C * sizeof(float);
}

// dx (2,B,N,C) direct path; dsw (B,N,2); dcw (B, 2C) = [dcw0 | dcw1] (overwritten)
int cmx_frm_combine_bwd(const void* dout, const void* x, const float* cw, const float* sw, void* dx, float* dsw,
                        float* dcw, float* workspace, int B, int N, int C, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0 && C / V <= 4 * 64, CMX_ERR_SHAPE, "frm_combine_bwd: C=%d", C);
  const int nb = combine_nblk(N, 16);
  // lanes per row = the row's 16-B chunks rounded up to a power of two (C = 64 bf16: 8 lanes,
  // 32 rows per block in flight), capped at a wave
  const int chunks = C / V;
  int tpr = 4;
  while (tpr < chunks && tpr < 64) tpr <<= 1;
#define CMB(TPR) hipLaunchKernelGGL((combine_bwd_kernel<T, TPR>), dim3(nb, B), dim3(256), 0, s, (const T*)dout, \
                                    (const T*)x, cw, sw, (T*)dx, dsw, workspace, B, N, C)
  CMX_DISPATCH(dtype, T, {
    if (tpr == 4) CMB(4);
    else if (tpr == 8) CMB(8);
    else if (tpr == 16) CMB(16);
    else if (tpr == 32) CMB(32);
    else CMB(64);
  });
#undef CMB
  int st = cmx_check_launch("frm_combine_bwd");
  if (st) return st;
  return cmx_reduce_partials(workspace, dcw, B, nb, 2 * C, 0, 1.f, s);
}

}  // extern "C"
