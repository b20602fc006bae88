// CM-FRM feature rectification (FeatureRectifyModule, net_utils.py:124-152) on token-major
// activations x (2, B, N, C) = (x1 = RGB stream, x2 = X stream).
//
//  pool        ChannelWeights avg/max pooling of cat(x1, x2) over H*W (net_utils.py:22-27):
//              pooled (B, 4C) = [avg x1 | avg x2 | max x1 | max x2]; argmax (B, 2C) int32 keeps
//              the FIRST maximal token (the index PyTorch's CPU max pool routes gradient to).
//  small_linear  y = act(x W^T + b) for the tiny-M channel MLP (B rows, :16-20) - a GEMV
//              over LDS-staged rows; its backward is ONE pass over W that forms dz from the
//              producer's partial slabs, writes dW/db and leaves dx as partial slices for
//              the next consumer (no separate dz / reduce launches).
//  combine     SpatialWeights' second 1x1 conv (C -> 2) + sigmoid (:74-83) fused with the
//              rectification out1 = x1 + 0.5*cw1*x2 + 0.5*sw1*x2 ; out2 = x2 + 0.5*cw0*x1 +
//              0.5*sw0*x1 (:147-152); its backward also runs the spatial head's backward
//              (dh, dw2 / db2 partials) and leaves the dcw partials for the MLP backward.
//  The first SpatialWeights 1x1 conv (2C -> C) is a cmx_gemm (forward: two A segments, no cat;
//  dgrad: both modality slices in one G = 2 launch).
#include "cmx_common.h"

namespace {

// Row-parallel layout shared by the token kernels: a row of C channels is C / V 16-B chunks;
// TPR lanes per row (the chunk count rounded up to a power of two, at most 64), each lane
// owning chunks lane, lane + TPR (MAXCH <= 2), RPB = 256 / TPR rows in flight per block.
constexpr int MAXCH = 2;
inline int row_lanes(int C, int V) {
  int tpr = 4;
  while (tpr < C / V && tpr < 64) tpr <<= 1;
  return tpr;
}

// ------------------------------------------------------------------------ pooling (forward)
// ONE launch: block (z, cg, gb) reduces token chunk z of the 32-channel group cg of one (group,
// image) gb to a partial [sum | max | argmax]; the last block of (cg, gb) to arrive folds the
// nz partials into pooled / argmax (last_arrival, cmx_common.h).  Lanes per token row = 32 / V
// (4 for 16-bit storage, 8 for fp32), one 16-B vector each; the row slots combine in LDS with
// 8 threads per channel and a lane shuffle.  Max ties -> the lowest token index (the sequential
// scan PyTorch's CPU max does), whatever order the slots / chunks combine in.
constexpr int PG = 32;                          // channels per block
constexpr int PZ_MAX = 32;                      // token chunks per (channel group, image): the fold
                                                // reads PG * nz * 3 values, <= 12 per thread
constexpr int POOL_TICKETS = 4096;
__device__ unsigned g_pool_ticket[POOL_TICKETS];

__device__ __forceinline__ void maxidx_merge(float& m, int& mi, float v, int i) {
  if (v > m || (v == m && i < mi)) { m = v; mi = i; }
}
// combine (s, m, mi) over the 8 consecutive lanes of a channel, fixed order (deterministic)
__device__ __forceinline__ void group8_merge(float& s, float& m, int& mi) {
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) {
    const float s2 = __shfl_xor(s, o, 64), m2 = __shfl_xor(m, o, 64);
    const int i2 = __shfl_xor(mi, o, 64);
    s += s2;
    maxidx_merge(m, mi, m2, i2);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void pool_kernel(const T* __restrict__ x, float* __restrict__ psum,
                                                   float* __restrict__ pmax, int* __restrict__ pidx,
                                                   float* __restrict__ pooled, int* __restrict__ argmax, int B,
                                                   int N, int C, int chunk, unsigned* __restrict__ tickets) {
  constexpr int V = VecT<T>::N, LPR = PG / V, RPB = 256 / LPR;
  __shared__ float rs[RPB][PG + 1], rm[RPB][PG + 1];
  __shared__ int ri[RPB][PG + 1];
  const int z = blockIdx.x, cg = blockIdx.y, gb = blockIdx.z, nz = gridDim.x, ng = gridDim.y;
  const int lane = threadIdx.x % LPR, slot = threadIdx.x / LPR;
  const int n0 = z * chunk, n1 = min(N, n0 + chunk);
  float sm[V], mx[V];
  int ix[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { sm[j] = 0.f; mx[j] = -INFINITY; ix[j] = 0x7fffffff; }
  const T* base = x + (long)gb * N * C + cg * PG + lane * V;
#pragma unroll 4
  for (int n = n0 + slot; n < n1; n += RPB) {
    float v[V];
    load_vec<T>(base + (long)n * C, v);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      sm[j] += v[j];
      if (v[j] > mx[j]) { mx[j] = v[j]; ix[j] = n; }
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) { rs[slot][lane * V + j] = sm[j]; rm[slot][lane * V + j] = mx[j]; ri[slot][lane * V + j] = ix[j]; }
  __syncthreads();
  // 8 threads per channel: slots q = k, k + 8, ... then the 8-lane merge
  const int c = threadIdx.x >> 3, k = threadIdx.x & 7;
  float s = 0.f, m = -INFINITY;
  int mi = 0x7fffffff;
  for (int q = k; q < RPB; q += 8) {
    s += rs[q][c];
    maxidx_merge(m, mi, rm[q][c], ri[q][c]);
  }
  group8_merge(s, m, mi);
  const long po = ((long)(gb * ng + cg) * nz + z) * PG + c;
  if (k == 0) { st_agent(psum + po, s); st_agent(pmax + po, m); st_agent(pidx + po, mi); }
  if (!last_arrival((tickets ? tickets : g_pool_ticket) + gb * ng + cg, nz)) return;
  // fold: channel c, chunks z = k, k + 8, k + 16, k + 24 (all loads issued before the merge)
  const long pb = (long)(gb * ng + cg) * nz * PG + c;
  float ls[PZ_MAX / 8], lm[PZ_MAX / 8];
  int li[PZ_MAX / 8];
#pragma unroll
  for (int u = 0; u < PZ_MAX / 8; ++u) {
    const int zz = k + 8 * u;
    const bool ok = zz < nz;
    ls[u] = ok ? ld_agent(psum + pb + (long)zz * PG) : 0.f;
    lm[u] = ok ? ld_agent(pmax + pb + (long)zz * PG) : -INFINITY;
    li[u] = ok ? ld_agent(pidx + pb + (long)zz * PG) : 0x7fffffff;
  }
  s = 0.f; m = -INFINITY; mi = 0x7fffffff;
#pragma unroll
  for (int u = 0; u < PZ_MAX / 8; ++u) { s += ls[u]; maxidx_merge(m, mi, lm[u], li[u]); }
  group8_merge(s, m, mi);
  if (k == 0) {
    const int g = gb / B, b = gb % B, ch = cg * PG + c;
    pooled[(long)b * 4 * C + g * C + ch] = s / N;
    pooled[(long)b * 4 * C + 2 * C + g * C + ch] = m;
    argmax[(long)b * 2 * C + g * C + ch] = mi;
  }
}

// ------------------------------------------------------------------------ channel MLP
// y[m][n] = act(x[m] . w[n] + b[n]) for the B-row MLP of ChannelWeights (net_utils.py:16-20):
// x (M x K) staged once per block in LDS, one wave per 4 output features, float4 weight loads
// (each weight row read once for all M rows).
constexpr int MMAX = 8;
constexpr int LIN_FPW = 1;                      // output features per wave
__global__ __launch_bounds__(256) void linear_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ b, float* __restrict__ y, int M,
                                                         int K, int Nout, int act) {
  extern __shared__ float xs[];                 // M * K
  for (int e = threadIdx.x; e < M * K; e += 256) xs[e] = x[e];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int K4 = K >> 2;
  const int n = blockIdx.x * 4 + wave;
  if (n >= Nout) return;
  const float4* wr = reinterpret_cast<const float4*>(w + (long)n * K);
  float acc[MMAX];
#pragma unroll
  for (int m = 0; m < MMAX; ++m) acc[m] = 0.f;
  int k4 = lane;
  for (; k4 + 192 < K4; k4 += 256) {            // four independent 16-B weight loads in flight
    float4 wv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) wv[u] = wr[k4 + 64 * u];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int m = 0; m < MMAX; ++m) {
        if (m < M) {
          const float4 xv = *reinterpret_cast<const float4*>(xs + m * K + 4 * (k4 + 64 * u));
          acc[m] += wv[u].x * xv.x + wv[u].y * xv.y + wv[u].z * xv.z + wv[u].w * xv.w;
        }
      }
  }
  for (; k4 < K4; k4 += 64) {
    const float4 wv = wr[k4];
#pragma unroll
    for (int m = 0; m < MMAX; ++m) {
      if (m < M) {
        const float4 xv = *reinterpret_cast<const float4*>(xs + m * K + 4 * k4);
        acc[m] += wv.x * xv.x + wv.y * xv.y + wv.z * xv.z + wv.w * xv.w;
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MMAX; ++m) {
    if (m >= M) break;
    const float s = wave_sum(acc[m]);
    if (lane == 0) y[(long)m * Nout + n] = act_fwd(s + (b ? b[n] : 0.f), act);
  }
}

// dz = dy * act'(.) evaluated from the saved OUTPUT y (relu / sigmoid / none)
__device__ __forceinline__ float act_grad_from_out(float y, int act) {
  if (act == ACT_RELU) return y > 0.f ? 1.f : 0.f;
  if (act == ACT_SIGMOID) return y * (1.f - y);
  return 1.f;
}

// Backward of y = act(x w^T + b) in ONE pass over w: block = 64 k-columns x 4 row lanes over
// an n-slice of NSLICE.  dy arrives as partial slabs dy[m][n] = sum_s part[s*ss + m*sm + n]
// (the producer's per-block partials: no separate reduce launch); dz = dy * act'(y).
//   dx partial  dxp[slice][m][k] = sum_{n in slice} dz[m][n] w[n][k]     (consumer sums slices)
//   dw[n][k] (+)= sum_m dz[m][n] x[m][k]                                 (written here)
//   db[n]    (+)= sum_m dz[m][n]                                          (column block 0)
constexpr int NSLICE = 16;
constexpr int SLICE_MAX = 256;                  // rows per slice: Nout <= 16 * 256 = 4096
constexpr int LBR = 8;                          // weight rows per lane with loads in flight together
__global__ __launch_bounds__(256) void linear_bwd_kernel(const float* __restrict__ dyp, int nsl, long ss, long sm,
                                                         const float* __restrict__ y, const float* __restrict__ x,
                                                         const float* __restrict__ w, float* __restrict__ dxp,
                                                         float* __restrict__ dw, float* __restrict__ db, int M, int K,
                                                         int Nout, int act, int accumulate) {
  __shared__ float dzs[MMAX][SLICE_MAX];
  __shared__ float red[4][MMAX][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int per = (Nout + NSLICE - 1) / NSLICE;
  const int n0 = blockIdx.y * per, n1 = min(Nout, n0 + per);
  const int rows = n1 > n0 ? n1 - n0 : 0;
  // dz of the slice: T consecutive lanes sum the nsl partial slabs of one value (strided over
  // q), combined by shuffles in a fixed order (deterministic)
  const int nval = M * rows;
  int T = 1;
  while (T < 64 && T * 2 * nval <= 256 && T * 2 <= nsl) T <<= 1;
  for (int base = 0; base < nval * T; base += 256) {
    const int t = base + threadIdx.x;
    const int e = t / T, sub = t % T;
    float d = 0.f;
    int m = 0, n = n0;
    if (e < nval) {
      m = e / rows; n = n0 + e % rows;
      const float* pp = dyp + m * sm + n;
      int q = sub;
      // eight slabs' loads in flight before the adds (same summation order): with T = 1 a lane
      // walked its 16 slabs one dependent round trip at a time (8 launches: 83 -> 69 us per step)
      for (; q + 7 * T < nsl; q += 8 * T) {
        float t8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t8[u] = pp[(long)(q + u * T) * ss];
#pragma unroll
        for (int u = 0; u < 8; ++u) d += t8[u];
      }
      for (; q < nsl; q += T) d += pp[(long)q * ss];
    }
    d = group_sum(d, T);
    if (e < nval && sub == 0) dzs[m][n - n0] = d * act_grad_from_out(y[(long)m * Nout + n], act);
  }
  __syncthreads();
  if (blockIdx.x == 0 && db) {
    for (int r = threadIdx.x; r < rows; r += 256) {
      float sb = 0.f;
      for (int m = 0; m < M; ++m) sb += dzs[m][r];
      db[n0 + r] = accumulate ? db[n0 + r] + sb : sb;
    }
  }
  const int k = blockIdx.x * 64 + tx;
  float acc[MMAX], xk[MMAX];
#pragma unroll
  for (int m = 0; m < MMAX; ++m) {
    acc[m] = 0.f;
    xk[m] = (m < M && k < K) ? x[(long)m * K + k] : 0.f;
  }
  if (k < K) {
    // LBR rows' weights (and old dW) loaded together before any is used: the pass streams W and
    // dW once, and with one 4-B load per lane in flight its rate was latency-bound (bytes in
    // flight / latency); same accumulation order as row-at-a-time
    for (int r0 = ty; r0 < rows; r0 += 4 * LBR) {
      float wv[LBR], dwo[LBR];
#pragma unroll
      for (int u = 0; u < LBR; ++u) {
        const int r = r0 + 4 * u;
        wv[u] = r < rows ? w[(long)(n0 + r) * K + k] : 0.f;
        dwo[u] = accumulate && r < rows ? dw[(long)(n0 + r) * K + k] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < LBR; ++u) {
        const int r = r0 + 4 * u;
        if (r < rows) {
          float g = 0.f;
#pragma unroll
          for (int m = 0; m < MMAX; ++m) {
            if (m < M) {
              const float dz = dzs[m][r];
              acc[m] += dz * wv[u];
              g += dz * xk[m];
            }
          }
          dw[(long)(n0 + r) * K + k] = accumulate ? dwo[u] + g : g;
        }
      }
    }
  }
  if (!dxp) return;
#pragma unroll
  for (int m = 0; m < MMAX; ++m) red[ty][m][tx] = acc[m];
  __syncthreads();
  if (ty == 0 && k < K) {
    for (int m = 0; m < M; ++m)
      dxp[((long)blockIdx.y * M + m) * K + k] = ((red[0][m][tx] + red[1][m][tx]) + red[2][m][tx]) + red[3][m][tx];
  }
}

// ------------------------------------------------------------------------ spatial + combine (forward)
// SpatialWeights' second 1x1 conv + sigmoid (net_utils.py:79-83) fused with the rectification
// (:147-152): per row, sw = sigmoid(relu(h) . w2 + b2) (saved for the backward), then
//   out1 = x1 + 0.5*cw1*x2 + 0.5*sw1*x2 ;  out2 = x2 + 0.5*cw0*x1 + 0.5*sw0*x1
template <typename T, int TPR>
__global__ __launch_bounds__(256) void combine_fwd_kernel(const T* __restrict__ x, const float* __restrict__ cw,
                                                          const T* __restrict__ h, const float* __restrict__ w2,
                                                          const float* __restrict__ b2, float* __restrict__ sw,
                                                          T* __restrict__ out, int B, int N, int C) {
  constexpr int V = VecT<T>::N, RPB = 256 / TPR;
  const int lane = threadIdx.x % TPR, slot = threadIdx.x / TPR;
  const int nch = C / V;
  const long rows = (long)B * N, per = rows * C;
  float wa[MAXCH][V], wb[MAXCH][V];
#pragma unroll
  for (int k = 0; k < MAXCH; ++k)
#pragma unroll
    for (int j = 0; j < V; ++j) {
      // unconditional loads (a lane past the row reads chunk 0), zeroed by a select after: under
      // `ok ? w2[c] : 0` each was sunk into its branch and waited for, 2 V MAXCH round trips
      const int c = (lane + k * TPR < nch ? lane + k * TPR : 0) * V + j;
      wa[k][j] = w2[c];
      wb[k][j] = w2[C + c];
    }
#pragma unroll
  for (int k = 0; k < MAXCH; ++k)
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const bool ok = lane + k * TPR < nch;
      wa[k][j] = ok ? wa[k][j] : 0.f;
      wb[k][j] = ok ? wb[k][j] : 0.f;
    }
  for (long row = (long)blockIdx.x * RPB + slot; row < rows; row += (long)gridDim.x * RPB) {
    const int b = (int)(row / N);
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int k = 0; k < MAXCH; ++k) {
      const int ch = lane + k * TPR;
      if (ch >= nch) continue;
      float v[V];
      load_vec<T>(h + row * C + ch * V, v);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float r = v[j] > 0.f ? v[j] : 0.f;
        s0 += r * wa[k][j];
        s1 += r * wb[k][j];
      }
    }
    s0 = group_sum(s0, TPR);
    s1 = group_sum(s1, TPR);
    const float sw0 = 1.f / (1.f + __expf(-(s0 + b2[0]))), sw1 = 1.f / (1.f + __expf(-(s1 + b2[1])));
    if (lane == 0) { sw[row * 2] = sw0; sw[row * 2 + 1] = sw1; }
    const float h0 = 0.5f * sw0, h1 = 0.5f * sw1;
#pragma unroll
    for (int k = 0; k < MAXCH; ++k) {
      const int ch = lane + k * TPR;
      if (ch >= nch) continue;
      const long e = row * C + ch * V;
      float a[V], bb[V], o1[V], o2[V];
      load_vec<T>(x + e, a);
      load_vec<T>(x + per + e, bb);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float c0w = 0.5f * cw[(long)b * 2 * C + ch * V + j];
        const float c1w = 0.5f * cw[(long)b * 2 * C + C + ch * V + j];
        o1[j] = (a[j] + c1w * bb[j]) + h1 * bb[j];
        o2[j] = (bb[j] + c0w * a[j]) + h0 * a[j];
      }
      store_vec<T>(out + e, o1);
      store_vec<T>(out + per + e, o2);
    }
  }
}

// ------------------------------------------------------------------------ combine + spatial (backward)
// Per row: the direct-path dx of the rectification; dsw (row sums); the spatial head's backward
// dz2 = dsw * sw (1 - sw), dh = [h > 0] (dz2 . w2).  Per block (blockIdx = (slab, b)): partials
// dcw (B, nblk, 2C) = [dcw0 | dcw1] and [dw2 (2C) | db2 (2)] (B * nblk, 2C + 2), combined over
// the block's row slots in LDS (no atomics: deterministic).
template <typename T, int TPR, int MCH>
__global__ __launch_bounds__(256) void combine_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ dout2,
                                                          const T* __restrict__ x,
                                                          const float* __restrict__ cw, const float* __restrict__ sw,
                                                          const T* __restrict__ h, const float* __restrict__ w2,
                                                          T* __restrict__ dx, T* __restrict__ dh,
                                                          float* __restrict__ pcw, float* __restrict__ psp, int B,
                                                          int N, int C) {
  constexpr int V = VecT<T>::N, RPB = 256 / TPR, CMAX = MCH * TPR * V;
  __shared__ float red[RPB][CMAX];
  __shared__ float rdb[2][RPB];
  const int b = blockIdx.y, nblk = gridDim.x;
  const int lane = threadIdx.x % TPR, slot = threadIdx.x / TPR;
  const int nch = C / V;
  const long per = (long)B * N * C;
  float a0[MCH][V], a1[MCH][V], p0[MCH][V], p1[MCH][V];
#pragma unroll
  for (int k = 0; k < MCH; ++k)
#pragma unroll
    for (int j = 0; j < V; ++j) a0[k][j] = a1[k][j] = p0[k][j] = p1[k][j] = 0.f;
  float db0 = 0.f, db1 = 0.f;
  // per-channel constants of this block's image (blockIdx.y = b), loaded once
  float c0h[MCH][V], c1h[MCH][V], wa[MCH][V], wb[MCH][V];
#pragma unroll
  for (int k = 0; k < MCH; ++k)
#pragma unroll
    for (int j = 0; j < V; ++j) {
      // unconditional loads (a lane past the row reads chunk 0), zeroed by a select after (as
      // combine_fwd_kernel: conditional loads were one round trip each)
      const int c = (lane + k * TPR < nch ? lane + k * TPR : 0) * V + j;
      c0h[k][j] = cw[(long)b * 2 * C + c];
      c1h[k][j] = cw[(long)b * 2 * C + C + c];
      wa[k][j] = w2[c];
      wb[k][j] = w2[C + c];
    }
#pragma unroll
  for (int k = 0; k < MCH; ++k)
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const bool ok = lane + k * TPR < nch;
      c0h[k][j] = ok ? 0.5f * c0h[k][j] : 0.f;
      c1h[k][j] = ok ? 0.5f * c1h[k][j] : 0.f;
      wa[k][j] = ok ? wa[k][j] : 0.f;
      wb[k][j] = ok ? wb[k][j] : 0.f;
    }
  for (int n = blockIdx.x * RPB + slot; n < N; n += nblk * RPB) {
    const long row = (long)b * N + n;
    const float sw0 = sw[row * 2], sw1 = sw[row * 2 + 1];
    const float s0 = 0.5f * sw0, s1 = 0.5f * sw1;
    float r0 = 0.f, r1 = 0.f;
#pragma unroll
    for (int k = 0; k < MCH; ++k) {
      const int ch = lane + k * TPR;
      if (ch >= nch) continue;
      const long e = row * C + ch * V;
      float d1[V], d2[V], x1[V], x2[V], o1[V], o2[V];
      load_vec<T>(dout + e, d1);
      load_vec<T>(dout + per + e, d2);
      if (dout2) {    // the output's second consumer: summed (and rounded) as autograd's add would
        float e1[V], e2[V];
        load_vec<T>(dout2 + e, e1);
        load_vec<T>(dout2 + per + e, e2);
#pragma unroll
        for (int j = 0; j < V; ++j) {
          d1[j] = to_f32(from_f32<T>(d1[j] + e1[j]));
          d2[j] = to_f32(from_f32<T>(d2[j] + e2[j]));
        }
      }
      load_vec<T>(x + e, x1);
      load_vec<T>(x + per + e, x2);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float c0w = c0h[k][j], c1w = c1h[k][j];
        o1[j] = d1[j] + (c0w + s0) * d2[j];
        o2[j] = d2[j] + (c1w + s1) * d1[j];
        const float q1 = d1[j] * x2[j];   // feeds dcw1, dsw1
        const float q0 = d2[j] * x1[j];   // feeds dcw0, dsw0
        r1 += q1; r0 += q0;
        a1[k][j] += q1; a0[k][j] += q0;
      }
      store_vec<T>(dx + e, o1);
      store_vec<T>(dx + per + e, o2);
    }
    r0 = group_sum(r0, TPR);
    r1 = group_sum(r1, TPR);
    const float g0 = 0.5f * r0 * sw0 * (1.f - sw0), g1 = 0.5f * r1 * sw1 * (1.f - sw1);
    if (lane == 0) { db0 += g0; db1 += g1; }
#pragma unroll
    for (int k = 0; k < MCH; ++k) {
      const int ch = lane + k * TPR;
      if (ch >= nch) continue;
      const long e = row * C + ch * V;
      float v[V], o[V];
      load_vec<T>(h + e, v);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const bool pos = v[j] > 0.f;
        o[j] = pos ? g0 * wa[k][j] + g1 * wb[k][j] : 0.f;
        const float r = pos ? v[j] : 0.f;
        p0[k][j] += g0 * r;
        p1[k][j] += g1 * r;
      }
      store_vec<T>(dh + e, o);
    }
  }
  // slot-combine the four per-channel partials, one quantity at a time through LDS
  float* outc = pcw + ((long)b * nblk + blockIdx.x) * 2 * C;
  float* outs = psp + ((long)b * nblk + blockIdx.x) * (2 * C + 2);
#pragma unroll
  for (int qn = 0; qn < 4; ++qn) {             // unrolled: a runtime pick among the four arrays
#pragma unroll                                   // would put them in scratch memory
    for (int k = 0; k < MCH; ++k)
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int c = (lane + k * TPR) * V + j;
        const float v = qn == 0 ? a0[k][j] : qn == 1 ? a1[k][j] : qn == 2 ? p0[k][j] : p1[k][j];
        if (c < C) red[slot][c] = v;
      }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      float t = 0.f;
      for (int q = 0; q < RPB; ++q) t += red[q][c];
      if (qn < 2) outc[qn * C + c] = 0.5f * t;
      else outs[(qn - 2) * C + c] = t;
    }
    __syncthreads();
  }
  if (lane == 0) { rdb[0][slot] = db0; rdb[1][slot] = db1; }
  __syncthreads();
  if (threadIdx.x < 2) {
    float t = 0.f;
    for (int q = 0; q < RPB; ++q) t += rdb[threadIdx.x][q];
    outs[2 * C + threadIdx.x] = t;
  }
}

// ------------------------------------------------------------------------ pooling (backward)
constexpr int PB_SL = 16;                       // partial slices of dpooled (small_linear_bwd's NSLICE)
// dx[g][b][n][c] += dpooled_avg[b][gC+c] / N + (n == argmax[b][gC+c]) * dpooled_max[b][2C+gC+c];
// dpooled arrives as partial slices dp[b][k] = sum_s part[s*ss + b*sm + k].
template <typename T, int TPR>
__global__ __launch_bounds__(256) void pool_bwd_kernel(const float* __restrict__ part, int nsl, long ss, long sm,
                                                       const int* __restrict__ argmax, T* __restrict__ dx, int B,
                                                       int N, int C) {
  constexpr int V = VecT<T>::N, RPB = 256 / TPR;
  __shared__ float sdp[2 * 1024];                 // [avg | max] gradient of this (g, b), C <= 1024
  const int gb = blockIdx.y, g = gb / B, b = gb % B;
  const int lane = threadIdx.x % TPR, slot = threadIdx.x / TPR;
  const int nch = C / V;
  // the block's 2C dpooled values, each summed over the nsl (<= PB_SL) partial slices, once per
  // block: every slice's load issued before the sum (a runtime-bounded serial loop waited one
  // L2 round trip per slice: 18 us per launch at stages 3 / 4)
  for (int e = threadIdx.x; e < 2 * C; e += 256) {
    const int k = e < C ? g * C + e : 2 * C + g * C + (e - C);
    const float* p = part + b * sm + k;
    float v[PB_SL];
#pragma unroll
    for (int q = 0; q < PB_SL; ++q) v[q] = p[(q < nsl ? q : 0) * ss];     // (unconditional: in flight together)
#pragma unroll
    for (int q = 0; q < PB_SL; ++q) v[q] = q < nsl ? v[q] : 0.f;
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < PB_SL; ++q) t += v[q];
    sdp[e] = e < C ? t / N : t;
  }
  __syncthreads();
  float dav[MAXCH][V], dmx[MAXCH][V];
  int am[MAXCH][V];
#pragma unroll
  for (int k = 0; k < MAXCH; ++k)
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = (lane + k * TPR) * V + j;
      const bool ok = lane + k * TPR < nch;
      dav[k][j] = ok ? sdp[c] : 0.f;
      dmx[k][j] = ok ? sdp[C + c] : 0.f;
      am[k][j] = argmax[(long)b * 2 * C + g * C + (ok ? c : 0)];        // (unconditional, selected below)
    }
#pragma unroll
  for (int k = 0; k < MAXCH; ++k)
#pragma unroll
    for (int j = 0; j < V; ++j) am[k][j] = lane + k * TPR < nch ? am[k][j] : -1;
  T* base = dx + (long)gb * N * C;
  for (int n = blockIdx.x * RPB + slot; n < N; n += gridDim.x * RPB) {
#pragma unroll
    for (int k = 0; k < MAXCH; ++k) {
      const int ch = lane + k * TPR;
      if (ch >= nch) continue;
      float v[V];
      T* p = base + (long)n * C + ch * V;
      load_vec<T>(p, v);
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] += dav[k][j] + (am[k][j] == n ? dmx[k][j] : 0.f);
      store_vec<T>(p, v);
    }
  }
}

// token chunks per (channel group, image): ~1024 blocks in all, >= 16 tokens each, <= PZ_MAX
int pool_nchunk(int N, int GB, int C) {
  const long blocks_per_z = (long)GB * (C / PG);
  long nz = (1024 + blocks_per_z - 1) / blocks_per_z;
  const long maxz = (N + 15) / 16;
  if (nz > maxz) nz = maxz;
  if (nz > PZ_MAX) nz = PZ_MAX;
  return nz < 1 ? 1 : (int)nz;
}
int combine_nblk(int N, int C, int V) {        // blocks per image of the backward (<= 256: its partials are
  const int rpb = 256 / row_lanes(C, V);       // summed by the channel-MLP backward's prologue)
  int nb = (N + rpb - 1) / rpb;
  return nb < 256 ? nb : 256;
}
unsigned rows_grid(long rows, int rpb) {
  const long g = (rows + rpb - 1) / rpb;
  return (unsigned)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

#define FRM_TPR_DISPATCH(tpr, TPR, ...)                   \
  do {                                                    \
    switch (tpr) {                                        \
      case 4: { constexpr int TPR = 4; __VA_ARGS__; break; }   \
      case 8: { constexpr int TPR = 8; __VA_ARGS__; break; }   \
      case 16: { constexpr int TPR = 16; __VA_ARGS__; break; } \
      case 32: { constexpr int TPR = 32; __VA_ARGS__; break; } \
      default: { constexpr int TPR = 64; __VA_ARGS__; break; } \
    }                                                     \
  } while (0)

}  // namespace

extern "C" {

size_t cmx_frm_pool_workspace(int B, int N, int C) {
  const int nz = pool_nchunk(N, 2 * B, C > 0 ? C : PG);
  return (size_t)2 * B * nz * (C > 0 ? C : 0) * 3 * sizeof(float);
}

size_t cmx_frm_pool_tickets(int B, int C) { return (size_t)2 * B * (C / PG); }

int cmx_frm_pool_fwd(const void* x, float* pooled, int* argmax, float* workspace, unsigned* tickets, int B, int N, int C,
                     int dtype, hipStream_t s) {
  CMX_REQUIRE(B > 0 && N > 0 && C > 0 && C % PG == 0 && 2L * B * (C / PG) <= POOL_TICKETS, CMX_ERR_SHAPE,
              "frm_pool: B=%d N=%d C=%d (C %% %d == 0)", B, N, C, PG);
  const int nz = pool_nchunk(N, 2 * B, C);
  const int chunk = (N + nz - 1) / nz;
  float* psum = workspace;
  float* pmax = psum + (size_t)2 * B * nz * C;
  int* pidx = (int*)(pmax + (size_t)2 * B * nz * C);
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(pool_kernel<T>, dim3(nz, C / PG, 2 * B), dim3(256), 0, s, (const T*)x, psum, pmax, pidx,
                       pooled, argmax, B, N, C, chunk, tickets);
  });
  return cmx_check_launch("frm_pool_fwd");
}

int cmx_frm_pool_bwd(const float* dpooled_part, int nslice, int64_t slice_stride, const int* argmax, void* dx, int B,
                     int N, int C, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0 && C / V <= MAXCH * 64 && C <= 1024 && nslice > 0 && nslice <= PB_SL, CMX_ERR_SHAPE,
              "frm_pool_bwd: C=%d nslice=%d", C, nslice);
  const int tpr = row_lanes(C, V);
  const int rpb = 256 / tpr;
  long nb = (N + rpb - 1) / rpb;
  const long want = (512 + 2 * B - 1) / (2 * B);
  if (nb > want) nb = want;
  CMX_DISPATCH(dtype, T, {
    FRM_TPR_DISPATCH(tpr, TPR, hipLaunchKernelGGL((pool_bwd_kernel<T, TPR>), dim3((unsigned)nb, 2 * B), dim3(256), 0,
                                                  s, dpooled_part, nslice, (long)slice_stride, (long)4 * C, argmax,
                                                  (T*)dx, B, N, C));
  });
  return cmx_check_launch("frm_pool_bwd");
}

int cmx_small_linear_fwd(const float* x, const float* w, const float* b, float* y, int M, int K, int Nout, int act,
                         hipStream_t s) {
  CMX_REQUIRE(M > 0 && M <= MMAX && K % 4 == 0 && (long)M * K * 4 <= 64 * 1024 && ((uintptr_t)w & 15) == 0 &&
              ((uintptr_t)x & 15) == 0, CMX_ERR_SHAPE, "small_linear_fwd: M=%d K=%d", M, K);
  const unsigned grid = cdiv(Nout, 4 * LIN_FPW);
  hipLaunchKernelGGL(linear_fwd_kernel, dim3(grid), dim3(256), (size_t)M * K * sizeof(float), s, x, w, b, y, M, K,
                     Nout, act);
  return cmx_check_launch("small_linear_fwd");
}

int cmx_small_linear_nslice(void) { return NSLICE; }

size_t cmx_small_linear_bwd_workspace(int M, int K, int Nout) { return (size_t)NSLICE * M * K * sizeof(float); }

int cmx_small_linear_bwd(const float* dy_part, int dy_nslice, int64_t dy_slice_stride, int64_t dy_row_stride,
                         const float* y, const float* x, const float* w, float* dx_part, float* dw, float* db, int M,
                         int K, int Nout, int act, int accumulate, hipStream_t s) {
  CMX_REQUIRE(M > 0 && M <= MMAX && dy_nslice > 0 && (Nout + NSLICE - 1) / NSLICE <= SLICE_MAX, CMX_ERR_SHAPE,
              "small_linear_bwd: M=%d Nout=%d", M, Nout);
  hipLaunchKernelGGL(linear_bwd_kernel, dim3(cdiv(K, 64), NSLICE), dim3(256), 0, s, dy_part, dy_nslice,
                     (long)dy_slice_stride, (long)dy_row_stride, y, x, w, dx_part, dw, db, M, K, Nout, act,
                     accumulate);
  return cmx_check_launch("small_linear_bwd");
}

int cmx_frm_combine_fwd(const void* x, const float* cw, const void* h, const float* w2, const float* b2, float* sw,
                        void* out, int B, int N, int C, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0 && C / V <= MAXCH * 64, CMX_ERR_SHAPE, "frm_combine: C=%d", C);
  const int tpr = row_lanes(C, V);
  const unsigned grid = rows_grid((long)B * N, 256 / tpr);
  CMX_DISPATCH(dtype, T, {
    FRM_TPR_DISPATCH(tpr, TPR, hipLaunchKernelGGL((combine_fwd_kernel<T, TPR>), dim3(grid), dim3(256), 0, s,
                                                  (const T*)x, cw, (const T*)h, w2, b2, sw, (T*)out, B, N, C));
  });
  return cmx_check_launch("frm_combine_fwd");
}

int cmx_frm_combine_bwd_nblk(int N, int C, int dtype) { return combine_nblk(N, C, dtype == 0 ? 4 : 8); }

size_t cmx_frm_combine_bwd_workspace(int B, int N, int C, int dtype) {
  const int nb = combine_nblk(N, C, dtype == 0 ? 4 : 8);
  return ((size_t)B * nb * 2 * C + (size_t)B * nb * (2 * C + 2)) * sizeof(float);
}

// dx (2,B,N,C) direct path, dh (B*N, C); workspace: dcw partials (B, nblk, 2C) then the
// [dw2 | db2] partials (B * nblk, 2C + 2); dout2 (may be NULL): a second gradient of the output
int cmx_frm_combine_bwd(const void* dout, const void* dout2, const void* x, const float* cw, const float* sw, const void* h,
                        const float* w2, void* dx, void* dh, float* workspace, int B, int N, int C, int dtype,
                        hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0 && C / V <= MAXCH * 64, CMX_ERR_SHAPE, "frm_combine_bwd: C=%d", C);
  const int nb = combine_nblk(N, C, V);
  const int tpr = row_lanes(C, V);
  float* pcw = workspace;
  float* psp = workspace + (size_t)B * nb * 2 * C;
  // chunks per lane: 1 unless the row has more than 64 chunks (fp32 with C > 256); the
  // one-chunk instantiation keeps the per-channel accumulators at half the registers
#define CMX_CB(MCH_) FRM_TPR_DISPATCH(tpr, TPR, hipLaunchKernelGGL((combine_bwd_kernel<T, TPR, MCH_>), dim3(nb, B), \
                                                  dim3(256), 0, s, (const T*)dout, (const T*)dout2, (const T*)x, cw, sw, (const T*)h, \
                                                  w2, (T*)dx, (T*)dh, pcw, psp, B, N, C))
  CMX_DISPATCH(dtype, T, {
    if (C / V <= tpr) CMX_CB(1);
    else CMX_CB(2);
  });
#undef CMX_CB
  return cmx_check_launch("frm_combine_bwd");
}

}  // extern "C"
