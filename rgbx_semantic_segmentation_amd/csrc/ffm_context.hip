// FFM cross-attention (efficient / linear attention) of CrossAttention.forward
// (net_utils.py:199-214):
//   ctx_g = softmax_{dim=-2}( k_g^T v_g * d^-1/2 )      (a D x D matrix per (b, head))
//   out_1 = q_1 @ ctx_2 ,  out_2 = q_2 @ ctx_1         (contexts crossed between modalities)
// q is the raw (ReLU'd) channel_proj half u, k/v the two halves of the kv projection.
//
// Kernels
//  ctx_reduce   : partial sums of X^T Y over a chunk of tokens, slab (nchunk, BH, D*D)
//  ctx_finalize : sum the slab and apply (mode 0) scale, (1) softmax over rows with scale,
//                 (2) the softmax backward dA = s * ctx * (dctx - colsum(ctx * dctx));
//                 optional modality swap of the output / ctx index
//  rowmat       : out[n, head*D + j] (+)= alpha * sum_i X[n, head*D + i] * M[i, j] (or M^T),
//                 M optionally taken from the other modality group (the crossing)
// Layout: token-major rows with explicit row strides; BH index = (g*B + b)*heads + head.
// These are skinny (K = D = 64) products; fp32 FMA on the VALU with LDS tiles.
#include "cmx_common.h"

namespace {
constexpr int NT = 64;  // tokens per LDS tile

template <typename T, int D>
__global__ __launch_bounds__(256) void ctx_reduce_kernel(const T* __restrict__ X, const T* __restrict__ Y,
                                                         float* __restrict__ slab, int N, int heads, long xs,
                                                         long ys, int chunk, int nchunk, int BH) {
  __shared__ float Xs[NT][D + 4];
  __shared__ float Ys[NT][D + 4];
  constexpr int TPD = D / 4;                 // threads per output dim
  const int bh = blockIdx.y, c = blockIdx.x;
  const int b = bh / heads, head = bh % heads;
  const int ti = threadIdx.x / TPD, tj = threadIdx.x % TPD;
  const bool act = threadIdx.x < TPD * TPD;
  float acc[4][4] = {};
  const int n0 = c * chunk, n1 = min(N, n0 + chunk);
  const T* xb = X + (long)b * N * xs + head * D;
  const T* yb = Y + (long)b * N * ys + head * D;
  constexpr int V = VecT<T>::N;
  for (int t0 = n0; t0 < n1; t0 += NT) {
    __syncthreads();
    for (int e = threadIdx.x; e < NT * (D / V); e += 256) {
      const int r = e / (D / V), ch = e % (D / V);
      float xv[V], yv[V];
      if (t0 + r < n1) {
        load_vec<T>(xb + (long)(t0 + r) * xs + ch * V, xv);
        load_vec<T>(yb + (long)(t0 + r) * ys + ch * V, yv);
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) xv[j] = yv[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < V; ++j) { Xs[r][ch * V + j] = xv[j]; Ys[r][ch * V + j] = yv[j]; }
    }
    __syncthreads();
    if (act) {
#pragma unroll 4
      for (int n = 0; n < NT; ++n) {
        const float4 xi = *reinterpret_cast<const float4*>(&Xs[n][ti * 4]);
        const float4 yj = *reinterpret_cast<const float4*>(&Ys[n][tj * 4]);
        const float xa[4] = {xi.x, xi.y, xi.z, xi.w}, ya[4] = {yj.x, yj.y, yj.z, yj.w};
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int bb = 0; bb < 4; ++bb) acc[a][bb] += xa[a] * ya[bb];
      }
    }
  }
  if (!act) return;
  float* out = slab + ((long)c * BH + bh) * D * D;
#pragma unroll
  for (int a = 0; a < 4; ++a)
    *reinterpret_cast<float4*>(&out[(ti * 4 + a) * D + tj * 4]) =
        make_float4(acc[a][0], acc[a][1], acc[a][2], acc[a][3]);
}

// one block per BH; thread per column j (D threads) for the softmax modes
template <int D>
__global__ __launch_bounds__(256) void ctx_finalize_kernel(const float* __restrict__ slab, const float* __restrict__ ctx,
                                                           float* __restrict__ out, int nchunk, int BH, int mode,
                                                           float alpha, int swapB, int heads) {
  // 256 threads: column j = tid % D, row slice rg = tid / D (256 / D slices); per-column max /
  // sum / dot over the slices meet in LDS (one thread per column walking D rows serially, with
  // three exp passes, took ~30 us per launch)
  constexpr int NS = 256 / D;
  const int bh = blockIdx.x;
  int obh = bh;
  if (swapB > 0) {  // (g, b, head) -> (1 - g, b, head)
    const int g = bh / (swapB * heads), rest = bh % (swapB * heads);
    obh = (1 - g) * swapB * heads + rest;
  }
  __shared__ float S[D][D + 1];
  __shared__ float red[NS][D];
  for (int e = threadIdx.x; e < D * D; e += 256) {
    float sm = 0.f;
    for (int c = 0; c < nchunk; ++c) sm += slab[((long)c * BH + bh) * D * D + e];
    S[e / D][e % D] = sm;
  }
  __syncthreads();
  float* o = out + (long)obh * D * D;
  if (mode == 0) {
    for (int e = threadIdx.x; e < D * D; e += 256) o[e] = alpha * S[e / D][e % D];
    return;
  }
  const int j = threadIdx.x % D, rg = threadIdx.x / D;
  constexpr int RPS = D / NS;                    // rows per slice
  const int i0 = rg * RPS;
  if (mode == 1) {                               // softmax over rows i (dim -2) of column j
    float m = -INFINITY;
    for (int i = i0; i < i0 + RPS; ++i) m = fmaxf(m, alpha * S[i][j]);
    red[rg][j] = m;
    __syncthreads();
    m = red[0][j];
#pragma unroll
    for (int q = 1; q < NS; ++q) m = fmaxf(m, red[q][j]);
    __syncthreads();
    float l = 0.f;
    for (int i = i0; i < i0 + RPS; ++i) l += __expf(alpha * S[i][j] - m);
    red[rg][j] = l;
    __syncthreads();
    l = 0.f;
#pragma unroll
    for (int q = 0; q < NS; ++q) l += red[q][j];
    const float inv = 1.f / l;
    for (int i = i0; i < i0 + RPS; ++i) o[i * D + j] = __expf(alpha * S[i][j] - m) * inv;
  } else {
    // S holds dctx for context obh; ctx (BH, D, D)
    const float* cx = ctx + (long)obh * D * D;
    float dot = 0.f;
    for (int i = i0; i < i0 + RPS; ++i) dot += cx[i * D + j] * S[i][j];
    red[rg][j] = dot;
    __syncthreads();
    dot = 0.f;
#pragma unroll
    for (int q = 0; q < NS; ++q) dot += red[q][j];
    for (int i = i0; i < i0 + RPS; ++i) o[i * D + j] = alpha * cx[i * D + j] * (S[i][j] - dot);
  }
}

template <typename T, int D>
__global__ __launch_bounds__(256) void rowmat_kernel(const T* __restrict__ X, const float* __restrict__ M,
                                                     T* __restrict__ out, int N, int heads, long xs, long os,
                                                     int trans, float alpha, int accumulate, int swapB) {
  __shared__ float Ms[D][D + 4];
  __shared__ float Xs[NT][D + 1];
  constexpr int V = VecT<T>::N;
  const int bh = blockIdx.y;
  const int b = bh / heads, head = bh % heads;
  int mbh = bh;
  if (swapB > 0) {
    const int g = bh / (swapB * heads), rest = bh % (swapB * heads);
    mbh = (1 - g) * swapB * heads + rest;
  }
  const float* mp = M + (long)mbh * D * D;
  for (int e = threadIdx.x; e < D * D; e += 256) {
    const int i = e / D, j = e % D;
    Ms[i][j] = trans ? mp[j * D + i] : mp[i * D + j];
  }
  const int n0 = blockIdx.x * NT;
  const T* xb = X + (long)b * N * xs + head * D;
  for (int e = threadIdx.x; e < NT * (D / V); e += 256) {
    const int r = e / (D / V), ch = e % (D / V);
    float xv[V];
    if (n0 + r < N) {
      load_vec<T>(xb + (long)(n0 + r) * xs + ch * V, xv);
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) xv[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < V; ++j) Xs[r][ch * V + j] = xv[j];
  }
  __syncthreads();
  // thread -> 4 consecutive output columns of (NT * D / 4 / 256) rows
  constexpr int CG = D / 4;                 // column groups
  constexpr int RPT = NT * CG / 256;        // rows per thread
  const int cg = threadIdx.x % CG;
  const int rbase = threadIdx.x / CG;
  constexpr int RSTEP = 256 / CG;
  float acc[RPT][4] = {};
#pragma unroll 8
  for (int i = 0; i < D; ++i) {
    const float4 m4 = *reinterpret_cast<const float4*>(&Ms[i][cg * 4]);
#pragma unroll
    for (int rr = 0; rr < RPT; ++rr) {
      const float xv = Xs[rbase + rr * RSTEP][i];
      acc[rr][0] += xv * m4.x; acc[rr][1] += xv * m4.y; acc[rr][2] += xv * m4.z; acc[rr][3] += xv * m4.w;
    }
  }
  T* ob = out + (long)b * N * os + head * D;
#pragma unroll
  for (int rr = 0; rr < RPT; ++rr) {
    const int n = n0 + rbase + rr * RSTEP;
    if (n >= N) continue;
    T* p = ob + (long)n * os + cg * 4;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float v = alpha * acc[rr][u];
      if (accumulate) v += to_f32(p[u]);
      p[u] = from_f32<T>(v);
    }
  }
}

int ctx_nchunk(int N, int BH) {
  // aim for ~512 blocks, chunks of at least NT tokens
  long nc = (512 + BH - 1) / BH;
  const long maxc = (N + NT - 1) / NT;
  if (nc > maxc) nc = maxc;
  return nc < 1 ? 1 : (int)nc;
}
}  // namespace

#define CTX_D_DISPATCH(D, ...)                                           \
  do {                                                                   \
    if ((D) == 64) { constexpr int DD = 64; __VA_ARGS__; }               \
    else if ((D) == 32) { constexpr int DD = 32; __VA_ARGS__; }          \
    else { cmx_set_error("ffm ctx: D=%d unsupported", (int)(D)); return CMX_ERR_SHAPE; } \
  } while (0)

extern "C" {

size_t cmx_ffm_ctx_workspace(int BH, int N, int D) {
  return ((size_t)ctx_nchunk(N, BH) + 1) * BH * D * D * sizeof(float);
}

// out (BH, D, D) fp32 = finalize(sum_n X^T Y); mode 0: alpha*sum; 1: softmax over dim -2 of
// alpha*sum; 2: softmax backward using ctx (the sum is dctx).  swapB > 0 writes the
// result of (g, b) to (1-g, b) (B = swapB per group).
int cmx_ffm_ctx_reduce(const void* X, const void* Y, const float* ctx, float* out, float* workspace, int Bt,
                       int N, int heads, int D, int64_t xs, int64_t ys, int mode, float alpha, int swapB,
                       int dtype, hipStream_t s) {
  const int BH = Bt * heads;
  CMX_REQUIRE(Bt > 0 && N > 0 && xs % 8 == 0 && ys % 8 == 0, CMX_ERR_SHAPE, "ffm_ctx_reduce: shape");
  CMX_REQUIRE(mode != 2 || ctx, CMX_ERR_ARG, "ffm_ctx_reduce: mode 2 needs ctx");
  const int nc = ctx_nchunk(N, BH);
  const int chunk = (N + nc - 1) / nc;
  CTX_D_DISPATCH(D, CMX_DISPATCH(dtype, T, {
    float* sum = workspace + (size_t)nc * BH * DD * DD;
    hipLaunchKernelGGL((ctx_reduce_kernel<T, DD>), dim3(nc, BH), dim3(256), 0, s, (const T*)X, (const T*)Y,
                       workspace, N, heads, (long)xs, (long)ys, chunk, nc, BH);
    const int st = cmx_reduce_partials(workspace, sum, 1, nc, BH * DD * DD, 0, 1.f, s);
    if (st) return st;
    hipLaunchKernelGGL((ctx_finalize_kernel<DD>), dim3(BH), dim3(256), 0, s, sum, ctx, out, 1, BH, mode,
                       alpha, swapB, heads);
  }));
  return cmx_check_launch("ffm_ctx_reduce");
}

int cmx_ffm_rowmat(const void* X, const float* M, void* out, int Bt, int N, int heads, int D, int64_t xs,
                   int64_t os, int trans, float alpha, int accumulate, int swapB, int dtype, hipStream_t s) {
  CMX_REQUIRE(Bt > 0 && N > 0 && xs % 8 == 0, CMX_ERR_SHAPE, "ffm_rowmat: shape");
  CTX_D_DISPATCH(D, CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((rowmat_kernel<T, DD>), dim3(cdiv(N, NT), Bt * heads), dim3(256), 0, s, (const T*)X, M,
                       (T*)out, N, heads, (long)xs, (long)os, trans, alpha, accumulate, swapB);
  }));
  return cmx_check_launch("ffm_rowmat");
}

}  // extern "C"
