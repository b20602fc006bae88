// CM-FRM channel branch as ONE launch per direction: the north_star's "global-pool + 1x1 as one
// wavefront-reduction + GEMV op" -- ChannelWeights (net_utils.py:11-30) as FeatureRectifyModule
// calls it (:145) on token-major x (2, B, N, C) = (x1, x2).
//
//  cmx_frm_channel_fwd   avg || max pooling of cat(x1, x2) over H*W (:22-27)
//                          -> pooled (B, 4C) = [avg x1 | avg x2 | max x1 | max x2], argmax (B, 2C)
//                        y1 = relu(pooled W1^T + b1) (B, 4C)   (mlp[0], mlp[1], :16-17)
//                        cw = sigmoid(y1 W2^T + b2) (B, 2C)    (mlp[2], mlp[3], :18-19)
//  cmx_frm_channel_bwd   dcw (the combine backward's per-block partial slabs) * sigmoid'
//                        -> W2 pass (dW2, dy1) -> W1 pass (dW1, db1, dpooled) -> pooling
//                        backward into dx (avg: 1/N to every token, max: to the FIRST argmax
//                        token, as PyTorch's CPU max pool routes it)
//
// One workgroup per CU, all resident at once; the phases are separated by grid barriers: an
// arrival counter in device memory that each block bumps once per barrier and polls until the
// whole grid has arrived, with agent-scope release / acquire fences around it so that a phase's
// global writes (held in eight non-coherent XCD L2s) are visible to every block after it.  The
// last block out resets the counters, so the barrier needs no host-side clearing and the launch
// is graph-capturable.  A poll bound turns a grid that could never become resident into a flag
// (cmx_frm_barrier_timeouts) instead of a hang, so every wave reaches the exit.  One barrier slot
// per direction: launches of one direction must not run concurrently (they serialise on the
// step's stream).
//
// Phase work is laid out for the chip, not per op: pooling = 16-B row loads over ~512 token
// chunks, the GEMVs = one wave per output feature with float4 weight rows (each weight byte
// read once), the weight passes = 64 k-columns x 8 row lanes per n-slice (dW written once, dx
// left as 16 slice partials summed by the next phase).
#include "cmx_common.h"
#include <algorithm>

namespace {

constexpr int NT = 512, NW = NT / 64;  // threads / waves per block
constexpr int MB = 8;                  // B <= 8 (rows of the channel MLP)
constexpr int NSL = 16;                // n-slices of the backward weight passes
constexpr int SLMAX = 256;             // rows per slice: Nout <= 16 * 256
constexpr int MAXCH = 2;               // 16-B chunks per lane of a token row
constexpr int PF_CH = 16, PF_SL = NT / PF_CH;

__device__ unsigned g_frm_bar[2][4];   // [fwd | bwd][arrivals, exits, timed out, -]

__device__ __forceinline__ void grid_sync(unsigned* bar, unsigned target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    atomicAdd(bar, 1u);
    int polls = 0;
    while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(4);
      if (++polls == (1 << 24)) {          // ~2 s: the grid cannot be resident
        atomicOr(bar + 2, 1u);
        break;
      }
    }
    __threadfence();
  }
  __syncthreads();
}

__device__ __forceinline__ void grid_exit(unsigned* bar) {
  if (threadIdx.x == 0) {
    const unsigned out = atomicAdd(bar + 1, 1u);
    if (out == gridDim.x - 1) {            // every other block is past its last poll
      atomicExch(bar, 0u);
      atomicExch(bar + 1, 0u);
    }
  }
}

inline int row_lanes(int C, int V) {
  int tpr = 4;
  while (tpr < C / V && tpr < 64) tpr <<= 1;
  return tpr;
}
int pool_chunks(int N, int GB) {
  long nc = (512 + GB - 1) / GB;
  const long maxc = (N + 15) / 16;
  if (nc > maxc) nc = maxc;
  return nc < 1 ? 1 : (int)nc;
}

// ---------------------------------------------------------------- forward phases
// partial sum / max / first argmax of one (token chunk, g*B + b); the block's row slots meet in
// LDS in two levels (NT / C thread groups per channel, then one thread per channel)
template <typename T, int TPR>
__device__ void pool_part(const T* x, float* psum, float* pmax, int* pidx, int gb, int ci, int nc, int N, int C,
                          int chunk, float* sh) {
  constexpr int V = VecT<T>::N, RPB = NT / TPR;
  float* rs = sh;
  float* rm = sh + RPB * C;
  int* ri = reinterpret_cast<int*>(sh + 2 * RPB * C);
  const int lane = threadIdx.x % TPR, slot = threadIdx.x / TPR, nch = C / V;
  const int n0 = ci * chunk, n1 = min(N, n0 + chunk);
  float sm[MAXCH][V], mx[MAXCH][V];
  int ix[MAXCH][V];
#pragma unroll
  for (int k = 0; k < MAXCH; ++k)
#pragma unroll
    for (int j = 0; j < V; ++j) { sm[k][j] = 0.f; mx[k][j] = -INFINITY; ix[k][j] = 0x7fffffff; }
  const T* base = x + (long)gb * N * C;
#pragma unroll 2
  for (int n = n0 + slot; n < n1; n += RPB) {
#pragma unroll
    for (int k = 0; k < MAXCH; ++k) {
      const int ch = lane + k * TPR;
      if (ch >= nch) continue;
      float v[V];
      load_vec<T>(base + (long)n * C + ch * V, v);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        sm[k][j] += v[j];
        if (v[j] > mx[k][j]) { mx[k][j] = v[j]; ix[k][j] = n; }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < MAXCH; ++k)
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = (lane + k * TPR) * V + j;
      if (lane + k * TPR < nch) { rs[slot * C + c] = sm[k][j]; rm[slot * C + c] = mx[k][j]; ri[slot * C + c] = ix[k][j]; }
    }
  __syncthreads();
  // level 1: G2 groups per channel, group q folds slots q, q + G2, ... into slot q (its own rows)
  const int G2 = min(RPB, max(1, NT / C));
  if (threadIdx.x < G2 * C) {
    const int c = threadIdx.x % C, q0 = threadIdx.x / C;
    float s = 0.f, m = -INFINITY;
    int mi = 0x7fffffff;
    for (int q = q0; q < RPB; q += G2) {
      s += rs[q * C + c];
      const float v = rm[q * C + c];
      const int i = ri[q * C + c];
      if (v > m || (v == m && i < mi)) { m = v; mi = i; }
    }
    rs[q0 * C + c] = s; rm[q0 * C + c] = m; ri[q0 * C + c] = mi;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NT) {
    float s = 0.f, m = -INFINITY;
    int mi = 0x7fffffff;
    for (int q = 0; q < G2; ++q) {
      s += rs[q * C + c];
      const float v = rm[q * C + c];
      const int i = ri[q * C + c];
      if (v > m || (v == m && i < mi)) { m = v; mi = i; }
    }
    const long o = ((long)gb * nc + ci) * C + c;
    psum[o] = s; pmax[o] = m; pidx[o] = mi;
  }
  __syncthreads();
}

// 16 channels x 32 chunk slices of one (g, b) -> pooled / argmax
__device__ void pool_fin(const float* psum, const float* pmax, const int* pidx, float* pooled, int* argmax, int cb,
                         int gb, int B, int N, int C, int nc, float* sh) {
  float* rs = sh;
  float* rm = sh + PF_SL * PF_CH;
  int* ri = reinterpret_cast<int*>(sh + 2 * PF_SL * PF_CH);
  const int cl = threadIdx.x % PF_CH, zl = threadIdx.x / PF_CH, c = cb * PF_CH + cl;
  float s = 0.f, m = -INFINITY;
  int mi = 0x7fffffff;
  if (c < C) {
#pragma unroll 4
    for (int k = zl; k < nc; k += PF_SL) {
      const long o = ((long)gb * nc + k) * C + c;
      s += psum[o];
      const float v = pmax[o];
      const int i = pidx[o];
      if (v > m || (v == m && i < mi)) { m = v; mi = i; }
    }
  }
  rs[zl * PF_CH + cl] = s; rm[zl * PF_CH + cl] = m; ri[zl * PF_CH + cl] = mi;
  __syncthreads();
  if (zl < 4) {                          // 32 slices -> 4 -> 1
    for (int q = zl + 4; q < PF_SL; q += 4) {
      s += rs[q * PF_CH + cl];
      const float v = rm[q * PF_CH + cl];
      const int i = ri[q * PF_CH + cl];
      if (v > m || (v == m && i < mi)) { m = v; mi = i; }
    }
  }
  __syncthreads();
  if (zl < 4) { rs[zl * PF_CH + cl] = s; rm[zl * PF_CH + cl] = m; ri[zl * PF_CH + cl] = mi; }
  __syncthreads();
  if (zl == 0 && c < C) {
    for (int q = 1; q < 4; ++q) {
      s += rs[q * PF_CH + cl];
      const float v = rm[q * PF_CH + cl];
      const int i = ri[q * PF_CH + cl];
      if (v > m || (v == m && i < mi)) { m = v; mi = i; }
    }
    const int g = gb / B, b = gb % B;
    pooled[(long)b * 4 * C + g * C + c] = s / N;
    pooled[(long)b * 4 * C + 2 * C + g * C + c] = m;
    argmax[(long)b * 2 * C + g * C + c] = mi;
  }
  __syncthreads();
}

// y[m][n] = act(x[m] . w[n] + b[n]): x (M x K) staged in LDS once per block, one wave per output
// feature over the whole grid, four independent float4 weight loads in flight per lane
__device__ void gemv(const float* x, const float* __restrict__ w, const float* __restrict__ b, float* y, int M,
                     int K, int Nout, int act, float* sh) {
  const int K4 = K >> 2;
  for (int e = threadIdx.x; e < M * K4; e += NT)
    reinterpret_cast<float4*>(sh)[e] = reinterpret_cast<const float4*>(x)[e];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int n = blockIdx.x * NW + wave; n < Nout; n += gridDim.x * NW) {
    const float4* wr = reinterpret_cast<const float4*>(w + (long)n * K);
    float acc[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) acc[m] = 0.f;
    int k4 = lane;
    for (; k4 + 192 < K4; k4 += 256) {
      float4 wv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) wv[u] = wr[k4 + 64 * u];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int m = 0; m < MB; ++m)
          if (m < M) {
            const float4 xv = reinterpret_cast<const float4*>(sh)[m * K4 + k4 + 64 * u];
            acc[m] += wv[u].x * xv.x + wv[u].y * xv.y + wv[u].z * xv.z + wv[u].w * xv.w;
          }
    }
    for (; k4 < K4; k4 += 64) {
      const float4 wv = wr[k4];
#pragma unroll
      for (int m = 0; m < MB; ++m)
        if (m < M) {
          const float4 xv = reinterpret_cast<const float4*>(sh)[m * K4 + k4];
          acc[m] += wv.x * xv.x + wv.y * xv.y + wv.z * xv.z + wv.w * xv.w;
        }
    }
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      if (m >= M) break;
      const float s = wave_sum(acc[m]);
      if (lane == 0) y[(long)m * Nout + n] = act_fwd(s + b[n], act);
    }
  }
  __syncthreads();
}

struct FwdArgs {
  const void* x;
  const float *w1, *b1, *w2, *b2;
  float *pooled, *y1, *cw, *psum, *pmax;
  int *argmax, *pidx;
  int B, N, C, nc, chunk;
};

template <typename T, int TPR>
__global__ __launch_bounds__(NT) void frm_channel_fwd_kernel(FwdArgs a) {
  extern __shared__ float sh[];
  unsigned* bar = g_frm_bar[0];
  const unsigned P = gridDim.x;
  const int GB = 2 * a.B;
  for (int it = blockIdx.x; it < a.nc * GB; it += P)
    pool_part<T, TPR>((const T*)a.x, a.psum, a.pmax, a.pidx, it / a.nc, it % a.nc, a.nc, a.N, a.C, a.chunk, sh);
  grid_sync(bar, P);
  const int ncb = (a.C + PF_CH - 1) / PF_CH;
  for (int it = blockIdx.x; it < ncb * GB; it += P)
    pool_fin(a.psum, a.pmax, a.pidx, a.pooled, a.argmax, it % ncb, it / ncb, a.B, a.N, a.C, a.nc, sh);
  grid_sync(bar, 2 * P);
  gemv(a.pooled, a.w1, a.b1, a.y1, a.B, 4 * a.C, 4 * a.C, ACT_RELU, sh);
  grid_sync(bar, 3 * P);
  gemv(a.y1, a.w2, a.b2, a.cw, a.B, 4 * a.C, 2 * a.C, ACT_SIGMOID, sh);
  grid_exit(bar);
}

// ---------------------------------------------------------------- backward phases
// dz2[m][n] = (sum_s pcw[m][s][n]) * cw (1 - cw) and db2[n] = sum_m dz2[m][n] for 64 columns n;
// the waves split the slabs, LDS combines them in a fixed order
__device__ void dcw_sum(const float* pcw, int nslab, const float* cw, float* dz2, float* db2, int M, int C2, int nb,
                        float* sh) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, n = nb * 64 + lane;
  for (int m = 0; m < M; ++m) {
    float d = 0.f;
    if (n < C2)
      for (int s = wave; s < nslab; s += NW) d += pcw[((long)m * nslab + s) * C2 + n];
    sh[(wave * MB + m) * 64 + lane] = d;
  }
  __syncthreads();
  if (wave == 0 && n < C2) {
    float tb = 0.f;
    for (int m = 0; m < M; ++m) {
      float d = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) d += sh[(q * MB + m) * 64 + lane];
      const float c = cw[(long)m * C2 + n];
      const float dz = d * (c * (1.f - c));
      dz2[(long)m * C2 + n] = dz;
      tb += dz;
    }
    db2[n] = tb;
  }
  __syncthreads();
}

__device__ __forceinline__ float act_grad_out(float y, int act) {
  if (act == ACT_RELU) return y > 0.f ? 1.f : 0.f;
  return 1.f;
}

// one (64 k-columns, n-slice) item of the backward of y = act(x w^T + b): dz over the slice from
// nsl partial slabs of dy (times act' from the saved output), dw rows written, db over the slice
// (k-column block 0), dx partial of the slice: dxp[sl][m][k] = sum_{n in slice} dz[m][n] w[n][k]
__device__ void wpass(const float* dyp, int nsl, long ss, const float* y, int act, const float* x,
                      const float* __restrict__ w, float* dxp, float* dw, float* db, int M, int K, int Nout, int kc,
                      int sl, float* sh) {
  float* dzs = sh;                        // [MB][SLMAX]
  float* red = sh + MB * SLMAX;           // [NW][MB][64]
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int per = (Nout + NSL - 1) / NSL;
  const int n0 = sl * per, rows = max(0, min(Nout, n0 + per) - n0);
  for (int e = threadIdx.x; e < M * rows; e += NT) {
    const int m = e / rows, n = n0 + e % rows;
    float d = 0.f;
    for (int q = 0; q < nsl; ++q) d += dyp[q * ss + (long)m * Nout + n];
    dzs[m * SLMAX + (n - n0)] = y ? d * act_grad_out(y[(long)m * Nout + n], act) : d;
  }
  __syncthreads();
  if (kc == 0 && db)
    for (int r = threadIdx.x; r < rows; r += NT) {
      float sb = 0.f;
      for (int m = 0; m < M; ++m) sb += dzs[m * SLMAX + r];
      db[n0 + r] = sb;
    }
  const int k = kc * 64 + tx;
  float acc[MB], xk[MB];
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    acc[m] = 0.f;
    xk[m] = (m < M && k < K) ? x[(long)m * K + k] : 0.f;
  }
  if (k < K) {
#pragma unroll 4
    for (int r = ty; r < rows; r += NW) {
      const int n = n0 + r;
      const float wv = w[(long)n * K + k];
      float g = 0.f;
#pragma unroll
      for (int m = 0; m < MB; ++m)
        if (m < M) {
          const float dz = dzs[m * SLMAX + r];
          acc[m] += dz * wv;
          g += dz * xk[m];
        }
      dw[(long)n * K + k] = g;
    }
  }
#pragma unroll
  for (int m = 0; m < MB; ++m) red[(ty * MB + m) * 64 + tx] = acc[m];
  __syncthreads();
  if (ty == 0 && k < K)
    for (int m = 0; m < M; ++m) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) t += red[(q * MB + m) * 64 + tx];
      dxp[((long)sl * M + m) * K + k] = t;
    }
  __syncthreads();
}

// dx[g][b][n][c] += dpooled_avg / N + (n == argmax) * dpooled_max over one chunk of tokens; the
// (g, b)'s 2C dpooled values summed from the NSL slice partials once per item
template <typename T, int TPR>
__device__ void pool_bwd(const float* dpp, const int* argmax, T* dx, int gb, int rc, int nrc, int B, int N, int C,
                         float* sh) {
  constexpr int V = VecT<T>::N, RPB = NT / TPR;
  const int g = gb / B, b = gb % B;
  const long ss = (long)B * 4 * C;
  for (int e = threadIdx.x; e < 2 * C; e += NT) {
    const int k = e < C ? g * C + e : 2 * C + g * C + (e - C);
    float t = 0.f;
    for (int q = 0; q < NSL; ++q) t += dpp[q * ss + (long)b * 4 * C + k];
    sh[e] = e < C ? t / N : t;
  }
  __syncthreads();
  const int lane = threadIdx.x % TPR, slot = threadIdx.x / TPR, nch = C / V;
  float dav[MAXCH][V], dmx[MAXCH][V];
  int am[MAXCH][V];
#pragma unroll
  for (int k = 0; k < MAXCH; ++k)
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = (lane + k * TPR) * V + j;
      const bool ok = lane + k * TPR < nch;
      dav[k][j] = ok ? sh[c] : 0.f;
      dmx[k][j] = ok ? sh[C + c] : 0.f;
      am[k][j] = ok ? argmax[(long)b * 2 * C + g * C + c] : -1;
    }
  T* base = dx + (long)gb * N * C;
  for (int n = rc * RPB + slot; n < N; n += nrc * RPB) {
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
  __syncthreads();
}

struct BwdArgs {
  const float *pcw, *cw, *y1, *pooled, *w1, *w2;
  const int* argmax;
  float *dw1, *db1, *dw2, *db2, *dz2, *dy1p, *dpp;
  void* dx;
  int nslab, B, N, C, nrc;
};

template <typename T, int TPR>
__global__ __launch_bounds__(NT) void frm_channel_bwd_kernel(BwdArgs a) {
  extern __shared__ float sh[];
  unsigned* bar = g_frm_bar[1];
  const unsigned P = gridDim.x;
  const int C = a.C, M = a.B;
  const int ncb2 = (2 * C + 63) / 64;
  for (int it = blockIdx.x; it < ncb2; it += P) dcw_sum(a.pcw, a.nslab, a.cw, a.dz2, a.db2, M, 2 * C, it, sh);
  grid_sync(bar, P);
  const int nkc = (4 * C + 63) / 64;     // both weight passes have K = 4C columns
  for (int it = blockIdx.x; it < nkc * NSL; it += P)
    wpass(a.dz2, 1, 0, nullptr, ACT_NONE, a.y1, a.w2, a.dy1p, a.dw2, nullptr, M, 4 * C, 2 * C, it % nkc, it / nkc, sh);
  grid_sync(bar, 2 * P);
  for (int it = blockIdx.x; it < nkc * NSL; it += P)
    wpass(a.dy1p, NSL, (long)M * 4 * C, a.y1, ACT_RELU, a.pooled, a.w1, a.dpp, a.dw1, a.db1, M, 4 * C, 4 * C, it % nkc,
          it / nkc, sh);
  grid_sync(bar, 3 * P);
  for (int it = blockIdx.x; it < 2 * a.B * a.nrc; it += P)
    pool_bwd<T, TPR>(a.dpp, a.argmax, (T*)a.dx, it / a.nrc, it % a.nrc, a.nrc, a.B, a.N, C, sh);
  grid_exit(bar);
}

#define FRMC_TPR_DISPATCH(tpr, TPR, ...)                       \
  do {                                                         \
    switch (tpr) {                                             \
      case 4: { constexpr int TPR = 4; __VA_ARGS__; break; }   \
      case 8: { constexpr int TPR = 8; __VA_ARGS__; break; }   \
      case 16: { constexpr int TPR = 16; __VA_ARGS__; break; } \
      case 32: { constexpr int TPR = 32; __VA_ARGS__; break; } \
      default: { constexpr int TPR = 64; __VA_ARGS__; break; } \
    }                                                          \
  } while (0)

// one block per CU (queried once; a grid the chip can hold resident whatever else is running
// on a few CUs: one 512-thread block per CU leaves room for several more)
int channel_grid() {
  static const int p = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                               hipSuccess)
      n = 0;
    return n > 0 ? n : 256;
  }();
  return p;
}

bool shape_ok(int B, int N, int C, int V) {
  return B > 0 && B <= MB && N > 0 && C > 0 && C % V == 0 && C / V <= MAXCH * 64 && C % 16 == 0 &&
         (4 * C + NSL - 1) / NSL <= SLMAX && (size_t)B * 4 * C * sizeof(float) <= 64 * 1024;
}

}  // namespace

extern "C" {

size_t cmx_frm_channel_fwd_workspace(int B, int N, int C) {
  const int nc = pool_chunks(N, 2 * B);
  return (size_t)2 * B * nc * C * 3 * sizeof(float);
}

int cmx_frm_channel_fwd(const void* x, const float* w1, const float* b1, const float* w2, const float* b2,
                        float* pooled, int* argmax, float* y1, float* cw, float* workspace, int B, int N, int C,
                        int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(shape_ok(B, N, C, V), CMX_ERR_SHAPE, "frm_channel_fwd: B=%d N=%d C=%d (B <= 8, C %% 16 == 0)", B, N, C);
  CMX_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)w1 & 15) == 0 && ((uintptr_t)w2 & 15) == 0 &&
              ((uintptr_t)pooled & 15) == 0 && ((uintptr_t)y1 & 15) == 0, CMX_ERR_ARG,
              "frm_channel_fwd: x, w1, w2, pooled, y1 need 16-B alignment");
  FwdArgs a{};
  a.x = x; a.w1 = w1; a.b1 = b1; a.w2 = w2; a.b2 = b2; a.pooled = pooled; a.y1 = y1; a.cw = cw; a.argmax = argmax;
  a.B = B; a.N = N; a.C = C;
  a.nc = pool_chunks(N, 2 * B);
  a.chunk = (N + a.nc - 1) / a.nc;
  a.psum = workspace;
  a.pmax = workspace + (size_t)2 * B * a.nc * C;
  a.pidx = reinterpret_cast<int*>(a.pmax + (size_t)2 * B * a.nc * C);
  const int tpr = row_lanes(C, V);
  const size_t lds_pool = (size_t)3 * (NT / tpr) * C * sizeof(float);
  const size_t lds_gemv = (size_t)B * 4 * C * sizeof(float);
  const size_t lds = std::max(std::max(lds_pool, lds_gemv), (size_t)3 * NT * sizeof(float));
  const int P = channel_grid();
  CMX_DISPATCH(dtype, T, {
    FRMC_TPR_DISPATCH(tpr, TPR, hipLaunchKernelGGL((frm_channel_fwd_kernel<T, TPR>), dim3(P), dim3(NT), lds, s, a));
  });
  return cmx_check_launch("frm_channel_fwd");
}

size_t cmx_frm_channel_bwd_workspace(int B, int C) {
  return ((size_t)B * 2 * C + (size_t)2 * NSL * B * 4 * C) * sizeof(float);
}

int cmx_frm_channel_bwd(const float* dcw_part, int nslab, const float* cw, const float* y1, const float* pooled,
                        const int* argmax, const float* w1, const float* w2, float* dw1, float* db1, float* dw2,
                        float* db2, void* dx, float* workspace, int B, int N, int C, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(shape_ok(B, N, C, V) && nslab > 0, CMX_ERR_SHAPE, "frm_channel_bwd: B=%d N=%d C=%d nslab=%d", B, N, C,
              nslab);
  CMX_REQUIRE(((uintptr_t)dx & 15) == 0, CMX_ERR_ARG, "frm_channel_bwd: dx needs 16-B alignment");
  BwdArgs a{};
  a.pcw = dcw_part; a.cw = cw; a.y1 = y1; a.pooled = pooled; a.w1 = w1; a.w2 = w2; a.argmax = argmax;
  a.dw1 = dw1; a.db1 = db1; a.dw2 = dw2; a.db2 = db2; a.dx = dx;
  a.dz2 = workspace;
  a.dy1p = workspace + (size_t)B * 2 * C;
  a.dpp = a.dy1p + (size_t)NSL * B * 4 * C;
  a.nslab = nslab; a.B = B; a.N = N; a.C = C;
  const int tpr = row_lanes(C, V);
  const int P = channel_grid();
  long nrc = (2L * P + 2 * B - 1) / (2 * B);       // ~2 token chunks per block over the (g, b) images
  const long maxrc = (N + NT / tpr - 1) / (NT / tpr);
  a.nrc = (int)std::max(1L, std::min(nrc, maxrc));
  const size_t lds = std::max((size_t)(MB * SLMAX + NW * MB * 64) * sizeof(float), (size_t)2 * C * sizeof(float));
  CMX_DISPATCH(dtype, T, {
    FRMC_TPR_DISPATCH(tpr, TPR, hipLaunchKernelGGL((frm_channel_bwd_kernel<T, TPR>), dim3(P), dim3(NT), lds, s, a));
  });
  return cmx_check_launch("frm_channel_bwd");
}

int cmx_frm_barrier_timeouts(void) {
  unsigned h[2][4] = {};
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_frm_bar), sizeof(h), 0, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (int)(h[0][2] + h[1][2]);
}

}  // extern "C"
