// Spatial-reduction attention core: O = softmax(Q K^T * d^-1/2) V, forward and backward.
//
// Replaces the eager core of Attention.forward (dual_segformer.py:130-134):
//   attn = (q @ k.transpose(-2, -1)) * scale; attn = attn.softmax(-1); x = attn @ v
// which materialises a (B, h, N, Nk) fp32 score tensor.  Here scores never leave
// registers (flash-style online softmax over 32-key tiles).
//
// Layout (token-major, no permutes): q (Bt, N, heads*D) with row stride qs; k and v are the
// two halves of the kv projection output (Bt, Nk, 2*heads*D) (kv split order K|V, head-major
// inside each half, dual_segformer.py:125-128), row stride kvs; o like q.  Bt = G*B (both
// modality streams in one launch).  lse (Bt, heads, N) fp32 is saved for the backward.
//
// Work decomposition (gfx950, wave64, 32x32 MFMA tiles, cmx_mfma.h):
//  fwd   : workgroup = 4 waves = 128 queries of one (b, head); each wave owns 32 queries.
//          S^T = K Q^T keeps the query on the MFMA lane, so row max / row sum are per lane
//          (+1 cross-half shuffle); O^T = V^T P^T reuses the P^T accumulator as the B
//          operand with no data movement.  K (row-major) and V (transposed for bf16) are
//          staged per 32-key tile in LDS; Q stays in registers.
//  bwd-A : same decomposition, dQ^T = K^T dS^T accumulated per lane; also emits
//          Dq = rowsum(dO * O).
//  bwd-B : "key on the lane": workgroup = 128 keys x one query chunk; each wave keeps
//          dK^T, dV^T of its 32 keys in registers while sweeping 32-query tiles; partial
//          sums per query chunk go to an fp32 slab, reduced by a third kernel (no atomics,
//          bit-reproducible).
// MFMA FLOPs per (b, head): fwd 4*N*Nk*D, bwd 8*N*Nk*D (+ S recompute 2*N*Nk*D).
#include "cmx_mfma.h"

namespace {

constexpr int BQ = 128;  // queries per forward / dQ workgroup
constexpr int BK = 128;  // keys per dK/dV workgroup
constexpr int KT = 32;   // keys (or queries) per LDS tile

template <typename T, int D> struct Lds {
  static constexpr bool BF = sizeof(T) == 2;
  static constexpr int KS = BF ? D + 8 : D + 1;  // row-major [row][d] stride (elements)
  static constexpr int TS = BF ? KT + 4 : 1;     // transposed [d][row] stride (bf16 only)
};

// Stage rows [r0, r0 + KT) (rows >= nrows are zero) of a (rows x D) matrix with row
// stride `stride` into LDS: row-major image (stride KS) and/or transposed image (stride TS).
template <typename T, int D, bool ROW, bool TRANS>
__device__ __forceinline__ void stage_tile(const T* __restrict__ g, long stride, int r0, int nrows,
                                           T* rowimg, T* trimg) {
  constexpr int V = VecT<T>::N;
  constexpr int CPR = D / V;
  constexpr int KS = Lds<T, D>::KS, TS = Lds<T, D>::TS;
  for (int idx = threadIdx.x; idx < KT * CPR; idx += 256) {
    const int r = idx / CPR, ch = idx % CPR;
    float v[V];
    if (r0 + r < nrows) {
      load_vec<T>(g + (long)(r0 + r) * stride + ch * V, v);
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] = 0.f;
    }
    if constexpr (ROW) {
      if constexpr (Lds<T, D>::BF) {
        store_vec<T>(rowimg + r * KS + ch * V, v);
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) rowimg[r * KS + ch * V + j] = v[j];
      }
    }
    if constexpr (TRANS) {
#pragma unroll
      for (int j = 0; j < V; ++j) trimg[(ch * V + j) * TS + r] = from_f32<T>(v[j]);
    }
  }
}

// A-operand fragment for a k-permuted product whose k index is a 32-row LDS tile and
// whose output rows are d = 32*t + r: element j of lane half h is tile row
// accrow(E*s + j, h).  bf16 reads the transposed image, fp32 the row-major one.
template <typename T, int D>
__device__ __forceinline__ typename MF<T>::frag perm_frag(const T* rowimg, const T* trimg, int t, int s,
                                                          int r, int h) {
  if constexpr (Lds<T, D>::BF) {
    constexpr int TS = Lds<T, D>::TS;
    const T* p = trimg + (32 * t + r) * TS + 16 * s + 4 * h;
    return MF<T>::load2x4(p, p + 8);
  } else {
    constexpr int KS = Lds<T, D>::KS;
    return rowimg[accrow(s, h) * KS + 32 * t + r];
  }
}

template <typename T>
__device__ __forceinline__ void store4(T* p, const float* v) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    uint32_t a = pack2<T>(v[0], v[1]);
    uint32_t b = pack2<T>(v[2], v[3]);
    *reinterpret_cast<uint2*>(p) = make_uint2(a, b);
  }
}

// store the 32-row (d) x 32-col (lane) accumulator tile t of row `row_ptr` (d contiguous)
template <typename T>
__device__ __forceinline__ void store_acc_row(T* row_ptr, const f32x16& acc, int t, int h, float mul) {
#pragma unroll
  for (int k4 = 0; k4 < 4; ++k4) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = acc[4 * k4 + u] * mul;
    store4<T>(row_ptr + 32 * t + 8 * k4 + 4 * h, v);
  }
}

template <typename T, int E>
__device__ __forceinline__ float dot_e(const T* a, const T* b) {
  float s = 0.f;
  if constexpr (E == 1) {
    s = to_f32(a[0]) * to_f32(b[0]);
  } else {
    float x[8], y[8];
    load_vec<T>(a, x);
    load_vec<T>(b, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j] * y[j];
  }
  return s;
}

// ------------------------------------------------------------------------ forward
template <typename T, int D>
__global__ __launch_bounds__(256) void sra_fwd_kernel(const T* __restrict__ q, const T* __restrict__ k,
                                                      const T* __restrict__ v, T* __restrict__ o,
                                                      float* __restrict__ lse, int N, int Nk, int heads,
                                                      long qs, long kvs, long os, float scale_log2) {
  using M = MF<T>;
  constexpr int KI = M::KI, E = M::E, NQF = D / KI, NT = D / 32;
  constexpr int KS = Lds<T, D>::KS, TS = Lds<T, D>::TS;
  constexpr bool BF = Lds<T, D>::BF;
  __shared__ __attribute__((aligned(16))) T Ks[KT * KS];
  __shared__ __attribute__((aligned(16))) T Vs[BF ? D * TS : KT * KS];

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int b = blockIdx.z, head = blockIdx.y;
  const int qi = blockIdx.x * BQ + wave * 32 + r;
  const T* qb = q + (long)b * N * qs + head * D;
  const T* kb = k + (long)b * Nk * kvs + head * D;
  const T* vb = v + (long)b * Nk * kvs + head * D;

  typename M::frag qf[NQF];
#pragma unroll
  for (int s = 0; s < NQF; ++s) qf[s] = qi < N ? M::load(qb + (long)qi * qs + KI * s + E * h) : zfrag<T>();

  f32x16 acc_o[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc_o[t] = zero16();
  float m = -INFINITY, l = 0.f;

  for (int t0 = 0; t0 < Nk; t0 += KT) {
    __syncthreads();
    stage_tile<T, D, true, false>(kb, kvs, t0, Nk, Ks, nullptr);
    if constexpr (BF) stage_tile<T, D, false, true>(vb, kvs, t0, Nk, nullptr, Vs);
    else stage_tile<T, D, true, false>(vb, kvs, t0, Nk, Vs, nullptr);
    __syncthreads();

    f32x16 sacc = zero16();
#pragma unroll
    for (int s = 0; s < NQF; ++s) sacc = M::mma(M::load(&Ks[r * KS + KI * s + E * h]), qf[s], sacc);

    float mt = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float x = sacc[i] * scale_log2;
      if (t0 + accrow(i, h) >= Nk) x = -INFINITY;
      sacc[i] = x;
      mt = fmaxf(mt, x);
    }
    mt = fmaxf(mt, xor_lane<32>(mt));
    const float mn = fmaxf(m, mt);
    const float alpha = exp2f(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = exp2f(sacc[i] - mn);
      sacc[i] = p;
      rs += p;
    }
    rs += xor_lane<32>(rs);
    l = l * alpha + rs;
    m = mn;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc_o[t][i] *= alpha;

#pragma unroll
    for (int s = 0; s < KT / KI; ++s) {
      const typename M::frag pf = M::from_acc(sacc, s);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc_o[t] = M::mma(perm_frag<T, D>(Vs, Vs, t, s, r, h), pf, acc_o[t]);
    }
  }
  if (qi >= N) return;
  const float inv = 1.f / l;
  T* ob = o + ((long)b * N + qi) * os + head * D;
#pragma unroll
  for (int t = 0; t < NT; ++t) store_acc_row<T>(ob, acc_o[t], t, h, inv);
  if (h == 0 && lse) lse[((long)b * heads + head) * N + qi] = (m + log2f(l)) * 0.69314718055994531f;
}

// ------------------------------------------------------------------------ backward A: dQ, Dq
template <typename T, int D>
__global__ __launch_bounds__(256) void sra_bwd_dq_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, const T* __restrict__ o,
    const T* __restrict__ dout, const float* __restrict__ lse, float* __restrict__ Dws, T* __restrict__ dq,
    int N, int Nk, int heads, long qs, long kvs, long os, long dos, long dqs, float scale_log2,
    float scale) {
  using M = MF<T>;
  constexpr int KI = M::KI, E = M::E, NQF = D / KI, NT = D / 32;
  constexpr int KS = Lds<T, D>::KS, TS = Lds<T, D>::TS;
  constexpr bool BF = Lds<T, D>::BF;
  __shared__ __attribute__((aligned(16))) T Ks[KT * KS];
  __shared__ __attribute__((aligned(16))) T Vs[KT * KS];
  __shared__ __attribute__((aligned(16))) T Kt[BF ? D * TS : 1];

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int b = blockIdx.z, head = blockIdx.y;
  const int qi = blockIdx.x * BQ + wave * 32 + r;
  const bool live = qi < N;
  const T* kb = k + (long)b * Nk * kvs + head * D;
  const T* vb = v + (long)b * Nk * kvs + head * D;
  const T* qrow = q + ((long)b * N + qi) * qs + head * D;
  const T* orow = o + ((long)b * N + qi) * os + head * D;
  const T* drow = dout + ((long)b * N + qi) * dos + head * D;

  typename M::frag qf[NQF], df[NQF];
  float dot = 0.f;
#pragma unroll
  for (int s = 0; s < NQF; ++s) {
    if (live) {
      qf[s] = M::load(qrow + KI * s + E * h);
      df[s] = M::load(drow + KI * s + E * h);
      dot += dot_e<T, E>(drow + KI * s + E * h, orow + KI * s + E * h);
    } else {
      qf[s] = zfrag<T>();
      df[s] = zfrag<T>();
    }
  }
  dot += xor_lane<32>(dot);
  const long sidx = ((long)b * heads + head) * N + qi;
  const float Dq = dot;
  const float lse2 = live ? lse[sidx] * 1.4426950408889634f : 0.f;
  if (live && h == 0) Dws[sidx] = Dq;

  f32x16 acc_q[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc_q[t] = zero16();

  for (int t0 = 0; t0 < Nk; t0 += KT) {
    __syncthreads();
    if constexpr (BF) stage_tile<T, D, true, true>(kb, kvs, t0, Nk, Ks, Kt);
    else stage_tile<T, D, true, false>(kb, kvs, t0, Nk, Ks, nullptr);
    stage_tile<T, D, true, false>(vb, kvs, t0, Nk, Vs, nullptr);
    __syncthreads();

    f32x16 sacc = zero16(), dpacc = zero16();
#pragma unroll
    for (int s = 0; s < NQF; ++s) {
      sacc = M::mma(M::load(&Ks[r * KS + KI * s + E * h]), qf[s], sacc);
      dpacc = M::mma(M::load(&Vs[r * KS + KI * s + E * h]), df[s], dpacc);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float p = exp2f(sacc[i] * scale_log2 - lse2);
      if (t0 + accrow(i, h) >= Nk) p = 0.f;
      sacc[i] = p * (dpacc[i] - Dq);  // dS^T
    }
#pragma unroll
    for (int s = 0; s < KT / KI; ++s) {
      const typename M::frag sf = M::from_acc(sacc, s);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc_q[t] = M::mma(perm_frag<T, D>(Ks, Kt, t, s, r, h), sf, acc_q[t]);
    }
  }
  if (!live) return;
  T* out = dq + ((long)b * N + qi) * dqs + head * D;
#pragma unroll
  for (int t = 0; t < NT; ++t) store_acc_row<T>(out, acc_q[t], t, h, scale);
}

// ------------------------------------------------------------------------ backward B: dK, dV
template <typename T, int D>
__global__ __launch_bounds__(256) void sra_bwd_dkv_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, const T* __restrict__ dout,
    const float* __restrict__ lse, const float* __restrict__ Dws, float* __restrict__ ws_dk,
    float* __restrict__ ws_dv, int Bt, int N, int Nk, int heads, long qs, long kvs, long dos, int QC,
    int nchunk, float scale_log2, float scale) {
  using M = MF<T>;
  constexpr int KI = M::KI, E = M::E, NQF = D / KI, NT = D / 32;
  constexpr int KS = Lds<T, D>::KS, TS = Lds<T, D>::TS;
  constexpr bool BF = Lds<T, D>::BF;
  __shared__ __attribute__((aligned(16))) T Qs[KT * KS];
  __shared__ __attribute__((aligned(16))) T Ds[KT * KS];
  __shared__ __attribute__((aligned(16))) T Qt[BF ? D * TS : 1];
  __shared__ __attribute__((aligned(16))) T Dt[BF ? D * TS : 1];
  __shared__ float lse_s[KT], D_s[KT];

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int head = blockIdx.y;
  const int b = blockIdx.z / nchunk, c = blockIdx.z % nchunk;
  const int kw0 = blockIdx.x * BK + wave * 32;
  const int key = kw0 + r;
  const bool wave_live = kw0 < Nk;
  const T* qb = q + (long)b * N * qs + head * D;
  const T* db = dout + (long)b * N * dos + head * D;
  const long sbase = ((long)b * heads + head) * N;

  typename M::frag kf[NQF], vf[NQF];
#pragma unroll
  for (int s = 0; s < NQF; ++s) {
    if (key < Nk) {
      kf[s] = M::load(k + ((long)b * Nk + key) * kvs + head * D + KI * s + E * h);
      vf[s] = M::load(v + ((long)b * Nk + key) * kvs + head * D + KI * s + E * h);
    } else {
      kf[s] = zfrag<T>();
      vf[s] = zfrag<T>();
    }
  }
  f32x16 acc_k[NT], acc_v[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc_k[t] = acc_v[t] = zero16();

  const int qbeg = c * QC;
  const int qend = min(N, qbeg + QC);
  for (int qt0 = qbeg; qt0 < qend; qt0 += KT) {
    __syncthreads();
    stage_tile<T, D, true, BF>(qb, qs, qt0, qend, Qs, Qt);
    stage_tile<T, D, true, BF>(db, dos, qt0, qend, Ds, Dt);
    if (threadIdx.x < KT) {
      const int qq = qt0 + threadIdx.x;
      lse_s[threadIdx.x] = qq < qend ? lse[sbase + qq] * 1.4426950408889634f : INFINITY;
      D_s[threadIdx.x] = qq < qend ? Dws[sbase + qq] : 0.f;
    }
    __syncthreads();
    if (!wave_live) continue;

    f32x16 sacc = zero16(), dpacc = zero16();
#pragma unroll
    for (int s = 0; s < NQF; ++s) {
      sacc = M::mma(M::load(&Qs[r * KS + KI * s + E * h]), kf[s], sacc);
      dpacc = M::mma(M::load(&Ds[r * KS + KI * s + E * h]), vf[s], dpacc);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qq = accrow(i, h);
      const float p = exp2f(sacc[i] * scale_log2 - lse_s[qq]);
      sacc[i] = p;
      dpacc[i] = p * (dpacc[i] - D_s[qq]);
    }
#pragma unroll
    for (int s = 0; s < KT / KI; ++s) {
      const typename M::frag pf = M::from_acc(sacc, s);
      const typename M::frag sf = M::from_acc(dpacc, s);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc_v[t] = M::mma(perm_frag<T, D>(Ds, Dt, t, s, r, h), pf, acc_v[t]);
        acc_k[t] = M::mma(perm_frag<T, D>(Qs, Qt, t, s, r, h), sf, acc_k[t]);
      }
    }
  }
  if (key >= Nk) return;
  const long o = ((((long)c * Bt + b) * heads + head) * Nk + key) * D;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int d = 32 * t + accrow(i, h);
      ws_dk[o + d] = acc_k[t][i] * scale;
      ws_dv[o + d] = acc_v[t][i];
    }
  }
}

// dk/dv[(b*Nk + key)*kvs + head*D + d] = sum_c slab[c][b][head][key][d].  A thread owns 4
// consecutive d (16-B loads) and every 4th chunk; the 4 chunk slices meet in LDS (a single
// thread walking up to 64 chunks serially was latency-bound).
template <typename T>
__global__ __launch_bounds__(256) void sra_dkv_reduce_kernel(const float* __restrict__ ws_dk,
                                                             const float* __restrict__ ws_dv, T* __restrict__ dk,
                                                             T* __restrict__ dv, int Bt, int Nk, int heads, int D,
                                                             long kvs, int nchunk) {
  __shared__ float4 red[3][64][2];
  const long total = (long)Bt * heads * Nk * D;
  const int gl = threadIdx.x & 63, zl = threadIdx.x >> 6;
  const long i = ((long)blockIdx.x * 64 + gl) * 4;
  float4 sk = make_float4(0.f, 0.f, 0.f, 0.f), sv = sk;
  if (i < total) {
    for (int c = zl; c < nchunk; c += 4) {
      const float4 a = *reinterpret_cast<const float4*>(ws_dk + (long)c * total + i);
      const float4 b = *reinterpret_cast<const float4*>(ws_dv + (long)c * total + i);
      sk.x += a.x; sk.y += a.y; sk.z += a.z; sk.w += a.w;
      sv.x += b.x; sv.y += b.y; sv.z += b.z; sv.w += b.w;
    }
  }
  if (zl > 0) { red[zl - 1][gl][0] = sk; red[zl - 1][gl][1] = sv; }
  __syncthreads();
  if (zl > 0 || i >= total) return;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const float4 a = red[q][gl][0], b = red[q][gl][1];
    sk.x += a.x; sk.y += a.y; sk.z += a.z; sk.w += a.w;
    sv.x += b.x; sv.y += b.y; sv.z += b.z; sv.w += b.w;
  }
  const int d = (int)(i % D);
  const int key = (int)((i / D) % Nk);
  const int head = (int)((i / ((long)D * Nk)) % heads);
  const int b = (int)(i / ((long)D * Nk * heads));
  const long oo = ((long)b * Nk + key) * kvs + head * D + d;
  const float kk[4] = {sk.x, sk.y, sk.z, sk.w}, vv[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    dk[oo + e] = from_f32<T>(kk[e]);
    dv[oo + e] = from_f32<T>(vv[e]);
  }
}

int bwd_nchunk(int Bt, int N, int Nk, int heads) {
  const int nkb = (Nk + BK - 1) / BK;
  const long base = (long)Bt * heads * nkb;
  long nc = (512 + base - 1) / base;
  const long maxc = (N + KT - 1) / KT;
  if (nc > maxc) nc = maxc;
  if (nc < 1) nc = 1;
  return (int)nc;
}
int bwd_qc(int N, int nchunk) {
  int qc = (N + nchunk - 1) / nchunk;
  return (qc + KT - 1) / KT * KT;
}

}  // namespace

// sra_fast.hip: LDS-resident K/V path for bf16 / fp16, D = 64
bool sra_fast_ok(int D, int Nk, int dtype, const void* const* ptrs, int nptr, const long* strides, int nstr);
bool sra_fast_fwd_ok(int D, int Nk, int dtype, const void* const* ptrs, int nptr, const long* strides, int nstr);
void sra_fwd_fast_launch(const void* q, const void* k, const void* v, void* o, float* lse, int Bt, int N, int Nk,
                         int heads, long qs, long kvs, long os, float sl2, int dtype, hipStream_t s);
void sra_dq_fast_launch(const void* q, const void* k, const void* v, const void* o, const void* dout,
                        const float* lse, float* Dws, void* dq, int Bt, int N, int Nk, int heads, long qs, long kvs,
                        long os, long dos, long dqs, float sl2, float scale, int dtype, hipStream_t s);
int sra_dkv_fast_chunks(int Bt, int N, int Nk, int heads);
void sra_dkv_fast_launch(const void* q, const void* k, const void* v, const void* dout, const float* lse,
                         const float* Dws, float* ws_dk, float* ws_dv, void* dk, void* dv, long dkvs, int Bt, int N,
                         int Nk, int heads, long qs,
                         long kvs, long dos, int nchunk, float sl2, float scale, int dtype, hipStream_t s);

bool sra_small_ok(int D, int N, int Nk, int dtype, const void* const* ptrs, int nptr, const long* strides, int nstr);
bool sra_small_fwd_ok(int D, int N, int Nk, int dtype, const void* const* ptrs, int nptr, const long* strides,
                      int nstr);
void sra_fwd_small_launch(const void* q, const void* k, const void* v, void* o, float* lse, int Bt, int N, int Nk,
                          int heads, long qs, long kvs, long os, float sl2, int dtype, hipStream_t s);
void sra_dq_small_launch(const void* q, const void* k, const void* v, const void* o, const void* dout,
                         const float* lse, float* Dws, void* dq, int Bt, int N, int Nk, int heads, long qs, long kvs,
                         long os, long dos, long dqs, float sl2, float scale, int dtype, hipStream_t s);
void sra_dkv_small_launch(const void* q, const void* k, const void* v, const void* dout, const float* lse,
                          const float* Dws, void* dk, void* dv, long dkvs, int Bt, int N, int Nk, int heads, long qs,
                          long kvs, long dos, float sl2, float scale, int dtype, hipStream_t s);

#define SRA_D_DISPATCH(D, ...)                                              \
  do {                                                                      \
    if ((D) == 64) { constexpr int DD = 64; __VA_ARGS__; }                  \
    else if ((D) == 32) { constexpr int DD = 32; __VA_ARGS__; }             \
    else { cmx_set_error("sra: head dim %d unsupported", (int)(D)); return CMX_ERR_SHAPE; } \
  } while (0)

extern "C" {

// q, k, v, o: see header; lse (Bt, heads, N) fp32 (may be NULL for inference).
int cmx_sra_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int Bt, int N,
                     int Nk, int heads, int D, long qs, long kvs, long os, float scale, int dtype,
                     hipStream_t s) {
  CMX_REQUIRE(Bt > 0 && N > 0 && Nk > 0 && heads > 0, CMX_ERR_SHAPE, "sra_fwd: bad shape");
  CMX_REQUIRE(qs % 8 == 0 && kvs % 8 == 0 && os % 8 == 0, CMX_ERR_SHAPE, "sra_fwd: strides %% 8");
  const float sl2 = scale * 1.4426950408889634f;
  {
    const void* ptrs[] = {q, k, v, o};
    const long strides[] = {qs, kvs, os};
    if (sra_small_fwd_ok(D, N, Nk, dtype, ptrs, 4, strides, 3)) {
      sra_fwd_small_launch(q, k, v, o, lse, Bt, N, Nk, heads, qs, kvs, os, sl2, dtype, s);
      return cmx_check_launch("sra_fwd");
    }
    if (sra_fast_fwd_ok(D, Nk, dtype, ptrs, 4, strides, 3)) {
      sra_fwd_fast_launch(q, k, v, o, lse, Bt, N, Nk, heads, qs, kvs, os, sl2, dtype, s);
      return cmx_check_launch("sra_fwd");
    }
  }
  const dim3 grid(cdiv(N, BQ), heads, Bt);
  SRA_D_DISPATCH(D, CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((sra_fwd_kernel<T, DD>), grid, dim3(256), 0, s, (const T*)q, (const T*)k,
                       (const T*)v, (T*)o, lse, N, Nk, heads, qs, kvs, os, sl2);
  }));
  return cmx_check_launch("sra_fwd");
}

size_t cmx_sra_attn_bwd_workspace(int Bt, int N, int Nk, int heads, int D) {
  int nc = bwd_nchunk(Bt, N, Nk, heads);
  const int ncf = sra_dkv_fast_chunks(Bt, N, Nk, heads);   // the bf16 fast path may take either
  if (ncf > nc) nc = ncf;
  const size_t slab = (size_t)nc * Bt * heads * Nk * D;
  return ((size_t)Bt * heads * N + 2 * slab) * sizeof(float);
}

int cmx_sra_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                     const float* lse, void* dq, void* dk, void* dv, float* workspace, int Bt, int N,
                     int Nk, int heads, int D, long qs, long kvs, long os, long dos, long dqs, long dkvs,
                     float scale, int dtype, hipStream_t s) {
  CMX_REQUIRE(Bt > 0 && N > 0 && Nk > 0 && heads > 0, CMX_ERR_SHAPE, "sra_bwd: bad shape");
  CMX_REQUIRE(qs % 8 == 0 && kvs % 8 == 0 && os % 8 == 0 && dos % 8 == 0 && dqs % 8 == 0 && dkvs % 8 == 0,
              CMX_ERR_SHAPE, "sra_bwd: strides %% 8");
  const float sl2 = scale * 1.4426950408889634f;
  const void* ptrs[] = {q, k, v, o, dout, dq};
  const long strides[] = {qs, kvs, os, dos, dqs};
  if (sra_small_ok(D, N, Nk, dtype, ptrs, 6, strides, 5) && ((uintptr_t)dk & 15) == 0 && ((uintptr_t)dv & 15) == 0 &&
      dkvs % 8 == 0) {
    // short sequences: keys split over waves (dQ), query tiles over waves (dK / dV), no slabs
    float* Dws = workspace;
    sra_dq_small_launch(q, k, v, o, dout, lse, Dws, dq, Bt, N, Nk, heads, qs, kvs, os, dos, dqs, sl2, scale, dtype, s);
    sra_dkv_small_launch(q, k, v, dout, lse, Dws, dk, dv, dkvs, Bt, N, Nk, heads, qs, kvs, dos, sl2, scale, dtype, s);
    return cmx_check_launch("sra_bwd");
  }
  // fast path for any Nk: dQ streams K / V in LDS-sized chunks, dK / dV splits keys over workgroups
  const bool fast = sra_fast_fwd_ok(D, Nk, dtype, ptrs, 6, strides, 5);
  const bool fast_dq = fast;
  const int nc = fast ? sra_dkv_fast_chunks(Bt, N, Nk, heads) : bwd_nchunk(Bt, N, Nk, heads);
  const int qc = bwd_qc(N, nc);
  float* Dws = workspace;
  float* ws_dk = Dws + (size_t)Bt * heads * N;
  float* ws_dv = ws_dk + (size_t)nc * Bt * heads * Nk * D;
  SRA_D_DISPATCH(D, CMX_DISPATCH(dtype, T, {
    if (fast_dq)
      sra_dq_fast_launch(q, k, v, o, dout, lse, Dws, dq, Bt, N, Nk, heads, qs, kvs, os, dos, dqs, sl2, scale, dtype, s);
    else
      hipLaunchKernelGGL((sra_bwd_dq_kernel<T, DD>), dim3(cdiv(N, BQ), heads, Bt), dim3(256), 0, s,
                         (const T*)q, (const T*)k, (const T*)v, (const T*)o, (const T*)dout, lse, Dws,
                         (T*)dq, N, Nk, heads, qs, kvs, os, dos, dqs, sl2, scale);
    if (fast)
      sra_dkv_fast_launch(q, k, v, dout, lse, Dws, ws_dk, ws_dv, dk, dv, dkvs, Bt, N, Nk, heads, qs, kvs, dos, nc, sl2,
                          scale, dtype, s);
    else
      hipLaunchKernelGGL((sra_bwd_dkv_kernel<T, DD>), dim3(cdiv(Nk, BK), heads, Bt * nc), dim3(256), 0, s,
                         (const T*)q, (const T*)k, (const T*)v, (const T*)dout, lse, Dws, ws_dk, ws_dv, Bt,
                         N, Nk, heads, qs, kvs, dos, qc, nc, sl2, scale);
    const long total = (long)Bt * heads * Nk * D;     // D % 4 == 0: 4-wide groups never straddle a row
    if (!(fast && nc == 1))                           // one chunk: the fast kernel wrote dK / dV
    hipLaunchKernelGGL((sra_dkv_reduce_kernel<T>), dim3(cdiv(total / 4, 64)), dim3(256), 0, s, ws_dk, ws_dv, (T*)dk,
                       (T*)dv, Bt, Nk, heads, D, dkvs, nc);
  }));
  return cmx_check_launch("sra_bwd");
}

}  // extern "C"
